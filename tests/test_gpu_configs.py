"""BASELINE.json configs[2] and configs[1] at their full per-snapshot size (needs a GPU).

configs[2]: 1e8 particles in 1e4 halos, float32, every halo on the packed k_step path.
configs[1]: 1e7 particles in 1e2 halos, float64, every halo (1e5 particles) on the
partitioned large-halo path (k_part_scatter / k_part_join / k_gather_recs).  Three
snapshots each, device-generated (synthetic_device.DevicePlummer), run through
OrbitEngine (the path track_orbits uses).

At full size the checks are size-independent properties (reference semantics,
track_orbits.py:199-227, 300-351):
  * offsets non-decreasing from 0 to the record count;
  * every apsis ID is in its halo's previous block, once, in previous-block order;
  * an apsis particle's new angle is 0 (calc_angles resets it, :346);
  * a second run on another kernel path gives identical outputs: configs[2] with
    every halo forced onto the large-halo path (tiny LDS items), configs[1] with the
    large halos on the per-halo global tables (k_big_frame / k_big_join,
    ``part_large = False``) instead of the partitions;
plus oracle parity on a halo sample (the oracle's per-halo path on the same arrays):
apsis IDs and per-halo offsets bit-exact, f16 apsis angles within one ulp with at most
ANGLE_MISMATCH_MAX of them off.
"""
import numpy as np
import pytest

from test_gpu_parity import mismatch_ok

pytestmark = pytest.mark.gpu


def _run(gen, steps, eng):
    from orbitanalysis_amd.utils import hubble_parameter
    cos = gen.cosmology
    H = hubble_parameter(cos['redshift'], cos['H0'], cos['Omega_m'], cos['Omega_L'])
    ex = np.arange(gen.n_halos)
    out = []
    for s in range(steps):
        snap = gen.snapshot(s)
        c = gen.catalogue(s)
        res = eng.step(snap, c[0], c[2], H, cos['redshift'], ex, s > 0)
        if s > 0:
            offs, ids, ang = eng.fetch(res, np.dtype(np.int64))
            out.append(dict(offs=offs, ids=ids, ang=ang, meta=eng.state_meta().clone()))
        out_snap = snap
    return out, out_snap, H


def _check_properties(gen, prev_snap, cur_snap, r):
    import torch
    offs, ids = r['offs'], r['ids']
    nh = gen.n_halos
    assert offs[0] == 0 and np.all(np.diff(offs) >= 0) and offs[-1] == len(ids)
    dev = prev_snap['ids'].device
    # apsis IDs inside their halo's previous block, in that block's order, once each
    po = np.append(prev_snap['region_offsets'], prev_snap['ids'].numel())
    halo_of = torch.repeat_interleave(torch.arange(nh, device=dev),
                                      torch.from_numpy(np.diff(po)).to(dev))
    pkey = halo_of * (1 << 40) + prev_snap['ids']
    srt, perm = torch.sort(pkey)
    ah = torch.repeat_interleave(torch.arange(nh, device=dev), torch.from_numpy(np.diff(offs)).to(dev))
    akey = ah * (1 << 40) + torch.from_numpy(ids).to(dev)
    k = torch.searchsorted(srt, akey).clamp_(max=srt.numel() - 1)
    assert bool((srt[k] == akey).all()), 'apsis ID not in its previous block'
    pos = perm[k]                                   # position in the previous snapshot
    same_halo = ah[1:] == ah[:-1]
    assert bool((pos[1:] > pos[:-1])[same_halo].all()), 'apsis IDs out of previous-block order'
    # their new angle (current snapshot's state word) is 0
    co = np.append(cur_snap['region_offsets'], cur_snap['ids'].numel())
    ch = torch.repeat_interleave(torch.arange(nh, device=dev), torch.from_numpy(np.diff(co)).to(dev))
    ckey = ch * (1 << 40) + cur_snap['ids']
    csrt, cperm = torch.sort(ckey)
    j = torch.searchsorted(csrt, akey).clamp_(max=csrt.numel() - 1)
    assert bool((csrt[j] == akey).all()), 'apsis particle missing from the current block'
    ang = (r['meta'][cperm[j]] & 0xFFFF)
    assert bool((ang == 0).all()), 'apsis angle not reset'


def _oracle_sample(gen, s, H, n_halos, got, mode='pericentric'):
    """The oracle's per-halo path on the first n_halos blocks of snapshot pair (s-1, s)."""
    from oracle import orbit_oracle as O
    prv, cur = gen_host(gen, s - 1, n_halos), gen_host(gen, s, n_halos)
    cp, cc = gen.catalogue(s - 1), gen.catalogue(s)
    ang = np.zeros(prv['n'], np.float16)          # snapshot s-1 = 0: angles start at 0
    want, want_ang, lens = [], [], []
    for j in range(n_halos):
        pb, cb = prv['off'], cur['off']
        rp, vp, _ = O.region_frame(prv, (pb[j], pb[j + 1]), cp[0][j], cp[2][j], H)
        rc, vc, _ = O.region_frame(cur, (cb[j], cb[j + 1]), cc[0][j], cc[2][j], H)
        d = O.compare_radial_velocities(cur['ids'][cb[j]:cb[j + 1]], prv['ids'][pb[j]:pb[j + 1]],
                                        vc, vp, rc, rp, mode)
        _, aang = O.calc_angles(cb[j + 1] - cb[j], ang[pb[j]:pb[j + 1]], d)
        want.append(d['apsis_ids'])
        want_ang.append(aang)
        lens.append(len(d['apsis_ids']))
    want = np.concatenate(want)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    assert np.array_equal(got['offs'][:n_halos + 1], offs), 'per-halo offsets'
    assert np.array_equal(got['ids'][:got['offs'][n_halos]], want)
    a = got['ang'][:got['offs'][n_halos]].astype(np.float64)
    b = np.concatenate(want_ang).astype(np.float64)
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    ulp = np.spacing(np.maximum(np.abs(a), np.abs(b)).astype(np.float16)).astype(np.float64)
    assert np.all(same | (np.abs(a - b) <= ulp)), 'apsis angle off by more than 1 f16 ulp'
    assert mismatch_ok(int((~same).sum()), a.size), (int((~same).sum()), a.size)
    return a.size


_HOST = {}


def gen_host(gen, s, n_halos):
    snap = _HOST[(id(gen), s)]
    off = np.append(snap['region_offsets'], snap['ids'].numel())
    end = int(off[n_halos])
    d = {k: snap[k][:end].cpu().numpy() for k in ('ids', 'coordinates', 'velocities')}
    d.update(masses=snap['masses'], box_size=snap['box_size'], redshift=snap['redshift'],
             n=end, off=off[:n_halos + 1])
    return d


@pytest.mark.parametrize('cfg', ['configs2', 'configs1'])
def test_baseline_config_full_size(cfg):
    import torch
    from orbitanalysis_amd.engine import OrbitEngine
    from orbitanalysis_amd.synthetic_device import DevicePlummer
    if cfg == 'configs2':
        kw = dict(n_halos=10000, n_particles=100_000_000, dtype='float32')
        sample = 200
    else:
        kw = dict(n_halos=100, n_particles=10_000_000, dtype='float64')
        sample = 5
    steps = 3
    gen = DevicePlummer(seed=3, **kw)
    snaps = []
    orig = gen.snapshot

    def keep(s):                                  # the host sample needs snapshots 0..2
        snap = orig(s)
        _HOST[(id(gen), s)] = snap
        snaps.append(snap)
        return snap
    gen.snapshot = keep
    eng = OrbitEngine()
    first = []
    orig1 = eng.prepare

    def prepare1(*a, **k):
        pr = orig1(*a, **k)
        if pr.compare:
            first.append((pr.n_small, pr.n_global, pr.part))
        return pr
    eng.prepare = prepare1
    packed, last, H = _run(gen, steps, eng)
    if cfg == 'configs2':                         # every halo packed into k_step items
        assert first and all(ng == 0 for _, ng, _ in first), first
    else:                                         # every halo partitioned
        assert first and all(ns == 0 and ng > 0 and part for ns, ng, part in first), first
    for s in range(1, steps):
        _check_properties(gen, _HOST[(id(gen), s - 1)], _HOST[(id(gen), s)], packed[s - 1])
    assert _oracle_sample(gen, 1, H, sample, packed[0]) > 0
    # the same snapshots through another kernel path
    gen2 = DevicePlummer(seed=3, **kw)
    if cfg == 'configs2':
        eng2 = OrbitEngine(lds_entries=64)        # every halo a large halo
    else:
        eng2 = OrbitEngine()                      # large halos on the global tables
        eng2.part_large = False
    seen = []
    orig2 = eng2.prepare

    def prepare2(*a, **k):
        pr = orig2(*a, **k)
        if pr.compare:
            seen.append((pr.n_small, pr.n_global, pr.part))
        return pr
    eng2.prepare = prepare2
    glob, _, _ = _run(gen2, steps, eng2)
    # the second run really took the other path (and the first one the partitions)
    assert seen and all(ns == 0 and ng > 0 for ns, ng, _ in seen), seen
    if cfg == 'configs1':
        assert not any(part for _, _, part in seen), seen
    for a, b in zip(packed, glob):
        for k in ('offs', 'ids', 'ang'):
            assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), k
        assert bool(torch.equal(a['meta'], b['meta']))
    _HOST.clear()
