"""BASELINE.json's multi-GPU configurations at their workload on the product paths
(needs a GPU; the ranks share it and talk over gloo).

* configs[4] -- the track_orbits_onthefly stream, 1e9 particles over 8 GPUs: one rank's
  share (1.25e8 f32 particles, 12,500 halos) through ``ShardedOnTheFly`` at world 1,
  three chained calls with the frame state carried, checked by size-independent
  properties, against the oracle on a halo sample, and bit for bit against the
  single-GPU on-the-fly path; and the same share over two ranks handed whole
  snapshots (stripes, the owner all-to-all and the root's merge at size).
* configs[3] -- 1e8 particles in total sharded by ID range: two ranks run
  ``ShardedEngine`` over 1e4 halos, three snapshots, with the reference's whole-snapshot
  loader (stripes + all-to-all) and with a presharded loader; rank 0's savefile
  (groups and checkpoint) equals a single-process ``OrbitEngine`` run's bit for bit
  (track_orbits.py:189-194 is the reference's parallel axis).
"""
import json
import os
import tempfile

import numpy as np

from golden_util import check_changes
import pytest
import torch.multiprocessing as mp

from device_universe import DeviceUniverse, rank_major, digest
from test_sharding import _free_port

pytestmark = pytest.mark.gpu


def _keys(snap, nh):
    """(halo << 40 | ID) of every row of a device snapshot, and each row's halo."""
    import torch
    dev = snap['ids'].device
    off = np.append(snap['region_offsets'], snap['ids'].numel())
    h = torch.repeat_interleave(torch.arange(nh, device=dev), torch.from_numpy(np.diff(off)).to(dev))
    return (h << 40) | snap['ids'], h


def _member(sorted_keys, q):
    import torch
    if not sorted_keys.numel():
        return torch.zeros_like(q, dtype=torch.bool)
    k = torch.searchsorted(sorted_keys, q).clamp_(max=sorted_keys.numel() - 1)
    return sorted_keys[k] == q


def check_apsis_in_prev_blocks(prev_snap, nh, offs, ids):
    """Apsis IDs: offsets from 0 to the record count, every ID in its halo's previous
    block once, in that block's order (track_orbits.py:300-316)."""
    import torch
    assert offs[0] == 0 and np.all(np.diff(offs) >= 0) and offs[-1] == len(ids)
    pkey, _ = _keys(prev_snap, nh)
    srt, perm = torch.sort(pkey)
    dev = pkey.device
    ah = torch.repeat_interleave(torch.arange(nh, device=dev), torch.from_numpy(np.diff(offs)).to(dev))
    akey = (ah << 40) | torch.from_numpy(np.asarray(ids, np.int64)).to(dev)
    assert bool(_member(srt, akey).all()), 'apsis ID not in its previous block'
    pos = perm[torch.searchsorted(srt, akey)]
    same = ah[1:] == ah[:-1]
    assert bool((pos[1:] > pos[:-1])[same].all()), 'apsis IDs out of previous-block order'
    return akey


def check_onthefly_properties(prev_snap, cur_snap, nh, data, tag='pericenter'):
    """Size-independent properties of one on-the-fly file (track_orbits_onthefly.py:
    123-205): apsis IDs in previous-block order and matched; one angle change per
    matched particle; per halo, departed = previous minus current and entered =
    current minus previous, each sorted and unique."""
    import torch
    pkey, ph = _keys(prev_snap, nh)
    ckey, ch = _keys(cur_snap, nh)
    psrt, csrt = torch.sort(pkey)[0], torch.sort(ckey)[0]
    matched_p = _member(csrt, pkey)
    n_match = torch.bincount(ph[matched_p], minlength=nh).cpu().numpy()
    akey = check_apsis_in_prev_blocks(prev_snap, nh, data[tag + '_offsets'], data[tag + '_IDs'])
    assert bool(_member(csrt, akey).all()), 'apsis particle not in the current block'
    assert len(data['angles']) == int(n_match.sum())
    p_cnt = np.diff(np.append(prev_snap['region_offsets'], prev_snap['ids'].numel()))
    c_cnt = np.diff(np.append(cur_snap['region_offsets'], cur_snap['ids'].numel()))
    dev = pkey.device
    for name, own, other, cnt in (('departed', psrt, csrt, p_cnt), ('entered', csrt, psrt, c_cnt)):
        off, ids = data[name + '_offsets'], np.asarray(data[name + '_IDs'], np.int64)
        assert np.array_equal(np.diff(off), cnt - n_match), name
        h = torch.repeat_interleave(torch.arange(nh, device=dev), torch.from_numpy(np.diff(off)).to(dev))
        key = (h << 40) | torch.from_numpy(ids).to(dev)
        assert bool(_member(own, key).all()) and not bool(_member(other, key).any()), name
        assert bool((key[1:] > key[:-1]).all()), name + ' not sorted unique per halo'


def test_configs4_onthefly_rank_share_world1():
    """configs[4] at one GPU's share through the sharded on-the-fly driver (world 1):
    1.25e8 f32 particles in 12,500 halos, calls s = 1, 2, 3 with the carry on (each
    snapshot loaded once)."""
    import torch
    import torch.distributed as dist
    from oracle import orbit_oracle as O
    from orbitanalysis_amd import track_orbits_onthefly as T
    from orbitanalysis_amd.engine import OrbitEngine
    from orbitanalysis_amd.savefile import MemorySavefile
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d' % _free_port(),
                            rank=0, world_size=1)
    try:
        T.clear_carry()
        nh = 12500
        u = DeviceUniverse(4, n_halos=nh, n_particles=125_000_000, seed=9, dtype='float32')
        links = np.tile(np.arange(nh), (2, 1))
        eng = T.ShardedOnTheFly(OrbitEngine(mode='pericentric'))
        out = MemorySavefile()
        for s in (1, 2, 3):
            T.track_orbits(s, links, u.regions_otf, u.load_snapshot_data, out, verbose=False,
                           engine=eng)
            data = out.files[s][0]
            assert data['angles'].dtype == np.float32
            check_onthefly_properties(u.snaps[s - 1], u.snaps[s], nh, data)
        assert u.loads == [1, 0, 2, 3], u.loads            # s - 1 carried, not reloaded
        got = out.files[3][0]
        # the oracle on the first 40 halos of the pair (2, 3)
        k = 40
        hs = {s: u.host_blocks(s, k) for s in (2, 3)}
        want = O.onthefly_track_orbits(3, np.tile(np.arange(k), (2, 1)),
                                       lambda s, ids: (u.cats[s][0][ids], u.cats[s][1][ids]),
                                       lambda s, p, r: hs[s], mode='pericentric')
        for name in ('pericenter', 'entered', 'departed'):
            o = want[name + '_offsets']
            assert np.array_equal(got[name + '_offsets'][:k + 1], o), name
            assert np.array_equal(got[name + '_IDs'][:o[-1]], want[name + '_IDs']), name
        w = want['angles']
        check_changes(got['angles'][:len(w)], w, np.float32, 'configs[4] share')
        for a, b in zip(got['bulk_velocities'], want['bulk_velocities']):
            assert np.array_equal(a[:k], b), 'bulk velocities'
        # the single-GPU on-the-fly path on the same pair: the same file bit for bit
        T.clear_carry()
        single = MemorySavefile()
        T.track_orbits(3, links, u.regions_otf, u.load_snapshot_data, single, verbose=False)
        ref = single.files[3][0]
        assert sorted(ref) == sorted(got)
        for key in ref:
            a, b = np.asarray(got[key]), np.asarray(ref[key])
            assert a.dtype == b.dtype and a.shape == b.shape, key
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), key
    finally:
        T.clear_carry()
        dist.destroy_process_group()


def test_configs4_pinned_ring_stream_world1():
    """configs[4]'s double-buffered H2D under test: one GPU's share
    (1.25e8 f32 particles, 12,500 halos) streamed from page-locked host memory by
    ``streaming.PinnedRing`` -- the copy of snapshot s + 1 runs on a high-priority copy
    stream into one of three device slots while s is compared -- through
    ``ShardedOnTheFly`` at world 1 (RCCL is not needed at world 1: gloo), three chained
    calls with the carry on.  Every file equals the device-tensor loader's bit for bit,
    and the oracle's on 40 halos of the last pair."""
    import torch
    import torch.distributed as dist
    from oracle import orbit_oracle as O
    from orbitanalysis_amd import track_orbits_onthefly as T
    from orbitanalysis_amd.engine import OrbitEngine
    from orbitanalysis_amd.savefile import MemorySavefile
    from orbitanalysis_amd.streaming import PinnedRing, pin_snapshot
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d' % _free_port(),
                            rank=0, world_size=1)
    try:
        nh = 12500
        u = DeviceUniverse(4, n_halos=nh, n_particles=125_000_000, seed=29, dtype='float32')
        links = np.tile(np.arange(nh), (2, 1))
        ring = PinnedRing({s: pin_snapshot(u.snaps[s]) for s in range(4)})
        outs = []
        for loader in (ring.loader, u.load_snapshot_data):
            T.clear_carry()
            eng = T.ShardedOnTheFly(OrbitEngine(mode='pericentric'))
            out = MemorySavefile()
            for s in (1, 2, 3):
                T.track_orbits(s, links, u.regions_otf, loader, out, verbose=False, engine=eng)
            outs.append(out)
        # every snapshot crossed PCIe once (32 B per particle), s - 1 carried, not reloaded
        assert ring.h2d_bytes == 32 * sum(int(u.snaps[s]['ids'].numel()) for s in range(4))
        for s in (1, 2, 3):
            a, b = outs[0].files[s][0], outs[1].files[s][0]
            assert sorted(a) == sorted(b)
            for key in a:
                x, y = np.asarray(a[key]), np.asarray(b[key])
                assert x.dtype == y.dtype and x.shape == y.shape, (s, key)
                assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), (s, key)
        check_onthefly_properties(u.snaps[2], u.snaps[3], nh, outs[0].files[3][0])
        got = outs[0].files[3][0]
        k = 40
        hs = {s: u.host_blocks(s, k) for s in (2, 3)}
        want = O.onthefly_track_orbits(3, np.tile(np.arange(k), (2, 1)),
                                       lambda s, ids: (u.cats[s][0][ids], u.cats[s][1][ids]),
                                       lambda s, p, r: hs[s], mode='pericentric')
        for name in ('pericenter', 'entered', 'departed'):
            o = want[name + '_offsets']
            assert np.array_equal(got[name + '_offsets'][:k + 1], o), name
            assert np.array_equal(got[name + '_IDs'][:o[-1]], want[name + '_IDs']), name
        check_changes(got['angles'][:len(want['angles'])], want['angles'], np.float32,
                      'configs[4] pinned ring')
    finally:
        T.clear_carry()
        dist.destroy_process_group()


def _otf_digests(out, calls):
    return {'%d/%s' % (s, k): v for s in calls
            for k, v in digest({'f': out.files[s][0]}).items()}


def _otf_world2_worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from orbitanalysis_amd import track_orbits_onthefly as T
        from orbitanalysis_amd.engine import OrbitEngine
        from orbitanalysis_amd.savefile import MemorySavefile
        nh = 12500
        # the reference's loader contract: every rank is handed the whole snapshot
        u = DeviceUniverse(4, n_halos=nh, n_particles=125_000_000, seed=19, dtype='float32')
        links = np.tile(np.arange(nh), (2, 1))
        eng = T.ShardedOnTheFly(OrbitEngine(mode='apocentric'))
        out = MemorySavefile()
        for s in (1, 2, 3):
            T.track_orbits(s, links, u.regions_otf, u.load_snapshot_data, out, verbose=False,
                           engine=eng, mode='apocentric')
        if rank == 0:
            d = _otf_digests(out, (1, 2, 3))
            d['loads'] = u.loads
            with open(os.path.join(outdir, 'otf.json'), 'w') as f:
                json.dump(d, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_configs4_onthefly_world2_whole_snapshots():
    """configs[4]'s stream over two ranks (gloo, one GPU): 1.25e8 f32 particles in
    12,500 halos handed whole to every rank (stripe upload + owner all-to-all at size),
    apocentric, three chained calls with the carry on: the ranks' records meet in the
    root's merge (counting placement of the angle changes, sorted departed / entered
    IDs); every file equals the single-GPU on-the-fly path's bit for bit, and that path's
    first 40 halos of the last pair equal the oracle's."""
    from oracle import orbit_oracle as O
    from orbitanalysis_amd import track_orbits_onthefly as T
    from orbitanalysis_amd.engine import OrbitEngine
    from orbitanalysis_amd.savefile import MemorySavefile
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_otf_world2_worker, args=(world, _free_port(), d), nprocs=world,
                           join=True, start_method='spawn')
        with open(os.path.join(d, 'otf.json')) as f:
            got = json.load(f)
    assert got.pop('loads') == [1, 0, 2, 3]             # s - 1 carried on every rank
    nh = 12500
    T.clear_carry()
    try:
        u = DeviceUniverse(4, n_halos=nh, n_particles=125_000_000, seed=19, dtype='float32')
        links = np.tile(np.arange(nh), (2, 1))
        single = MemorySavefile()
        eng = OrbitEngine(mode='apocentric')
        for s in (1, 2, 3):
            T.track_orbits(s, links, u.regions_otf, u.load_snapshot_data, single, verbose=False,
                           engine=eng, mode='apocentric')
        want = _otf_digests(single, (1, 2, 3))
        assert sorted(got) == sorted(want)
        bad = [k for k in want if got[k] != want[k]]
        assert not bad, bad
        ref = single.files[3][0]
        assert len(ref['apocentrer_IDs']) > 1e6 and len(ref['entered_IDs']) > 1e4
        check_onthefly_properties(u.snaps[2], u.snaps[3], nh, ref, tag='apocentrer')
        k = 40
        hs = {s: u.host_blocks(s, k) for s in (2, 3)}
        o = O.onthefly_track_orbits(3, np.tile(np.arange(k), (2, 1)),
                                    lambda s, ids: (u.cats[s][0][ids], u.cats[s][1][ids]),
                                    lambda s, p, r: hs[s], mode='apocentric')
        for name in ('apocentrer', 'entered', 'departed'):
            w = o[name + '_offsets']
            assert np.array_equal(ref[name + '_offsets'][:k + 1], w), name
            assert np.array_equal(ref[name + '_IDs'][:w[-1]], o[name + '_IDs']), name
        check_changes(ref['angles'][:len(o['angles'])], o['angles'], np.float32,
                      'configs[4] world 2')
    finally:
        T.clear_carry()


def _universe(contract, rank, world):
    if contract == 'whole':          # every rank generates (is handed) the whole snapshot
        return DeviceUniverse(3, n_halos=10000, n_particles=100_000_000, seed=13,
                              dtype='float32')
    return DeviceUniverse(3, n_halos=10000, n_particles=100_000_000 // world, seed=13,
                          rank=rank, world=world, dtype='float32')


def _cfg3_worker(rank, world, port, contract, outdir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from orbitanalysis_amd.engine import OrbitEngine
        from orbitanalysis_amd.savefile import MemorySavefile
        from orbitanalysis_amd.sharding import ShardedEngine, EngineLocal
        from orbitanalysis_amd.track_orbits import track_orbits
        u = _universe(contract, rank, world)
        eng = ShardedEngine(EngineLocal(OrbitEngine(mode='pericentric')),
                            presharded=contract == 'presharded')
        out = MemorySavefile()
        track_orbits(u.snapshot_numbers, u.main_branches(), u.regions, u.load_snapshot_data,
                     out, verbose=False, engine=eng, checkpoint=True)
        if rank == 0:
            d = digest(out.groups)
            d['checkpoint'] = digest({'c': {'a': out.checkpoint}})['c/a']
            with open(os.path.join(outdir, 'digest.json'), 'w') as f:
                json.dump(d, f)
    finally:
        dist.destroy_process_group()


def _oracle_pair(u, s, k, group, mode='pericentric'):
    """The oracle's per-halo path (region_frame, compare_radial_velocities, calc_angles)
    on the first k blocks of snapshot pair (s-1, s) of a universe whose snapshot 0 is the
    frame-only one (angles 0), against a savefile group: per-halo offsets and apsis IDs
    bit-exact, f16 angles within one ulp, at most ANGLE_MISMATCH_MAX of them off."""
    from oracle import orbit_oracle as O
    from orbitanalysis_amd.utils import hubble_parameter
    from test_gpu_parity import mismatch_ok
    from golden_util import ANGLE_TALLY
    cos = u.gen.cosmology
    H = hubble_parameter(cos['redshift'], cos['H0'], cos['Omega_m'], cos['Omega_L'])

    def host(t):
        d = u.host_blocks(t, k)
        n = u.snaps[t]['ids'].numel()
        d['redshift'] = u.snaps[t]['redshift']
        off = np.append(u.snaps[t]['region_offsets'], n)[:k + 1]
        return d, off
    (prv, pb), (cur, cb) = host(s - 1), host(s)
    cp, cc = u.cats[s - 1], u.cats[s]
    ang = np.zeros(int(pb[-1]), np.float16)
    ids, angs, lens = [], [], []
    for j in range(k):
        rp, vp, _ = O.region_frame(prv, (pb[j], pb[j + 1]), cp[0][j], cp[2][j], H)
        rc, vc, _ = O.region_frame(cur, (cb[j], cb[j + 1]), cc[0][j], cc[2][j], H)
        d = O.compare_radial_velocities(cur['ids'][cb[j]:cb[j + 1]], prv['ids'][pb[j]:pb[j + 1]],
                                        vc, vp, rc, rp, mode)
        _, aa = O.calc_angles(cb[j + 1] - cb[j], ang[pb[j]:pb[j + 1]], d)
        ids.append(d['apsis_ids'])
        angs.append(aa)
        lens.append(len(d['apsis_ids']))
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    g_off = np.asarray(group['region_offsets'])
    assert np.array_equal(g_off[:k + 1], offs), 'per-halo offsets'
    tag = mode[:-3] + 'er_IDs'
    assert np.array_equal(np.asarray(group[tag])[:offs[-1]], np.concatenate(ids)), 'apsis IDs'
    a = np.asarray(group['angles'])[:offs[-1]].astype(np.float64)
    b = np.concatenate(angs).astype(np.float64)
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    ulp = np.spacing(np.maximum(np.abs(a), np.abs(b)).astype(np.float16)).astype(np.float64)
    assert np.all(same | (np.abs(a - b) <= ulp)), 'apsis angle off by more than 1 f16 ulp'
    assert mismatch_ok(int((~same).sum()), a.size), (int((~same).sum()), a.size)
    ANGLE_TALLY['angles'] += int(a.size)
    ANGLE_TALLY['mismatch'] += int((~same).sum())
    return a.size


@pytest.mark.timeout(900)
@pytest.mark.parametrize('contract', ['whole', 'presharded'])
def test_configs3_sharded_engine_world2(contract):
    """configs[3]: 1e8 particles in total over two ranks (ID ranges), 1e4 halos, f32,
    three snapshots; rank 0's savefile equals the single-process run's (sha256 of every
    dataset and the checkpoint), and that run's first 120 halos equal the oracle's."""
    import torch
    from orbitanalysis_amd.engine import OrbitEngine
    from orbitanalysis_amd.savefile import MemorySavefile
    from orbitanalysis_amd.track_orbits import track_orbits
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_cfg3_worker, args=(world, _free_port(), contract, d), nprocs=world,
                           join=True, start_method='spawn')
        with open(os.path.join(d, 'digest.json')) as f:
            got = json.load(f)
    # the single-process reference on the global snapshots
    if contract == 'whole':
        u = _universe('whole', 0, 1)
    else:
        us = [_universe('presharded', r, world) for r in range(world)]
        u = us[0]
        u.snaps = [rank_major([x.snaps[s] for x in us]) for s in range(3)]
        del us
    want = MemorySavefile()
    track_orbits(u.snapshot_numbers, u.main_branches(), u.regions, u.load_snapshot_data,
                 want, verbose=False, engine=OrbitEngine(mode='pericentric'), checkpoint=True)
    wd = digest(want.groups)
    wd['checkpoint'] = digest({'c': {'a': want.checkpoint}})['c/a']
    assert sorted(got) == sorted(wd)
    bad = [k for k in wd if got[k] != wd[k]]
    assert not bad, bad
    for s in (1, 2):
        g = want.groups['snapshot_%03d' % s]
        assert len(g['pericenter_IDs']) > 1e6
        check_apsis_in_prev_blocks(u.snaps[s - 1], u.n_halos, g['region_offsets'],
                                   g['pericenter_IDs'])
    # oracle contact (the digests above tie the sharded run to this one)
    assert _oracle_pair(u, 1, 120, want.groups['snapshot_001']) > 0
    torch.cuda.empty_cache()
