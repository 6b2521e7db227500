"""SURVEY §8(f) rows f3/f4 on the device vs the reference's golden vectors
(g9_collate, g10_progenitors) and the pinned oracle (needs a GPU).

Bar: collated particle IDs, counts, offsets and halo tables, final counts, central
IDs and main-progenitor numbers bit-exact (integer work)."""
import numpy as np
import pytest

from golden_util import assert_same
from post_golden import collate_runs, central_cases, mainprog_cases
from oracle import post_oracle as PO

pytestmark = pytest.mark.gpu

RUNS = collate_runs()


class _Mem:
    def __init__(self, groups=None, attrs=None):
        self.groups = groups if groups is not None else {}
        self.attrs = attrs if attrs is not None else {}

    def write_group(self, name, datasets):
        if name in self.groups:
            raise ValueError(name)
        self.groups[name] = {k: np.asarray(v) for k, v in datasets.items()}


def _collate(groups, attrs, kw, fkw):
    from orbitanalysis_amd.postprocessing import Apsides
    src = _Mem({g: dict(d) for g, d in groups.items()}, dict(attrs))
    dst = _Mem()
    ap = Apsides(src)
    ap.collate_apsides(savefile=dst, verbose=False, **kw)
    if fkw is not None:
        ap.save_final_apsis_counts(dst, verbose=False, **fkw)
    return dst.groups


@pytest.mark.parametrize('run', RUNS, ids=['%s-%s' % r[:2] for r in RUNS])
def test_collate_matches_reference(run):
    case, tag, groups, attrs, kw, fkw, want = run
    got = _collate(groups, attrs, kw, fkw)
    assert sorted(got) == sorted(want)
    for g in want:
        assert list(got[g]) == list(want[g]), (g, list(got[g]), list(want[g]))
        for d in want[g]:
            assert_same(got[g][d], want[g][d], '%s/%s/%s' % (tag, g, d))


def _random_track_file(rng, n_halos, n_snap, per_halo, id_dtype, id_hi, mode='pericentric'):
    """Synthetic track_orbits output: per snapshot, apsis IDs drawn (with repeats
    across snapshots) from per-halo pools, f16 angles, a halo that appears late."""
    pools = [rng.choice(id_hi, size=per_halo * 3, replace=False).astype(id_dtype)
             for _ in range(n_halos)]
    groups = {}
    tag = '{}er'.format(mode[:-3])
    for s in range(1, n_snap + 1):
        present = np.arange(n_halos) if s > 1 else np.arange(n_halos - 1)
        lens = rng.integers(0, per_halo, len(present))
        if s == 2:
            lens[0] = 0
        ids = [rng.choice(pools[h], size=l, replace=False) for h, l in zip(present, lens)]
        g = {'region_offsets': np.cumsum([0] + [len(x) for x in ids]),
             tag + '_IDs': np.concatenate(ids).astype(id_dtype) if ids else np.zeros(0, id_dtype),
             'angles': rng.uniform(0, 3, int(lens.sum())).astype(np.float16),
             'halo_IDs': present + 100}
        if s != n_snap:
            g['final_descendant_IDs'] = present + 100
        g['region_radii'] = rng.uniform(1, 2, len(present))
        g['region_positions'] = rng.uniform(0, 9, (len(present), 3))
        g['bulk_velocities'] = rng.normal(0, 1, (len(present), 3))
        groups['snapshot_%03d' % s] = g
    return groups, {'mode': mode}


@pytest.mark.parametrize('id_dtype,id_hi,per_halo', [
    (np.int64, 2 ** 62, 3000),          # signed keys, large values
    (np.int32, 2 ** 31 - 1, 500),
    (np.uint32, 2 ** 32 - 1, 500),
    (np.uint64, 2 ** 62, 500),          # values past 2^63 after the offset below
    (np.int64, 100000, 20000),          # > OA_COLLATE_CHUNK records per halo: several rounds
])
def test_collate_random_vs_oracle(id_dtype, id_hi, per_halo):
    rng = np.random.default_rng(per_halo + np.dtype(id_dtype).itemsize)
    groups, attrs = _random_track_file(rng, 5, 4, per_halo, id_dtype, id_hi)
    if id_dtype == np.uint64:
        for g in groups.values():
            g['pericenter_IDs'] = g['pericenter_IDs'] + np.uint64(2 ** 63)
    for kw in ({}, {'angle_cut': 1.5, 'halo_ids': np.array([103, 101, 104])}):
        want = PO.collate_apsides(groups, attrs, **kw)
        fin = PO.save_final_apsis_counts(want, 'pericentric')
        for g, v in fin.items():
            want[g]['pericenter_counts_final'] = v
        got = _collate(groups, attrs, kw, {})
        assert sorted(got) == sorted(want)
        for g in want:
            for d in want[g]:
                assert_same(got[g][d], want[g][d], '%s/%s' % (g, d))


def test_collate_many_halos_several_snapshots():
    """Many halos through k_collate_rank / k_collate_offsets / k_collate_place: 3000
    halos over 5 snapshots (each halo's list merged into a growing state), all outputs
    vs the oracle."""
    rng = np.random.default_rng(11)
    groups, attrs = _random_track_file(rng, 3000, 5, 60, np.int64, 2 ** 40)
    want = PO.collate_apsides(groups, attrs)
    got = _collate(groups, attrs, {'save_final_counts': False}, None)
    assert sorted(got) == sorted(want)
    for g in want:
        for d in want[g]:
            assert_same(got[g][d], want[g][d], '%s/%s' % (g, d))


@pytest.mark.parametrize('id_dtype', [np.int64, np.uint64])
def test_collate_extreme_ids_vs_oracle(id_dtype):
    """IDs at the ends of the key range: the largest one's order key is all ones, the
    value k_collate_rank pads its sort with; the smallest is key 0."""
    rng = np.random.default_rng(17)
    groups, attrs = _random_track_file(rng, 6, 4, 300, np.int64, 10 ** 6)
    info = np.iinfo(id_dtype)
    for s, g in enumerate(sorted(groups)):
        ids = g_ids = groups[g]['pericenter_IDs'].astype(id_dtype)
        off = groups[g]['region_offsets']
        for h in range(len(off) - 1):
            if off[h + 1] - off[h] >= 3:            # extremes in several halos, repeated
                g_ids[off[h]] = info.max
                g_ids[off[h] + 1] = info.min
                if s % 2:
                    g_ids[off[h] + 2] = info.max - 1
        groups[g]['pericenter_IDs'] = ids
        groups[g]['angles'] = np.full(len(ids), 2.0, dtype=np.float16)
    want = PO.collate_apsides(groups, attrs)
    got = _collate(groups, attrs, {'save_final_counts': False}, None)
    assert sorted(got) == sorted(want)
    for g in want:
        for d in want[g]:
            assert_same(got[g][d], want[g][d], '%s/%s' % (g, d))


def test_collate_inconsistent_workspace_raises_bounds_status():
    """k_collate_place / k_collate_rank check every store against its halo's range: a
    corrupted workspace (lower bounds past a halo's merged range, a new_base past the
    workspace) sets
    OA_POST_BOUNDS and stores nothing out of range, instead of faulting.  The round runs
    as its two phases (rank, then offsets + place) with the corruption in between."""
    import ctypes
    import torch
    from orbitanalysis_amd import _native as N
    lib = N.load(require_device=True)
    dev = torch.device('cuda', 0)
    rng = np.random.default_rng(5)
    nh, per = 4, 300
    old_k = [np.unique(rng.choice(10 ** 6, per)) for _ in range(nh)]
    new_ids = [rng.choice(np.concatenate([old_k[h][:100], rng.choice(10 ** 6, 100)]), 150)
               for h in range(nh)]
    src_cnt = np.array([len(x) for x in new_ids], np.int64)
    src_off = np.concatenate([[0], np.cumsum(src_cnt)[:-1]]).astype(np.int64)
    ids = torch.from_numpy(np.concatenate(new_ids).astype(np.int64)).to(dev)
    ang = torch.full((ids.numel(),), 0x4000, dtype=torch.int16, device=dev)    # 2.0
    lut = torch.ones(65536, dtype=torch.uint8, device=dev)
    okeys = torch.from_numpy(np.concatenate(old_k).astype(np.int64) ^ np.int64(-2 ** 63)).to(dev)
    ooff = torch.from_numpy(np.concatenate([[0], np.cumsum([len(k) for k in old_k])])).to(dev)
    ocnt = torch.ones_like(okeys)
    cap, n_old = int(src_cnt.sum()), int(okeys.numel())
    src_off_d, src_cnt_d = torch.from_numpy(src_off).to(dev), torch.from_numpy(src_cnt).to(dev)

    def run(corrupt):
        i32 = dict(dtype=torch.int32, device=dev)
        w = dict(keys=torch.empty(cap, dtype=torch.int64, device=dev),
                 cnt=torch.empty(cap, **i32), lb=torch.empty(cap, **i32),
                 fp=torch.empty(cap, **i32), ulen=torch.empty(nh, **i32),
                 found=torch.empty(nh, **i32))
        base = torch.from_numpy(src_off.copy()).to(dev)
        new_off = torch.empty(nh + 1, dtype=torch.int64, device=dev)
        sentinel = -7
        new_keys = torch.full((n_old + cap,), sentinel, dtype=torch.int64, device=dev)
        new_cnt = torch.full((n_old + cap,), sentinel, dtype=torch.int64, device=dev)
        status = torch.zeros(1, **i32)
        p = lambda t: ctypes.c_void_p(t.data_ptr())             # noqa: E731
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

        def args(phases):
            return N.CollateArgs(
                n_halos=nh, in_kind=0, key_signed=1, chunk_start=0, lds_keys=256,
                phases=phases, apsis_ids=p(ids), angles=p(ang), keep_lut=p(lut),
                src_off=p(src_off_d), src_cnt=p(src_cnt_d), new_base=p(base),
                old_keys=p(okeys), old_cnt=p(ocnt), old_off=p(ooff), n_old=n_old,
                n_new_cap=cap, w_keys=p(w['keys']), w_cnt=p(w['cnt']), w_lb=p(w['lb']),
                w_fp=p(w['fp']), w_ulen=p(w['ulen']), w_found=p(w['found']),
                new_off=p(new_off), new_keys=p(new_keys), new_cnt=p(new_cnt),
                status=p(status))
        if corrupt == 'base':
            base[2] = cap - 10                       # its 150 rows would run past the end
        a1 = args(1)
        N.check(lib.oa_collate_step(ctypes.byref(a1), st), 'oa_collate_step rank')
        if corrupt == 'lb':
            # halo 1's absent keys placed past its merged range
            w['lb'][int(src_off[1]):int(src_off[2])] = 10 ** 6
        a2 = args(2)
        N.check(lib.oa_collate_step(ctypes.byref(a2), st), 'oa_collate_step merge')
        torch.cuda.synchronize()
        off = new_off.cpu().numpy()
        return int(status.item()), off, new_keys.cpu().numpy(), new_cnt.cpu().numpy()

    s0, off0, k0, c0 = run(None)
    assert s0 == 0
    want = [np.unique(np.concatenate([old_k[h], new_ids[h]])) for h in range(nh)]
    got = [(k0[off0[h]:off0[h + 1]] ^ np.int64(-2 ** 63)) for h in range(nh)]
    for h in range(nh):
        assert np.array_equal(got[h], want[h])
    for corrupt in ('lb', 'base'):
        s, off, k, c = run(corrupt)
        assert s & N.POST_BOUNDS, (corrupt, s)
        # nothing was stored past the merged state's end
        assert np.all(k[int(off0[-1]):] == -7) and np.all(c[int(off0[-1]):] == -7), corrupt


def test_retro_counts_missing_id_raises():
    from orbitanalysis_amd.postprocessing import Apsides
    rng = np.random.default_rng(3)
    groups, attrs = _random_track_file(rng, 3, 3, 200, np.int64, 10 ** 6)
    dst = _Mem()
    ap = Apsides(_Mem(groups, attrs))
    ap.collate_apsides(savefile=dst, verbose=False)
    first = sorted(dst.groups)[0]
    dst.groups[first]['particle_IDs'] = dst.groups[first]['particle_IDs'].copy()
    dst.groups[first]['particle_IDs'][0] = -5
    with pytest.raises(ValueError):
        ap.save_final_apsis_counts(dst, verbose=False)


@pytest.mark.parametrize('case', central_cases(), ids=lambda c: c[0])
def test_central_ids_match_reference(case):
    from orbitanalysis_amd.progenitors import get_central_particle_ids
    name, snap, pos, n, want_ids, want_off = case
    ids, off = get_central_particle_ids(snap, pos, n=n)
    assert_same(ids, want_ids, name + '/ids')
    assert_same(off, want_off, name + '/offsets')


@pytest.mark.parametrize('n,sizes,dtype,box', [
    (100, [20000, 9000, 50, 0, 8192], np.float32, 40.0),    # LDS cache and global-scratch blocks
    (4096, [5000, 4096, 100], np.float64, None),
    (1, [300, 1], np.float64, [10.0, 11.0, 12.0]),
])
def test_central_ids_random_vs_oracle(n, sizes, dtype, box):
    from orbitanalysis_amd.progenitors import get_central_particle_ids
    rng = np.random.default_rng(sum(sizes))
    x = rng.uniform(0, 40, (sum(sizes), 3)).astype(dtype)
    snap = {'ids': rng.permutation(10 ** 7)[:sum(sizes)].astype(np.int64), 'coordinates': x,
            'region_offsets': np.cumsum([0] + sizes[:-1])}
    if box is not None:
        snap['box_size'] = box
    pos = rng.uniform(0, 40, (len(sizes), 3)).astype(dtype)
    want = PO.get_central_particle_ids(snap, pos, n=n)
    got = get_central_particle_ids(snap, pos, n=n)
    assert_same(got[0], want[0], 'ids')
    assert_same(got[1], want[1], 'offsets')


@pytest.mark.parametrize('dtype', [np.float64, np.float32])
def test_central_ids_radius_ties_vs_oracle(dtype):
    """k_central selects on r^2 and orders the selected by (r, position): the n-th radius
    falls inside a shell of particles whose r^2 differ by a few ulps but whose radii
    round to the same values (sqrt plateaus), and inside a group of identical
    positions; the order must still be the stable (r, position) order."""
    from orbitanalysis_amd.progenitors import get_central_particle_ids
    rng = np.random.default_rng(5)
    blocks = []
    for R in (3.0, 1.0 + 2 ** -30, 7.25):
        th = rng.uniform(0, 2 * np.pi, 400)
        shell = np.stack([R * np.cos(th), R * np.sin(th), np.zeros_like(th)], 1)
        inner = rng.uniform(-R / 4, R / 4, (60, 3))
        same = np.tile(rng.uniform(-R, R, (1, 3)) * 0.5, (40, 1))
        outer = rng.uniform(-3 * R, 3 * R, (3000, 3))
        b = np.concatenate([outer[:1500], shell[:200], same, inner, shell[200:], outer[1500:]])
        blocks.append(b[rng.permutation(len(b))] if R == 7.25 else b)
    x = (np.concatenate(blocks) + 50.0).astype(dtype)
    sizes = [len(b) for b in blocks]
    snap = {'ids': rng.permutation(10 ** 6)[:sum(sizes)].astype(np.int64), 'coordinates': x,
            'region_offsets': np.cumsum([0] + sizes[:-1])}
    pos = np.full((len(sizes), 3), 50.0, dtype=dtype)
    for n in (100, 130, 300):
        want = PO.get_central_particle_ids(snap, pos, n=n)
        got = get_central_particle_ids(snap, pos, n=n)
        assert_same(got[0], want[0], 'ids n=%d' % n)
        assert_same(got[1], want[1], 'offsets n=%d' % n)


@pytest.mark.parametrize('case', mainprog_cases(), ids=lambda c: c[0])
def test_main_progenitors_match_reference(case):
    from orbitanalysis_amd.progenitors import find_main_progenitors
    name, hp, ho, tp, to, want = case
    got = find_main_progenitors(hp, ho, tp, to)
    assert np.array_equal(np.array([int(v) for v in got]), want), name
    assert all(v == -1 or isinstance(v, np.int64) for v in got)


def test_main_progenitors_random_vs_oracle():
    from orbitanalysis_amd.progenitors import find_main_progenitors
    rng = np.random.default_rng(11)
    sizes = rng.integers(0, 3000, 400)
    hp = rng.choice(2 ** 50, int(sizes.sum()), replace=False).astype(np.int64)
    ho = np.cumsum(np.concatenate([[0], sizes[:-1]]))
    blocks = [rng.choice(hp, int(rng.integers(0, 300)), replace=False) for _ in range(500)]
    blocks[7] = np.concatenate([blocks[7], blocks[3][:50]])            # duplicates
    blocks.append(rng.choice(hp, 20000, replace=False))                   # one long block
    to = np.cumsum([0] + [len(b) for b in blocks])[:-1]
    tp = np.concatenate(blocks)
    want = PO.find_main_progenitors(hp, ho, tp, to)
    got = find_main_progenitors(hp, ho, tp, to)
    assert [int(v) for v in got] == [int(v) for v in want]


def test_post_calls_raise_like_the_reference():
    from orbitanalysis_amd.progenitors import get_central_particle_ids, find_main_progenitors
    from orbitanalysis_amd.postprocessing import Apsides
    rng = np.random.default_rng(5)
    snap = {'ids': np.arange(20000, dtype=np.int64), 'coordinates': rng.uniform(0, 1, (20000, 3)),
            'region_offsets': np.array([0])}
    with pytest.raises(NotImplementedError):          # n beyond the LDS survivor sort
        get_central_particle_ids(snap, np.zeros((1, 3)), n=5000)
    ids, off = get_central_particle_ids(snap, np.zeros((1, 3)), n=0)
    assert ids.size == 0 and list(off) == [0]
    with pytest.raises(NotImplementedError):          # in1d would compare uint64 as float
        find_main_progenitors(np.arange(10, dtype=np.uint64), np.array([0]),
                              np.arange(3, dtype=np.uint64), np.array([0]))
    groups, attrs = _random_track_file(rng, 2, 3, 50, np.int64, 10 ** 6)
    with pytest.raises(ValueError):
        Apsides(_Mem(groups, attrs)).collate_apsides(halo_ids=np.array([999]), savefile=_Mem(),
                                                     verbose=False)
