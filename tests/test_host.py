"""CPU-only checks: the C-ABI library loads and exports every declared symbol, struct
layouts agree, host-side planning mirrors NumPy's promotion rules, and the device
path fails loudly without a GPU (no silent CPU fallback)."""
import os
import re
import ctypes

import numpy as np
import pytest

from conftest import ROOT


def test_library_exports_every_declared_symbol():
    from orbitanalysis_amd import _native as N
    lib = N.load()
    hdr = ''.join(open(os.path.join(ROOT, 'include', h)).read()
                  for h in ('orbit_hip.h', 'orbit_post.h'))
    declared = set(re.findall(r'\b(oa_[a-z_0-9]+)\s*\(', hdr))
    assert declared, 'no declarations parsed'
    raw = ctypes.CDLL(N.LIB_PATH)
    for name in declared:
        assert hasattr(raw, name), name
    assert declared == set(N.SYMBOLS), declared ^ set(N.SYMBOLS)
    assert lib.oa_abi_version() == N.ABI_VERSION
    assert lib.oa_struct_size(0) == 96 and lib.oa_struct_size(1) == 48
    from orbitanalysis_amd import engine as E
    for f64 in (False, True):
        assert lib.oa_step_lds_bytes(E.DEFAULT_ENTRIES[f64], E.DEFAULT_SLOTS[f64], int(f64)) \
            <= 160 * 1024
    assert lib.oa_build_info(0) % 64 == 0 and lib.oa_build_info(1) >= 1
    post = open(os.path.join(ROOT, 'include', 'orbit_post.h')).read()
    assert int(re.search(r'OA_COLLATE_CHUNK (\d+)', post).group(1)) == N.COLLATE_CHUNK
    assert int(re.search(r'OA_CENTRAL_MAX_N (\d+)', post).group(1)) == N.CENTRAL_MAX_N


def test_no_silent_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from orbitanalysis_amd import _native as N
    from orbitanalysis_amd.engine import OrbitEngine
    with pytest.raises(N.NativeUnavailable):
        OrbitEngine()


def test_post_calls_reject_bad_args_without_device():
    from orbitanalysis_amd import _native as N
    lib = N.load()
    a = N.CentralArgs()
    a.n_halos, a.n, a.id_bytes = 1, N.CENTRAL_MAX_N + 1, 8
    assert lib.oa_central_ids(a, None) == -1
    assert b'OA_CENTRAL_MAX_N' in lib.oa_last_error()
    m = N.MainProgArgs()
    m.n_blocks, m.halo_kind, m.tracked_kind = 1, 1, 0
    assert lib.oa_main_progenitors(m, None) == -1
    assert lib.oa_retro_counts(None, 7, 5, None, None, 0, None, None, None, None, None, None) == -1
    assert lib.oa_mainprog_workspace_bytes(10 ** 8, 10) >= 16 * 64 + 40   # tracked-side table only


def test_box_plan_follows_numpy_promotion():
    from orbitanalysis_amd.progenitors import _box_plan
    f32, f64 = np.dtype(np.float32), np.dtype(np.float64)
    # scalar box -> float64 array (utils.py:28-29): strong float64 comparisons
    assert [p[0] for p in _box_plan(30.0, f32)] == [True] * 3
    # list of Python floats: weak, compared and subtracted in the dx dtype
    p = _box_plan([20.0, 25.1, 30.0], f32)
    assert [q[0] for q in p] == [False] * 3
    assert p[1][2] == float(np.float32(25.1 / 2))
    # float32 array box: float32; 1-element float64 array: x only
    assert [q[0] for q in _box_plan(np.array([10.0, 12.0, 14.0], np.float32), f32)] == [False] * 3
    assert len(_box_plan(np.array([10.0]), f32)) == 1


def test_null_args_rejected_without_device():
    from orbitanalysis_amd import _native as N
    lib = N.load()
    a = N.StepArgs()
    a.id_bytes = 3
    assert lib.oa_step(a, None) == -1
    assert b'id_bytes' in lib.oa_last_error()


@pytest.mark.parametrize('coord,centre,vel,bulk,box', [
    (np.float64, np.float64, np.float64, None, None),
    (np.float32, np.float32, np.float32, None, 50.0),
    (np.float32, np.float32, np.float32, 'cat32', [60.0, 70.0, 80.0]),
    (np.float32, np.float64, np.float32, 'cat64', np.array([10.0, 10.0, 10.0], np.float32)),
    (np.float32, np.float32, np.float32, 'mass64', np.array([10.0], np.float64)),
])
def test_dtype_plan_follows_numpy(coord, centre, vel, bulk, box):
    from orbitanalysis_amd.engine import plan_dtypes
    from orbitanalysis_amd.utils import hubble_parameter
    n = 5
    snap = {'ids': np.arange(n), 'coordinates': np.ones((n, 3), coord),
            'velocities': np.ones((n, 3), vel), 'masses': 1.0, 'redshift': 0.3}
    if box is not None:
        snap['box_size'] = box
    cat = None
    if bulk == 'cat32':
        cat = np.zeros((1, 3), np.float32)
    elif bulk == 'cat64':
        cat = np.zeros((1, 3), np.float64)
    elif bulk == 'mass64':
        snap['masses'] = np.ones(n, np.float64)
    H = hubble_parameter(0.3, 70.0, 0.3, 0.7)
    c = np.zeros(3, centre)
    p = plan_dtypes(snap, c, None if cat is None else cat[0], H, 0.3)
    dx = snap['coordinates'] - c
    assert p.dx == dx.dtype
    from oracle import orbit_oracle as O
    if box is not None:
        ref = O.recenter_coordinates(dx.copy(), box)
        assert ref.dtype == p.dx
        assert len(p.box) == (3 if np.ndim(box) == 0 else len(box))
    b = cat[0] if cat is not None else O.bulk_velocity(snap['velocities'], snap['masses'])
    assert p.bulk == np.asarray(b).dtype
    assert p.vb == (snap['velocities'] - b).dtype


def test_wrap_dtype_python_list_box_is_weak():
    from orbitanalysis_amd.engine import plan_dtypes
    snap = {'ids': np.arange(2), 'coordinates': np.ones((2, 3), np.float32),
            'velocities': np.ones((2, 3), np.float32), 'masses': 1.0, 'box_size': [5.0, 5.0, 5.0]}
    p = plan_dtypes(snap, np.zeros(3, np.float32), None, np.float64(0.0), 0.0)
    assert p.wrap_f64 is False                       # Python floats are weak (NEP 50)
    snap['box_size'] = 5.0
    assert plan_dtypes(snap, np.zeros(3, np.float32), None, np.float64(0.0), 0.0).wrap_f64


def test_plan_items_invariants():
    from orbitanalysis_amd.engine import plan_items, plan_global, GCHUNK
    rng = np.random.default_rng(0)
    cur = rng.integers(0, 3000, 500)
    cur[::37] = 50000
    prev = cur + rng.integers(-10, 10, 500)
    prev[::11] = -1
    prev[5] = 9000                                  # a progenitor block beyond max_pv
    items, glob, scratch = plan_items(cur, prev, 4096, hmax=16, max_pv=8192)
    pv = (np.maximum(prev, 0) + 63) // 64 * 64
    covered = np.zeros(500, int)
    for it in items:
        assert it['h1'] - it['h0'] <= 16
        assert cur[it['h0']:it['h1']].sum() <= 4096
        assert pv[it['h0']:it['h1']].sum() <= 8192
        covered[it['h0']:it['h1']] += 1
    for g in glob:                                  # large halos: single-halo global items
        assert g['h1'] == g['h0'] + 1 and (cur[g['h0']] > 4096 or pv[g['h0']] > 8192)
        covered[g['h0']] += 1
    assert 5 in glob['h0']
    assert np.all(covered == 1)
    segs = 0
    for it in np.concatenate([items, glob]):
        assert it['n_pv'] == ((np.maximum(prev[it['h0']:it['h1']], 0) + 63) // 64 * 64).sum()
        assert it['scratch_off'] % 64 == 0 and it['scratch_off'] == segs
        segs += (int(it['n_pv']) + 63) // 64 * 64
    assert scratch == segs
    ch1, ch2, tab, total = plan_global(glob, cur, prev, len(items), True)
    assert total == tab[:, 1].sum() and np.all(tab[:, 1] >= 2 * cur[glob['h0']])
    assert np.all((tab[:, 1] & (tab[:, 1] - 1)) == 0)          # power-of-two capacities
    for k, g in enumerate(glob):
        c1 = ch1[ch1[:, 0] == len(items) + k]
        assert c1[:, 2].sum() == cur[g['h0']] and np.all(c1[:, 1] % GCHUNK == 0)
        c2 = ch2[ch2[:, 0] == len(items) + k]
        assert c2[:, 2].sum() == max(prev[g['h0']], 0) and np.all(c2[:, 1] % 64 == 0)


def test_items_single_flag(monkeypatch):
    """oa_step_args.items_single (ABI 13) is set only when every packed item holds one
    halo (the one-halo k_step specialisation compiles the packed-item paths out), and
    the plans that pack halos keep the general kernel."""
    from orbitanalysis_amd.engine import plan_items, items_single
    big = np.full(50, 9000)
    items, _, _ = plan_items(big, big, 11776, hmax=32, max_pv=12288)
    assert np.all(items['h1'] - items['h0'] == 1) and items_single(items) == 1
    small = np.full(50, 900)
    items, _, _ = plan_items(small, small, 11776, hmax=32, max_pv=12288)
    assert np.any(items['h1'] - items['h0'] > 1) and items_single(items) == 0
    assert items_single(items[:0]) == 0
    monkeypatch.setenv('ORBIT_SINGLE', '0')
    assert items_single(plan_items(big, big, 11776, hmax=32, max_pv=12288)[0]) == 0


def test_synthetic_generator_is_deterministic():
    from orbitanalysis_amd.synthetic import PlummerSnapshots
    a = PlummerSnapshots(n_halos=2, n_per_halo=300, n_snapshots=3, seed=5).input_digest()
    b = PlummerSnapshots(n_halos=2, n_per_halo=300, n_snapshots=3, seed=5).input_digest()
    assert a == b


def test_set_item_slots_first_output_slot():
    from orbitanalysis_amd import _native as N
    from orbitanalysis_amd.engine import set_item_slots
    out_slot = np.array([-1, 0, -1, -1, 1, 2, -1])
    items = np.zeros(4, dtype=N.ITEM_DTYPE)
    items['h0'] = [0, 2, 4, 6]
    items['h1'] = [2, 4, 6, 7]
    set_item_slots(items, out_slot)
    assert list(items['slot0']) == [0, -1, 1, -1]


def test_interleave_halos_matches_per_halo_concat():
    from orbitanalysis_amd.track_orbits_onthefly import _interleave_halos
    rng = np.random.default_rng(3)
    nh = 50
    take = rng.uniform(size=nh) < 0.6
    la, lb = rng.integers(0, 6, nh), rng.integers(0, 6, nh)
    a_off = np.concatenate([[0], np.cumsum(la)])
    b_off = np.concatenate([[0], np.cumsum(lb)])
    a, b = rng.integers(0, 100, a_off[-1]), rng.integers(100, 200, b_off[-1])
    got, off = _interleave_halos(take, a, a_off, b, b_off)
    want = [a[a_off[j]:a_off[j + 1]] if take[j] else b[b_off[j]:b_off[j + 1]] for j in range(nh)]
    assert np.array_equal(got, np.concatenate(want))
    assert np.array_equal(off, np.concatenate([[0], np.cumsum([len(w) for w in want])]))


def test_onthefly_carry_key_and_switch(monkeypatch):
    from orbitanalysis_amd import track_orbits_onthefly as T
    monkeypatch.setenv('ORBIT_OTF_CARRY', '0')
    assert not T._carry_enabled()
    monkeypatch.setenv('ORBIT_OTF_CARRY', '1')
    assert T._carry_enabled()
    assert T._same(np.array([1.0, np.nan]), np.array([1.0, np.nan]))
    assert not T._same(np.array([1.0], np.float32), np.array([1.0]))
    T.clear_carry()
    assert T._CARRY == {}


def test_plan_items_slots():
    """The host planner (C++) fills slot0 like set_item_slots (its speed, ~0.5 ms per
    1e4 halos against ~43 ms for the Python loop it replaced, is measured by
    tools/bench_e2e.py, not asserted here: a wall-clock bound flakes on loaded hosts)."""
    from orbitanalysis_amd.engine import plan_items, set_item_slots
    rng = np.random.default_rng(1)
    nh = 10000
    cur = rng.integers(9000, 11000, nh)
    prev = cur + rng.integers(-50, 50, nh)
    prev[::7] = -1
    out_slot = np.where(prev >= 0, np.cumsum(prev >= 0) - 1, -1)
    items, glob, scratch = plan_items(cur, prev, 11776, 32, out_slot=out_slot)
    want = items.copy()
    set_item_slots(want, out_slot)
    assert np.array_equal(items['slot0'], want['slot0'])


def test_checkpoint_angles_length_checked():
    from orbitanalysis_amd.engine import check_angles_in
    check_angles_in(None, 5)
    check_angles_in(np.zeros(5, np.float16), 5)
    with pytest.raises(ValueError):
        check_angles_in(np.zeros(4, np.float16), 5)


def test_resume_without_checkpoint_raises():
    """resume=True re-processes the last saved snapshot from its checkpoint angles
    (track_orbits.py:229-232); without them the reference fails opening the
    .checkpoint file, and so does the drop-in (before any device work)."""
    from orbitanalysis_amd.track_orbits import track_orbits
    from orbitanalysis_amd.savefile import MemorySavefile

    class StubEngine:
        mode, prev = 'pericentric', None

        def reset(self):
            pass

    out = MemorySavefile()
    out.initialize('pericentric', None)
    out.write_group('snapshot_001', {})
    snap = {'ids': np.arange(3), 'coordinates': np.zeros((3, 3)), 'velocities': np.zeros((3, 3)),
            'masses': 1.0, 'region_offsets': np.array([0]), 'redshift': 0.0, 'H0': 1.0,
            'Omega_m': 0.3, 'Omega_L': 0.7}
    with pytest.raises(FileNotFoundError):
        track_orbits([0, 1, 2], [[0], [0], [0]], lambda s, h: (np.zeros((1, 3)), np.ones(1), None),
                     lambda s, p, r: dict(snap), out, resume=True, verbose=False,
                     engine=StubEngine())


def test_plan_part_bucket_sets():
    """Partition plan of the large halos (engine.plan_part): power-of-two K, the current
    set's layout, and a previous step's bucket set inherited halo by halo (any K ratio);
    a halo without one gets a fresh previous set and counters after the current ones."""
    from types import SimpleNamespace
    from orbitanalysis_amd.engine import plan_part, PART_SPREAD, GPART_W
    cur = np.array([30000, 200000, 5000, 90000, 0])
    prev = np.array([29000, 190000, -1, 88000, 10])
    glob = {'h0': np.array([0, 1, 2, 3, 4])}
    prev_idx = np.array([3, 0, -1, 2, 1])                    # previous halo numbers
    ps = SimpleNamespace(K=np.array([64, 0, 16, 32]), base=np.array([0, -1, 64 * 4096, 80 * 4096]),
                         cbase=np.array([0, 0, 64, 80]), cap=4096, key4=True)
    # a set with keys of another width is not inherited
    assert not plan_part(glob, cur, prev, 4096, 4096, prev_idx, ps, key4=False)['inherited'].any()
    pl = plan_part(glob, cur, prev, 4096, 4096, prev_idx, ps, key4=True)
    K, g = pl['K'], pl['gpart']
    assert g.shape == (5, GPART_W)
    assert all(k == 0 or (k & (k - 1)) == 0 for k in K)
    assert K[0] == 16 and K[1] == 64 and K[3] == PART_SPREAD and K[2] == 0 and K[4] > 0
    assert np.all(K[K > 0] * 4096 * 0.9 >= cur[K > 0])
    # current set: consecutive K * part_e runs, counters consecutive
    assert np.array_equal(g[:, 0], (np.cumsum(K) - K) * 4096)
    assert np.array_equal(g[:, 2], np.cumsum(K) - K)
    # halo 0 inherits previous halo 3 (K 32), halo 3 previous halo 2 (K 16); halo 1's
    # progenitor (previous halo 0) is bucketed too; halo 4's (previous 1) is not
    assert list(g[:, 3]) == [1, 1, 0, 1, 0]
    assert g[0, 4] == 80 * 4096 and g[0, 5] == 32 and g[0, 6] == 4096 and g[0, 7] == 80
    assert g[3, 4] == 64 * 4096 and g[3, 5] == 16 and g[3, 7] == 64
    assert g[1, 5] == 64 and g[1, 7] == 0
    # the fresh previous set of halo 4: K of its own, counters after the current ones
    assert g[4, 5] == K[4] and g[4, 7] == K.sum() and g[4, 6] >= 10 / K[4]
    # then one record counter per previous-block chunk (GCHUNK positions), item by item
    from orbitanalysis_amd.engine import GCHUNK
    rows = -(-np.maximum(prev, 0) // GCHUNK)
    assert pl['rc0'] == K.sum() + K[4]
    assert np.array_equal(g[:, 8], pl['rc0'] + np.cumsum(rows) - rows)
    assert pl['n_pcnt'] == pl['rc0'] + rows.sum() and pl['n_prev'] == K[4] * g[4, 6]
    assert list(pl['inherited']) == [True, True, False, True, False]
    # every current partition listed once
    pl_ok = pl['plist'][pl['plist'][:, 0] >= 0]
    assert len(pl_ok) == K.sum() and len({tuple(r) for r in pl_ok}) == K.sum()
    # the join's descriptor rows: the item's gpart row, partition, item, record chunks
    pr = pl['prow']
    assert pr.shape == (len(pl['plist']), 16)
    assert np.array_equal(pr[:, 10], pl['plist'][:, 0]) and np.array_equal(pr[:, 9] * (pr[:, 10] >= 0), pl['plist'][:, 1] * (pl['plist'][:, 0] >= 0))
    live = pr[:, 10] >= 0
    assert np.array_equal(pr[live, :9], g[pr[live, 10], :9])
    assert np.array_equal(pr[live, 12], rows[pr[live, 10]])


def test_plan_part_memory_scales_with_halo_size():
    """the partition floor scales with the halo, so many global halos just
    past the item budget do not each take PART_SPREAD * part_e bucket entries; and a
    re-plan after an LDS table overflow leaves the partitioned path (its smaller items
    would turn every halo into a global item)."""
    from types import SimpleNamespace
    from orbitanalysis_amd import _native as N
    from orbitanalysis_amd.engine import plan_part, retry_plan, PART_SPREAD
    n = 2000
    cur = np.full(n, 6200)
    glob = {'h0': np.arange(n)}
    pl = plan_part(glob, cur, cur, 4096, 4096)
    assert pl['n_cur'] <= 3 * cur.sum(), pl['n_cur'] / cur.sum()
    big = plan_part({'h0': np.arange(3)}, np.full(3, 100000), np.full(3, 100000), 4096, 4096)
    assert np.all(big['K'] == PART_SPREAD)          # configs[1]'s halos keep the full spread
    pr = SimpleNamespace(entries=6144, part=True)
    assert retry_plan(pr, N.STATUS_TABLE_OVERFLOW) == (3072, False)
    assert retry_plan(pr, N.STATUS_PART_OVERFLOW) == (6144, False)
    assert retry_plan(pr, N.STATUS_PART_KEYS) == (6144, False)
    assert retry_plan(pr, N.STATUS_LOOKBACK) == (6144, True)
    pr.entries = 256
    assert retry_plan(pr, N.STATUS_TABLE_OVERFLOW) == (0, False)


def test_build_halos_matches_structured_fill():
    """oa_build_halos (host C++) writes the same oa_halo rows as field-by-field NumPy
    assignment into HALO_DTYPE (the table OrbitEngine.build_tables uploads)."""
    import numpy as np
    from orbitanalysis_amd import _native as N
    lib = N.load()
    rng = np.random.default_rng(4)
    n = 257
    cols = {k: rng.integers(-5, 1 << 40, n).astype(np.int64)
            for k in ('cur_off', 'cur_cnt', 'prev_off', 'prev_cnt', 'out_slot')}
    cen, blk = rng.normal(size=(n, 3)), rng.normal(size=(n, 3))
    for bulk in (blk, None):
        want = np.zeros(n, dtype=N.HALO_DTYPE)
        for k, v in cols.items():
            want[k] = v
        want['centre'] = cen
        if bulk is not None:
            want['bulk'] = bulk
        got = np.empty(n, dtype=N.HALO_DTYPE)
        rc = lib.oa_build_halos(*(cols[k].ctypes.data for k in ('cur_off', 'cur_cnt', 'prev_off',
                                                                 'prev_cnt', 'out_slot')),
                                cen.ctypes.data, None if bulk is None else bulk.ctypes.data, n,
                                got.ctypes.data)
        assert rc == 0
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    assert lib.oa_build_halos(None, None, None, None, None, None, None, 3, None) < 0


def test_block_starts_vectorised_matches_rule():
    """track_orbits_onthefly._block_starts (vectorised) equals the row-by-row rule on
    random repacked slices: absent halos, gaps, empty blocks, and out-of-order blocks
    (ValueError in both)."""
    import numpy as np
    from orbitanalysis_amd.track_orbits_onthefly import _block_starts, _block_starts_loop
    rng = np.random.default_rng(0)
    for _ in range(2000):
        nh = int(rng.integers(1, 30))
        sizes, gaps = rng.integers(0, 5, nh), rng.integers(0, 3, nh)
        st = np.cumsum(gaps + np.concatenate([[0], sizes[:-1]]))
        sl = np.stack([st, st + sizes], 1)
        sl[rng.uniform(size=nh) < 0.3] = -1
        if rng.uniform() < 0.2:
            i = int(rng.integers(0, nh))
            if sl[i, 0] >= 0:
                sl[i, 0] = max(sl[i, 0] - 3, 0)
        outs = []
        for f in (_block_starts_loop, lambda s: _block_starts(s, 100)):
            try:
                outs.append(f(sl))
            except ValueError:
                outs.append(None)
        assert (outs[0] is None) == (outs[1] is None)
        assert outs[0] is None or np.array_equal(outs[0], outs[1])
