"""The on-the-fly driver over ID-range shards (track_orbits_onthefly.ShardedOnTheFly).

CPU: the rank merge (merge_onthefly) against a single-rank result split between
ranks.  GPU: two ranks (gloo, HIP engine each, one GPU) reproduce the reference's
on-the-fly files g6 / g6b / g6c / g6d in both modes."""
import os
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from golden_util import load, universe
from test_sharding import _free_port


def test_merge_onthefly_restores_single_rank_order():
    from orbitanalysis_amd.track_orbits_onthefly import merge_onthefly, _interleave_halos
    rng = np.random.default_rng(3)
    nh, world = 7, 3
    cnt = rng.integers(0, 40, nh)
    cnt[2] = 0
    off = np.concatenate([[0], np.cumsum(cnt)])
    n = int(off[-1])
    # apsis records / angle changes: global previous rows, increasing
    gpos = np.sort(rng.choice(10 * n + 1, n, replace=False))
    ids = rng.permutation(10 ** 6)[:n].astype(np.int64)
    ang = rng.random(n).astype(np.float32)
    # departed: per-halo sorted unique IDs
    dep = np.concatenate([np.sort(ids[off[j]:off[j + 1]]) for j in range(nh)])
    # entered: halos with a progenitor sorted, the others in loader (row) order
    p_has = rng.random(nh) < 0.6
    srt = np.concatenate([np.sort(ids[off[j]:off[j + 1]]) if p_has[j] else [] for j in range(nh)]).astype(np.int64)
    s_cnt = np.where(p_has, cnt, 0)
    raw = np.concatenate([ids[off[j]:off[j + 1]] if not p_has[j] else [] for j in range(nh)]).astype(np.int64)
    r_cnt = np.where(p_has, 0, cnt)
    raw_g = np.concatenate([gpos[off[j]:off[j + 1]] if not p_has[j] else [] for j in range(nh)]).astype(np.int64)
    owner = rng.integers(0, world, n)                  # the rank of each particle
    o = lambda c: np.concatenate([[0], np.cumsum(c)])  # noqa: E731
    s_own = np.concatenate([owner[off[j]:off[j + 1]] for j in range(nh) if p_has[j]] or [np.zeros(0, int)])
    r_own = np.concatenate([owner[off[j]:off[j + 1]] for j in range(nh) if not p_has[j]] or [np.zeros(0, int)])
    parts = []
    for r in range(world):
        m = owner == r
        h = np.repeat(np.arange(nh), cnt)
        c = np.bincount(h[m], minlength=nh)
        # departed of rank r: its own IDs of each halo, sorted
        dsel = np.concatenate([np.sort(ids[off[j]:off[j + 1]][m[off[j]:off[j + 1]]]) for j in range(nh)]).astype(np.int64)
        ss = s_own == r
        rs = r_own == r
        sh = np.repeat(np.arange(nh), s_cnt)
        rh = np.repeat(np.arange(nh), r_cnt)
        sv = np.concatenate([np.sort(srt[sh == j][ss[sh == j]]) for j in range(nh)]).astype(np.int64)
        parts.append(dict(apsis_offsets=o(c), apsis_ids=ids[m], apsis_gpos=gpos[m],
                          angles=ang[m], angle_gpos=gpos[m],
                          departed_offsets=o(c), departed_ids=dsel,
                          srt=sv, s_off=o(np.bincount(sh[ss], minlength=nh)),
                          raw=raw[rs], r_off=o(np.bincount(rh[rs], minlength=nh)),
                          raw_gpos=raw_g[rs], p_has=p_has))
    got = merge_onthefly(parts, nh)
    assert np.array_equal(got['apsis_offsets'], off)
    assert np.array_equal(got['apsis_ids'], ids)
    assert np.array_equal(got['angles'], ang)
    assert np.array_equal(got['departed_ids'], dep) and np.array_equal(got['departed_offsets'], off)
    want_e, want_off = _interleave_halos(p_has, srt, o(s_cnt), raw, o(r_cnt))
    assert np.array_equal(got['entered_ids'], want_e)
    assert np.array_equal(got['entered_offsets'], want_off)


def _worker(rank, world, port, name, mode, outdir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from orbitanalysis_amd.engine import OrbitEngine
        from orbitanalysis_amd.savefile import MemorySavefile
        from orbitanalysis_amd.track_orbits_onthefly import track_orbits, ShardedOnTheFly
        fix = load(name)
        u, meta = universe(fix)
        s = meta.get('snapshot', 5)
        out = MemorySavefile()
        eng = ShardedOnTheFly(OrbitEngine(mode=mode))
        data = track_orbits(s, fix['links'], u.regions, u.load_snapshot_data, out, mode=mode,
                            verbose=False, engine=eng)
        if rank == 0:
            d, attrs = out.files[s]
            flat = {'data/' + k: np.asarray(v) for k, v in d.items()}
            flat.update({'attr/' + k: np.asarray(v) for k, v in attrs.items()})
            np.savez(os.path.join(outdir, 'out.npz'), **flat)
        else:
            assert getattr(out, 'files', {}) == {}   # one file, written by rank 0
            assert 'angles' in data
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['g6_onthefly', 'g6b_onthefly_f32', 'g6c_onthefly_f32_c64',
                                  'g6d_onthefly_empty'])
@pytest.mark.parametrize('mode', ['pericentric', 'apocentric'])
def test_sharded_onthefly_matches_reference_golden(name, mode):
    """World 2 over ID ranges: rank 0's file equals the reference's (IDs, offsets,
    radii, positions, bulk velocities bit-exact; angle changes within 2 ulp, NaN
    where the reference has NaN), as the single-GPU test requires."""
    fix = load(name)
    _, meta = universe(fix)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, _free_port(), name, mode, d), nprocs=2, join=True,
                           start_method='spawn')
        f = np.load(os.path.join(d, 'out.npz'))
        got = {k: f[k] for k in f.files}
    keys = [k for k in fix.files if k.startswith(mode + '/')]
    want = {k.split('/', 1)[1]: fix[k] for k in keys}
    if 'attr_box_size' in want:
        assert np.array_equal(got.pop('attr/box_size'), want.pop('attr_box_size'))
    data = {k.split('/', 1)[1]: v for k, v in got.items() if k.startswith('data/')}
    assert sorted(data) == sorted(want), (sorted(data), sorted(want))
    for k, w in want.items():
        v = data[k]
        assert v.dtype == w.dtype and v.shape == w.shape, (k, v.dtype, w.dtype, v.shape, w.shape)
        if k == 'angles':
            nan = np.isnan(w)
            assert np.array_equal(np.isnan(v), nan), k
            cd = np.dtype(meta['gen'].get('dtype', 'float64'))
            ulp = np.spacing(np.abs(w[~nan]).astype(cd)).astype(np.float64)
            assert np.all(np.abs(v[~nan].astype(np.float64) - w[~nan]) <= 2 * ulp), k
        elif w.dtype.kind == 'f':
            assert np.array_equal(v, w, equal_nan=True), k
        else:
            assert np.array_equal(v, w), k


def _stream_worker(rank, world, port, outdir):
    import json
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from orbitanalysis_amd import track_orbits_onthefly as T
        from orbitanalysis_amd.engine import OrbitEngine
        from orbitanalysis_amd.savefile import MemorySavefile
        from orbitanalysis_amd.synthetic import PlummerSnapshots
        u = PlummerSnapshots(n_halos=3, n_per_halo=[900, 700, 500], n_snapshots=5, seed=41,
                             dt=0.5, box_size=40.0, region_returns=2)
        links = np.array([[0, 1, 2], [0, 1, 2]])
        loads = []

        class Loader:
            def __call__(self, s, pos, rad):
                loads.append(s)
                return u.load_snapshot_data(s, pos, rad)
        flat, calls = {}, {}
        for carry in ('1', '0'):
            os.environ['ORBIT_OTF_CARRY'] = carry
            T.clear_carry()
            loads.clear()
            out = MemorySavefile()
            load = Loader()
            eng = T.ShardedOnTheFly(OrbitEngine(mode='pericentric'))
            for s in (2, 3, 4):
                T.track_orbits(s, links, u.regions, load, out, mode='pericentric',
                               verbose=False, engine=eng)
            calls[carry] = list(loads)
            if rank == 0:
                for s, (d, _) in out.files.items():
                    flat.update({'%s/%d/%s' % (carry, s, k): np.asarray(v) for k, v in d.items()})
        T.clear_carry()
        with open(os.path.join(outdir, 'loads%d.json' % rank), 'w') as f:
            json.dump(calls, f)
        if rank == 0:
            np.savez(os.path.join(outdir, 'stream.npz'), **flat)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_onthefly_stream_carry_matches_fresh_calls():
    """World 2: a stream of calls s = 2, 3, 4 reuses each rank's shard and device frame
    state of the previous call's current snapshot (s-1 is loaded once per rank) and
    writes exactly the files of calls that load and frame both snapshots."""
    import json
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_stream_worker, args=(2, _free_port(), d), nprocs=2, join=True,
                           start_method='spawn')
        f = np.load(os.path.join(d, 'stream.npz'))
        got = {k: f[k] for k in f.files}
        calls = [json.load(open(os.path.join(d, 'loads%d.json' % r))) for r in range(2)]
    for c in calls:
        assert c['1'] == [2, 1, 3, 4], c['1']
        assert c['0'] == [2, 1, 3, 2, 4, 3], c['0']
    on = sorted(k[2:] for k in got if k.startswith('1/'))
    off = sorted(k[2:] for k in got if k.startswith('0/'))
    assert on == off and len(on) > 0
    for k in on:
        assert np.array_equal(got['1/' + k], got['0/' + k], equal_nan=True), k
