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


@pytest.mark.parametrize('ids_dtype', [np.int64, np.uint64, np.uint32])
def test_merge_onthefly_restores_single_rank_order(ids_dtype):
    """The root's merge of every rank's records (rank-major concatenation of each
    rank's rows, each rank's rows in its own order) restores the single-process
    order: apsis records and angle changes by global previous row; departed and
    entered IDs sorted unique per halo (unsigned IDs in unsigned order, repeats
    dropped), except a halo without a progenitor block, whose entered IDs keep
    global current-row order."""
    import torch
    from orbitanalysis_amd.track_orbits_onthefly import merge_onthefly, id_order_key
    rng = np.random.default_rng(3)
    nh, world = 7, 3
    dt = np.dtype(ids_dtype)
    pcnt = rng.integers(0, 60, nh)
    pcnt[2] = 0
    p_has = pcnt > 0
    pstart = np.concatenate([[0], np.cumsum(pcnt)[:-1]])
    n_prev = int(pcnt.sum())
    big = (1 << 63) + 5 if dt == np.uint64 else (1 << 31) + 5 if dt == np.uint32 else 1 << 40
    pool = rng.permutation(10 ** 5)[:n_prev + 400].astype(dt) + dt.type(big)
    i64 = lambda a: torch.from_numpy(np.asarray(a).astype(dt).view(np.int64) if dt.itemsize == 8  # noqa: E731
                                     else np.asarray(a).astype(np.int64))
    # apsis / angles: a subset of previous rows
    arow = np.sort(rng.choice(n_prev, n_prev // 3, replace=False))
    mrow = np.sort(rng.choice(n_prev, n_prev // 2, replace=False))
    aval = rng.random(len(mrow)).astype(np.float32)
    # departed: per-halo IDs in any order (one duplicate row to drop)
    dh = np.repeat(np.arange(nh), rng.integers(0, 5, nh))
    did = pool[n_prev:n_prev + len(dh)]
    dh, did = np.append(dh, dh[:1]), np.append(did, did[:1])
    # entered: halos with a progenitor sorted, the others in current-row order
    eh = np.repeat(np.arange(nh), rng.integers(0, 6, nh))
    eid = pool[n_prev + 100:n_prev + 100 + len(eh)]
    eg = rng.permutation(10 ** 4)[:len(eh)].astype(np.int64)
    owner = {k: rng.integers(0, world, len(v)) for k, v in
             dict(a=arow, m=mrow, d=dh, e=eh).items()}

    def rank_major(key, *cols):
        o = np.argsort(owner[key], kind='stable')       # each rank keeps its own order
        return [np.asarray(c)[o] for c in cols]
    a_r, = rank_major('a', arow)
    m_r, v_r = rank_major('m', mrow, aval)
    d_h, d_i = rank_major('d', dh, did)
    e_h, e_i, e_g = rank_major('e', eh, eid, eg)
    parts = dict(apsis=torch.stack([torch.from_numpy(a_r), i64(pool[a_r])], 1),
                 angle_g=torch.from_numpy(m_r), angle_v=torch.from_numpy(v_r),
                 departed=torch.stack([torch.from_numpy(d_h), i64(d_i)], 1),
                 entered=torch.stack([torch.from_numpy(e_h), i64(e_i), torch.from_numpy(e_g)], 1))
    got = merge_onthefly(parts, nh, pstart, p_has, dt)
    halo_of = np.repeat(np.arange(nh), pcnt)
    assert np.array_equal(got['apsis_ids'], pool[arow]) and got['apsis_ids'].dtype == dt
    assert np.array_equal(got['apsis_offsets'],
                          np.concatenate([[0], np.cumsum(np.bincount(halo_of[arow], minlength=nh))]))
    assert np.array_equal(got['angles'], aval)
    # the same with the previous row count given (the counting placement's bound)
    again = merge_onthefly(parts, nh, pstart, p_has, dt, n_prev=n_prev)
    assert np.array_equal(again['angles'], aval)
    want_d = [np.unique(did[dh == j]) for j in range(nh)]
    assert np.array_equal(got['departed_ids'], np.concatenate(want_d))
    assert np.array_equal(got['departed_offsets'], np.cumsum([0] + [len(x) for x in want_d]))
    want_e = [np.unique(eid[eh == j]) if p_has[j] else eid[eh == j][np.argsort(eg[eh == j])]
              for j in range(nh)]
    assert np.array_equal(got['entered_ids'], np.concatenate(want_e).astype(dt))
    assert np.array_equal(got['entered_offsets'], np.cumsum([0] + [len(x) for x in want_e]))
    # the order key really is the unsigned order
    k = id_order_key(i64(pool[:50]), dt)
    assert np.array_equal(np.argsort(k.numpy(), kind='stable'), np.argsort(pool[:50], kind='stable'))


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
