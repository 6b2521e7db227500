"""Multi-rank (world_size 2 and 3, gloo on CPU) tests of the ID-sharded driver.

Every rank runs the product driver ``track_orbits(..., engine=ShardedEngine(...))``
on the whole loader output and keeps the rows whose ID it owns; rank 0 writes the
savefile.  The per-rank compute is the oracle (tests/oracle_local.py), so these
tests pin the sharding, the bulk-velocity exchange, the apsis merge by (halo,
previous-block position) and the checkpoint gather against the reference's golden
vectors bit for bit.  The GPU variant (tests/test_gpu_parity.py) swaps in the HIP
engine."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from golden_util import load, universe, groups, assert_groups_equal, assert_same


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_major(snap, own, world, keep_rank=None):
    """The snapshot with every block's rows reordered rank-major (stable), or only the
    rows of ``keep_rank``: what a distributed loader hands each rank."""
    ids = np.asarray(snap['ids'])
    n = len(ids)
    starts = np.asarray(snap['region_offsets'], dtype=np.int64)
    ends = np.append(starts[1:], n)
    r = own(ids, world)
    rows, offs = [], []
    for a, b in zip(starts, ends):
        offs.append(sum(len(x) for x in rows))
        blk = np.arange(a, b)
        ranks = range(world) if keep_rank is None else [keep_rank]
        rows.append(np.concatenate([blk[r[a:b] == q] for q in ranks]) if b > a else blk)
    sel = np.concatenate(rows) if rows else np.zeros(0, np.int64)
    out = dict(snap)
    for k in ('ids', 'coordinates', 'velocities'):
        out[k] = np.asarray(snap[k])[sel]
    if isinstance(snap['masses'], np.ndarray):
        out['masses'] = snap['masses'][sel]
    out['region_offsets'] = np.array(offs, dtype=np.int64)
    return out


def _worker(rank, world, port, name, owner, outdir, local='oracle'):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from orbitanalysis_amd.sharding import ShardedEngine, HashOwner, IdRangeOwner
        from orbitanalysis_amd.savefile import MemorySavefile
        from orbitanalysis_amd.track_orbits import track_orbits
        from oracle_local import OracleLocal
        if isinstance(name, dict):                  # a synthetic universe, not a fixture
            from orbitanalysis_amd.synthetic import PlummerSnapshots
            u, meta = PlummerSnapshots(**name['gen']), {'run': name['run']}
        else:
            fix = load(name)
            u, meta = universe(fix)
        run = meta['run']
        own = HashOwner() if owner == 'hash' else IdRangeOwner(int(u.ids.min()),
                                                              int(u.ids.max()) + 1)
        presharded = owner == 'presharded'
        eng_owner = None if owner in ('default', 'presharded') else own   # default: fitted
        mode = run.get('mode', 'pericentric')
        if local == 'hip':                      # product per-rank compute (GPU tests)
            from orbitanalysis_amd.engine import OrbitEngine
            from orbitanalysis_amd.sharding import EngineLocal
            loc = EngineLocal(OrbitEngine(mode=mode))
        else:
            loc = OracleLocal(mode)
        eng = ShardedEngine(loc, owner=eng_owner, presharded=presharded)
        out = MemorySavefile()
        loader = u.load_snapshot_data
        if presharded:
            def loader(s, pos, rad):            # this rank's rows only
                return _rank_major(u.load_snapshot_data(s, pos, rad), own, world, rank)
        track_orbits(u.snapshot_numbers, u.main_branches(), u.regions, loader,
                     out, verbose=False, engine=eng, **run)
        layout = eng.checkpoint_layout()
        if presharded and run.get('checkpoint'):
            # a checkpoint in this rank-major layout resumes only in the same layout
            # (ADVICE r02): another layout's tag is refused before any angle is read
            s = u.snapshot_numbers[-1]
            h = u.main_branches()[-1]
            pos, rad, bulk = u.regions(s, h)
            snap = loader(s, pos, rad)
            n_global = len(u.load_snapshot_data(s, pos, rad)['ids'])
            ang = np.zeros(n_global, np.float16)
            H0 = np.float64(0.0)                # hubble_parameter returns float64
            ok = eng.prepare(snap, pos, bulk, H0, 0.0, np.arange(len(h)), False,
                             angles_in=ang, angles_layout=layout)
            assert ok.layout == layout
            try:
                eng.prepare(snap, pos, bulk, H0, 0.0, np.arange(len(h)), False, angles_in=ang,
                            angles_layout=layout.replace('world=%d' % world, 'world=9'))
                raise AssertionError('a checkpoint of another layout was accepted')
            except ValueError:
                pass
            try:
                eng.prepare(snap, pos, bulk, H0, 0.0, np.arange(len(h)), False,
                            angles_in=ang[:-1], angles_layout=layout)
                raise AssertionError('a short checkpoint was accepted')
            except ValueError:
                pass
        if rank == 0:
            flat = {'attr/mode': np.array(out.attrs['mode'])}
            if out.checkpoint_layout is not None:
                flat['checkpoint/layout'] = np.array(out.checkpoint_layout)
            for g, ds in out.groups.items():
                for k, v in ds.items():
                    flat[g + '/' + k] = v
            if out.checkpoint is not None:
                flat['checkpoint/angles'] = out.checkpoint
            np.savez(os.path.join(outdir, 'out.npz'), **flat)
        else:
            assert out.groups == {} and out.checkpoint is None     # only rank 0 writes
    finally:
        dist.destroy_process_group()


def run_sharded(name, world, owner='hash', local='oracle'):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), name, owner, d, local),
                           nprocs=world,
                           join=True, start_method='spawn')
        f = np.load(os.path.join(d, 'out.npz'))
        return {k: f[k] for k in f.files}


def _groups(flat):
    out = {}
    for k, v in flat.items():
        if k.startswith('snapshot_'):
            g, d = k.split('/')
            out.setdefault(g, {})[d] = v
    return out


@pytest.mark.parametrize('name,world,owner', [
    ('g2_overlap_birth_massarray', 2, 'hash'),    # overlapping regions, birth, mass-array bulk
    ('g3_apo_periodic', 2, 'range'),              # apocentric, periodic box, checkpoint
    ('g5_fp32_centre32', 3, 'hash'),              # float32 path, computed f32 bulk, 3 ranks
    ('g8_many_small_halos', 2, 'hash'),           # 40 halos, IDs offset past 2^40
    ('g11_edges', 2, 'range'),                    # gaps, death, empty blocks / snapshot
    ('g3_apo_periodic', 3, 'default'),            # IdRangeOwner fitted on the first snapshot
])
def test_sharded_driver_matches_reference(name, world, owner):
    fix = load(name)
    got = run_sharded(name, world, owner)
    assert str(got['attr/mode']) == str(fix['attr/mode'])
    assert_groups_equal(_groups(got), groups(fix))
    if 'checkpoint/angles' in fix.files:
        assert_same(got['checkpoint/angles'], fix['checkpoint/angles'], 'checkpoint')


def test_owners_partition_ids():
    from orbitanalysis_amd.sharding import HashOwner, IdRangeOwner
    ids = np.random.default_rng(0).permutation(100000).astype(np.int64) + (1 << 40)
    for world in (1, 2, 3, 8):
        for own in (HashOwner(), IdRangeOwner(1 << 40, (1 << 40) + 100000)):
            r = own(ids, world)
            assert r.min() >= 0 and r.max() < world
            counts = np.bincount(r, minlength=world)
            assert counts.min() > 0.8 * len(ids) / world       # balanced
            assert np.array_equal(own(ids, world), r)          # deterministic


def test_shard_snapshot_keeps_block_order():
    from orbitanalysis_amd.sharding import shard_snapshot
    rng = np.random.default_rng(1)
    n = 1000
    snap = {'ids': rng.permutation(n).astype(np.int64), 'coordinates': rng.normal(size=(n, 3)),
            'velocities': rng.normal(size=(n, 3)), 'masses': rng.uniform(size=n),
            'region_offsets': np.array([0, 100, 100, 550])}
    keep = rng.uniform(size=n) < 0.5
    sh, sel, st, cnt = shard_snapshot(snap, keep)
    assert np.array_equal(sh['ids'], snap['ids'][keep])
    assert np.array_equal(sh['masses'], snap['masses'][keep])
    assert cnt.sum() == keep.sum() and np.array_equal(st, sh['region_offsets'])
    bounds = [0, 100, 100, 550, n]
    for j in range(4):
        blk = keep[bounds[j]:bounds[j + 1]]
        assert cnt[j] == blk.sum()


@pytest.mark.parametrize('name', ['g4_hubble_catalogue', 'g5_fp32_catalogue32'])
def test_presharded_loader_matches_rank_major_oracle(name):
    """A distributed loader hands each rank its own ID range's rows (presharded=True):
    the global block is then the rank-ordered concatenation of the ranks' blocks, and
    the output must equal the oracle's on a loader returning blocks in that order."""
    from oracle import orbit_oracle as O
    from orbitanalysis_amd.sharding import IdRangeOwner
    fix = load(name)
    u, meta = universe(fix)
    world = 2
    own = IdRangeOwner(int(u.ids.min()), int(u.ids.max()) + 1)
    want = O.track_orbits(u.snapshot_numbers, u.main_branches(), u.regions,
                          lambda s, p, r: _rank_major(u.load_snapshot_data(s, p, r), own, world),
                          O.MemoryRecord(), **meta['run']).groups
    got = run_sharded(name, world, 'presharded')
    assert_groups_equal(_groups(got), want)


def test_presharded_checkpoint_is_global_rank_major():
    """With a presharded loader the checkpoint still holds the global snapshot's angles
    (rows of the rank-major blocks), as the single-process run writes them."""
    from oracle import orbit_oracle as O
    from orbitanalysis_amd.sharding import IdRangeOwner
    from orbitanalysis_amd.synthetic import PlummerSnapshots
    gen = dict(n_halos=6, n_per_halo=400, n_snapshots=4, seed=11, box_size=80.0,
               bulk='catalogue')
    run = dict(mode='pericentric', checkpoint=True)
    u = PlummerSnapshots(**gen)
    own = IdRangeOwner(int(u.ids.min()), int(u.ids.max()) + 1)
    rec = O.MemoryRecord()
    want = O.track_orbits(u.snapshot_numbers, u.main_branches(), u.regions,
                          lambda s, p, r: _rank_major(u.load_snapshot_data(s, p, r), own, 2),
                          rec, **run)
    got = run_sharded({'gen': gen, 'run': run}, 2, 'presharded')
    assert_groups_equal(_groups(got), want.groups)
    assert np.array_equal(got['checkpoint/angles'].view(np.uint16),
                          np.asarray(rec.checkpoint).view(np.uint16))
    # the checkpoint records its row layout (world size + the ranks' block counts)
    assert str(got['checkpoint/layout']).startswith('rank-major/world=2/blocks=')


def test_checkpoint_layout_guard():
    """Resuming a checkpoint in another row layout raises instead of silently
    assigning each particle another particle's angle."""
    from orbitanalysis_amd.sharding import check_layout
    check_layout(None, None)
    check_layout('rank-major/world=2/blocks=ab', 'rank-major/world=2/blocks=ab')
    for want, have in (('rank-major/world=2/blocks=ab', None),
                       (None, 'rank-major/world=2/blocks=ab'),
                       ('rank-major/world=2/blocks=ab', 'rank-major/world=3/blocks=ab')):
        with pytest.raises(ValueError):
            check_layout(want, have)


@pytest.mark.parametrize('world', [1, 2, 3, 8])
def test_stripes_partition_rows_at_block_bounds(world):
    from orbitanalysis_amd.sharding import stripe_halos, stripe_rows
    rng = np.random.default_rng(world)
    cnt = rng.integers(0, 500, 40)
    cnt[5:9] = 0
    starts = 7 + np.concatenate([[0], np.cumsum(cnt)[:-1]])
    n = int(starts[-1] + cnt[-1])
    hb = stripe_halos(starts, n, world)
    assert hb[0] == 0 and hb[-1] == len(starts) and np.all(np.diff(hb) >= 0)
    rows = [stripe_rows(starts, n, hb, r) for r in range(world)]
    assert rows[0][0] == 7 and rows[-1][1] == n
    assert all(rows[r][1] == rows[r + 1][0] for r in range(world - 1))
    for lo, hi in rows:                              # balanced to within one block
        assert abs((hi - lo) - (n - 7) / world) <= cnt.max()


class _Boom(RuntimeError):
    pass


def _fail_worker(rank, world, port, outdir):
    """Rank 0's loader raises at the fifth snapshot (the other rank is then already in
    that step's collectives); every rank must end."""
    import datetime
    import time
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    t_err = None
    status = 'ok'
    try:
        from orbitanalysis_amd.sharding import ShardedEngine
        from orbitanalysis_amd.savefile import MemorySavefile
        from orbitanalysis_amd.track_orbits import track_orbits
        from oracle_local import OracleLocal
        from orbitanalysis_amd.synthetic import PlummerSnapshots
        u = PlummerSnapshots(n_halos=3, n_per_halo=[300, 200, 150], n_snapshots=7, seed=9)
        bad = u.snapshot_numbers[4]

        def load(s, pos, rad):
            nonlocal t_err
            if rank == 0 and s == bad:
                t_err = time.time()
                raise _Boom('loader failed')
            return u.load_snapshot_data(s, pos, rad)
        out = MemorySavefile()
        try:
            track_orbits(u.snapshot_numbers, u.main_branches(), u.regions, load, out,
                         verbose=False, engine=ShardedEngine(OracleLocal('pericentric')))
        except _Boom:
            status = 'boom %.2f %d' % (time.time() - t_err, len(out.groups))
        except Exception as e:          # a peer that left mid-collective: also an exit
            status = 'peer %s' % type(e).__name__
    finally:
        with open(os.path.join(outdir, 'rank%d' % rank), 'w') as f:
            f.write(status)
        try:
            dist.destroy_process_group()
        except Exception:
            pass


def test_sharded_error_on_root_ends_every_rank():
    """an error on rank 0 alone while the ranks are pipelined must not start
    a collective record fetch in the error path (the other rank is already in the next
    step's collectives, and an unmatched gather would hang or mix them): rank 0 writes
    the groups whose records it already has, re-raises at once, and every rank ends."""
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.start_processes(_fail_worker, args=(2, _free_port(), d), nprocs=2,
                                 join=False, start_method='spawn')
        import time
        t_end = time.time() + 150
        while not ctx.join(timeout=5):
            assert time.time() < t_end, 'a rank hung after the root failed'
        st = {r: open(os.path.join(d, 'rank%d' % r)).read() for r in range(2)}
    assert st[0].startswith('boom'), st
    _, dt, n = st[0].split()
    assert float(dt) < 5.0, st                        # no wait on an unmatched collective
    assert int(n) == 2, st                            # groups 1-2 of 3 computed before it


def test_salvage_starts_no_collective_fetch():
    """The error path writes only groups whose records' fetch was already issued when
    fetching is a collective (ShardedEngine) or after an interrupt."""
    from orbitanalysis_amd import track_orbits as T
    from orbitanalysis_amd.savefile import MemorySavefile

    class Eng:
        world = 2

        def step_ready(self, res):
            return True

        def fetch_async(self, *a):
            raise AssertionError('collective fetch started in the error path')

    class Done:
        def query(self):
            return True

    class Fetched:
        done = Done()

        def wait(self):
            return np.array([0, 1]), np.array([7]), np.array([0.5], np.float16)

    out = MemorySavefile()
    out.initialize('pericentric', None)
    ga = (np.zeros((1, 3)), np.ones(1), np.zeros((1, 3)), np.array([3]), None, 4,
          'pericentric', False, None, False)
    gb = ga[:5] + (5,) + ga[6:]
    groups = [[None, np.int64, Fetched(), ga, {}], [None, np.int64, None, gb, {}]]
    T._salvage(groups, Eng(), out, new_fetches=False)
    assert sorted(out.groups) == ['snapshot_004'] and len(groups) == 1


def test_nccl_wire_dtypes():
    """every tensor the sharded paths move travels in a dtype torch's NCCL
    backend maps to an RCCL type (int16 angle bits, uint dtypes as bytes), and comes
    back bit-identical."""
    import torch
    from orbitanalysis_amd.sharding import to_wire, from_wire, NCCL_WIRE
    rng = np.random.default_rng(0)
    cases = [torch.from_numpy(rng.integers(-2 ** 15, 2 ** 15, 37).astype(np.int16)),
             torch.from_numpy(rng.integers(0, 2 ** 16, (37, 3)).astype(np.uint16)),
             torch.from_numpy(rng.integers(0, 2 ** 32, 37).astype(np.uint32)),
             torch.from_numpy(rng.integers(0, 2 ** 63, 37).astype(np.uint64)),
             torch.from_numpy(rng.normal(size=37).astype(np.float16)),
             torch.from_numpy(rng.integers(-2 ** 62, 2 ** 62, (37, 2))),
             torch.from_numpy(rng.normal(size=(37, 3))),
             torch.from_numpy(rng.uniform(size=37) < 0.5)]
    for x in cases:
        for cpu in (False, True):
            w, bv = to_wire(x, cpu)
            if not cpu:
                assert w.dtype in NCCL_WIRE, x.dtype
            assert w.shape[0] == x.shape[0]              # rows stay rows (uneven splits)
            y = from_wire(w.clone(), x.dtype, tuple(x.shape[1:]), bv)
            assert y.dtype == x.dtype and y.shape == x.shape
            assert torch.equal(y.view(torch.uint8) if x.dtype == torch.bool else y, x) or \
                np.array_equal(y.numpy().view(np.uint8), x.numpy().view(np.uint8))


def _stage_worker(rank, world, port, outdir, presharded):
    """Records of random per-rank runs through host_share.SharedRecordStage: rank 0's
    result must equal the sorted merge, and each rank stores only its own records."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from orbitanalysis_amd.host_share import SharedRecordStage
        rng = np.random.default_rng(123)                  # the same universe on every rank
        S = 23
        blk = rng.integers(0, 50, size=(world, S))        # rank r's rows of prev block h
        gstart = np.concatenate([[0], np.cumsum(blk.sum(0))])[:-1]
        before = np.cumsum(blk, 0) - blk
        n_rows = int(blk.sum())
        perm = rng.permutation(n_rows)
        stage = SharedRecordStage(None, rank, world)
        assert stage.probe(None, torch.device('cpu'), False)
        for it in range(3):
            ids_all, key_all, cnt = [], [], np.zeros((world, S), np.int64)
            mine_rows = []
            for r in range(world):
                for h in range(S):
                    if presharded:
                        pos = np.sort(rng.choice(blk[r, h], size=rng.integers(0, blk[r, h] + 1),
                                                 replace=False)) if blk[r, h] else np.zeros(0, np.int64)
                        key = gstart[h] + before[r, h] + pos
                    else:
                        # stripes: any rows of block h, owned by rank r if perm % W == r
                        rows_h = gstart[h] + np.arange(blk[:, h].sum())
                        own = rows_h[perm[rows_h] % world == r]
                        key = np.sort(own[rng.uniform(size=len(own)) < 0.4])
                    cnt[r, h] = len(key)
                    key_all.append(key)
                    ids_all.append(key * 7 + 3)
                    if r == rank:
                        mine_rows.append(key)
            mk = np.concatenate(mine_rows).astype(np.int64) if mine_rows else np.zeros(0, np.int64)
            offs = torch.from_numpy(np.concatenate([[0], np.cumsum(cnt[rank])]).astype(np.int64))
            a_ids = torch.from_numpy(mk * 7 + 3)
            a_ang = torch.from_numpy((mk % 30000).astype(np.int16))
            prof = {}
            f = stage.fetch(None, None, None, offs, a_ids, a_ang, len(mk),
                            torch.from_numpy(cnt[rank]), S, np.int64,
                            rows=None if presharded else torch.from_numpy(mk), n_rows=n_rows,
                            comm_dev=torch.device('cpu'), profile=prof)
            assert prof['own_records'] == len(mk) and prof['bytes_moved'] == 10 * len(mk)
            off, ids, ang = f.wait()
            if rank == 0:
                key = np.concatenate(key_all).astype(np.int64)
                order = np.argsort(key, kind='stable')
                assert np.array_equal(off, np.concatenate([[0], np.cumsum(cnt.sum(0))]))
                assert np.array_equal(ids, (key * 7 + 3)[order])
                assert np.array_equal(ang.view(np.int16), (key % 30000).astype(np.int16)[order])
            else:
                assert len(ids) == 0
            # the on-the-fly driver's lists: 4-byte IDs alone, and 4/8-byte values ranked
            # by their global rows (ShardedOnTheFly._stage_outputs)
            f = stage.fetch(None, None, None, offs, torch.from_numpy((mk * 5 + 1).astype(np.int32)),
                            None, len(mk), torch.from_numpy(cnt[rank]), S, np.uint32,
                            rows=torch.from_numpy(mk), n_rows=n_rows, comm_dev=torch.device('cpu'))
            off2, ids2, _ = f.wait()
            vdt = np.float32 if it % 2 else np.float64
            vals = stage.place_ranked(None, torch.from_numpy((mk * 0.5 + 0.25).astype(vdt)),
                                      torch.from_numpy(mk), n_rows, torch.device('cpu'))
            if rank == 0:
                assert np.array_equal(off2, off) and ids2.dtype == np.uint32
                assert np.array_equal(ids2, (key * 5 + 1).astype(np.uint32)[order])
                assert vals.dtype == vdt and np.array_equal(vals, (key * 0.5 + 0.25).astype(vdt)[order])
            else:
                assert vals is None and len(ids2) == 0
        stage.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,presharded', [(2, True), (3, True), (3, False)])
def test_shared_record_stage_places_every_rank(world, presharded):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_stage_worker, args=(world, _free_port(), d, presharded),
                           nprocs=world, join=True, start_method='spawn')
    left = [f for f in os.listdir('/dev/shm') if f.startswith('oa_rec_')] \
        if os.path.isdir('/dev/shm') else []
    assert not left, left                               # every slot file was unlinked
