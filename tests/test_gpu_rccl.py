"""The RCCL legs of the multi-GPU paths, on this one GPU (needs a GPU).

torch's ``nccl`` backend is RCCL on ROCm.  Two RCCL ranks need two GPUs, so the world-2
tests run gloo; this runs the same collectives at world 1 over RCCL, with the dtypes and
devices the sharded paths hand it:

* every wire dtype of ``sharding.to_wire`` (int16 angle bits, unsigned IDs as bytes,
  float16, bool) through ``all_to_all_single`` with explicit splits (``RowExchange``),
  ``all_gather_into_tensor`` and ``broadcast``, back bit-identical;
* the output stage (``host_share.SharedRecordStage``) with a CUDA comm device: the
  probe's int32 MIN all-reduce, the int64 count all-gather, the slot broadcast, the
  uint8 bitmap all-reduce of the row ranks; records (with and without angles), ranked
  f32 / f64 values and checkpoint angles stored through the registered mapping;
* ``ShardedEngine`` through ``track_orbits`` with its catalogue all-gather on RCCL
  (issued from a side stream, overlapping the previous step), equal to ``OrbitEngine``.
"""
import json
import os
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from test_sharding import _free_port

pytestmark = pytest.mark.gpu


def _worker(rank, port, outdir):
    import torch
    import torch.distributed as dist
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0,
                            world_size=1, device_id=dev)
    try:
        from orbitanalysis_amd import _native as N
        from orbitanalysis_amd.host_share import SharedRecordStage
        from orbitanalysis_amd.sharding import to_wire, from_wire, NCCL_WIRE
        lib = N.load(require_device=True)
        rng = np.random.default_rng(7)
        done = []
        # 1. wire dtypes through the three collectives the sharded paths use
        cases = [rng.integers(-2 ** 15, 2 ** 15, 37).astype(np.int16),
                 rng.integers(0, 2 ** 16, (37, 3)).astype(np.uint16),
                 rng.integers(0, 2 ** 32, 37).astype(np.uint32),
                 rng.integers(0, 2 ** 63, 37).astype(np.uint64) | np.uint64(1 << 63),
                 rng.normal(size=37).astype(np.float16),
                 rng.integers(-2 ** 62, 2 ** 62, (37, 2)),
                 rng.normal(size=(37, 3)),
                 rng.uniform(size=37) < 0.5]
        for a in cases:
            x = torch.from_numpy(a).to(dev)
            w, bv = to_wire(x, False)
            assert w.dtype in NCCL_WIRE, a.dtype
            n = int(w.shape[0])
            out = torch.empty_like(w)
            dist.all_to_all_single(out, w, [n], [n])
            gat = torch.empty_like(w)
            dist.all_gather_into_tensor(gat, w.contiguous())
            b = w.clone()
            dist.broadcast(b, src=0)
            for t in (out, gat, b):
                y = from_wire(t, x.dtype, tuple(x.shape[1:]), bv).cpu().numpy()
                assert y.dtype == a.dtype and np.array_equal(y.view(np.uint8), a.view(np.uint8)), \
                    a.dtype
            done.append(str(a.dtype))
        # 2. the output stage with its collectives on the device
        stage = SharedRecordStage(None, 0, 1)
        assert stage.probe(lib, dev, True)
        S, n_rows = 29, 5000
        rows = np.sort(rng.choice(n_rows, 1800, replace=False)).astype(np.int64)
        halo = np.sort(rng.integers(0, S, len(rows)))   # rows grouped by halo, in row order
        cnt = np.bincount(halo, minlength=S).astype(np.int64)
        ids = rows * 11 + 5
        ang = (rows % 30011).astype(np.int16)
        order = rng.permutation(len(rows))              # records arrive in any order
        t_ids, t_ang, t_rows = (torch.from_numpy(v[order]).to(dev) for v in (ids, ang, rows))
        offs = torch.from_numpy(np.concatenate([[0], np.cumsum(cnt)])).to(dev)
        for with_ang in (True, False):
            f = stage.fetch(lib, None, None, offs, t_ids, t_ang if with_ang else None,
                            len(rows), torch.from_numpy(cnt).to(dev), S, np.int64,
                            rows=t_rows, n_rows=n_rows, comm_dev=dev)
            off, got_ids, got_ang = f.wait()
            assert np.array_equal(off, np.concatenate([[0], np.cumsum(cnt)]))
            assert np.array_equal(got_ids, ids)
            if with_ang:
                assert np.array_equal(got_ang.view(np.int16), ang)
            del got_ids, got_ang
        # presharded: a count scan, the records in order
        f = stage.fetch(lib, None, None, offs, torch.from_numpy(ids.astype(np.int32)).to(dev),
                        torch.from_numpy(ang).to(dev), len(rows), torch.from_numpy(cnt).to(dev),
                        S, np.uint32, comm_dev=dev)
        _, got_ids, got_ang = f.wait()
        assert got_ids.dtype == np.uint32 and np.array_equal(got_ids, ids.astype(np.uint32))
        assert np.array_equal(got_ang.view(np.int16), ang)
        del got_ids, got_ang
        for vdt in (np.float32, np.float64):
            v = (rows * 0.25 - 3.0).astype(vdt)
            got = stage.place_ranked(lib, torch.from_numpy(v[order]).to(dev), t_rows, n_rows, dev)
            assert got.dtype == vdt and np.array_equal(got, v)
            del got
        a16 = rng.integers(0, 2 ** 16, n_rows).astype(np.uint16)
        perm = rng.permutation(n_rows)
        got = stage.place_rows(lib, torch.from_numpy(a16[perm].astype(np.int64)).to(dev),
                               torch.from_numpy(perm.astype(np.int64)).to(dev), n_rows, dev)
        assert np.array_equal(got.view(np.uint16), a16)
        del got
        stage.close()
        done.append('stage')
        # 3. ShardedEngine through track_orbits over RCCL: the catalogue all-gather from
        # its side stream, overlapping the previous step; the savefile equals a plain
        # OrbitEngine run's bit for bit
        from orbitanalysis_amd.engine import OrbitEngine
        from orbitanalysis_amd.savefile import MemorySavefile
        from orbitanalysis_amd.sharding import ShardedEngine, EngineLocal
        from orbitanalysis_amd.synthetic import PlummerSnapshots
        from orbitanalysis_amd.track_orbits import track_orbits
        kw = dict(n_halos=30, n_per_halo=[3000, 800, 12000] * 10, n_snapshots=5, seed=17,
                  dtype=np.float32, centre_dtype=np.float32, bulk='catalogue', box_size=300.0)
        outs = []
        for eng in (ShardedEngine(EngineLocal(OrbitEngine(mode='pericentric'))),
                    OrbitEngine(mode='pericentric')):
            u = PlummerSnapshots(**kw)
            out = MemorySavefile()
            track_orbits(u.snapshot_numbers, u.main_branches(), u.regions, u.load_snapshot_data,
                         out, mode='pericentric', verbose=False, engine=eng)
            outs.append(out)
        assert sorted(outs[0].groups) == sorted(outs[1].groups) and outs[0].groups
        for g in outs[1].groups:
            for k, w in outs[1].groups[g].items():
                assert np.array_equal(np.asarray(outs[0].groups[g][k]).view(np.uint8),
                                      np.asarray(w).view(np.uint8)), (g, k)
        done.append('sharded')
        with open(os.path.join(outdir, 'ok.json'), 'w') as fo:
            json.dump(done, fo)
    finally:
        dist.destroy_process_group()


def test_rccl_collectives_and_output_stage_world1():
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(_free_port(), d), nprocs=1, join=True,
                           start_method='spawn')
        done = json.load(open(os.path.join(d, 'ok.json')))
    assert 'stage' in done and 'sharded' in done and len(done) == 10, done
