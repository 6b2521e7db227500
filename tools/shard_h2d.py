"""Bytes each rank moves from the loader's host arrays to its device under the
reference's whole-snapshot loader contract (ShardedEngine, block-aligned stripes +
all-to-all), world 1..4 over gloo on the CPU, with the per-rank
compute stubbed by the test oracle (the byte count does not depend on it).

  python tools/shard_h2d.py [--out profiles/r03/shard_h2d.json]
"""
import argparse
import json
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

GEN = dict(n_halos=24, n_per_halo=4000, n_snapshots=3, seed=5, box_size=120.0,
           bulk='catalogue')


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from orbitanalysis_amd.sharding import ShardedEngine
        from orbitanalysis_amd.savefile import MemorySavefile
        from orbitanalysis_amd.synthetic import PlummerSnapshots
        from orbitanalysis_amd.track_orbits import track_orbits
        from oracle_local import OracleLocal
        u = PlummerSnapshots(**GEN)
        eng = ShardedEngine(OracleLocal('pericentric'))
        seen = []
        orig = eng.prepare

        def prepare(snapshot, *a, **k):
            sp = orig(snapshot, *a, **k)
            full = sum(np.asarray(snapshot[key]).nbytes for key in ('ids', 'coordinates',
                                                                    'velocities'))
            seen.append((sp.h2d_bytes, full))
            return sp
        eng.prepare = prepare
        track_orbits(u.snapshot_numbers, u.main_branches(), u.regions, u.load_snapshot_data,
                     MemorySavefile(), verbose=False, engine=eng)
        with open(os.path.join(outdir, 'r%d.json' % rank), 'w') as f:
            json.dump(seen, f)
    finally:
        dist.destroy_process_group()


def main():
    import tempfile
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default=os.path.join(ROOT, 'profiles', 'r03', 'shard_h2d.json'))
    args = ap.parse_args()
    res = []
    for world in (1, 2, 3, 4):
        with tempfile.TemporaryDirectory() as d:
            mp.start_processes(_worker, args=(world, _port(), d), nprocs=world, join=True,
                               start_method='spawn')
            per = [json.load(open(os.path.join(d, 'r%d.json' % r))) for r in range(world)]
        for s in range(len(per[0])):
            full = per[0][s][1]
            got = [p[s][0] for p in per]
            res.append(dict(world=world, snapshot=s, snapshot_bytes=full, h2d_bytes_per_rank=got,
                            max_fraction=max(got) / full, sum_fraction=sum(got) / full))
    out = dict(what='loader bytes each rank moves host -> device per snapshot (ids, '
                    'coordinates, velocities), whole-snapshot loader contract',
               universe=GEN, rows=res)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, 'w') as f:
        json.dump(out, f, indent=1)
    for r in res:
        print(r['world'], r['snapshot'], ['%.3f' % (g / r['snapshot_bytes']) for g in r['h2d_bytes_per_rank']])


if __name__ == '__main__':
    main()
