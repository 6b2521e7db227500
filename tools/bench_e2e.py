"""End to end through the public batch API (SURVEY.md §8(d) "end-to-end"): BASELINE
configs[2] shape (1e8 f32 particles in 1e4 halos per snapshot) fed by a host NumPy
loader to ``orbitanalysis_amd.track_orbits.track_orbits``, the reference's call
(track_orbits.py:9-244), with a savefile that counts and drops each group's arrays (the HDF5
write is excluded, as §8(d) says).

Each snapshot pays what a drop-in user pays: the loader's host arrays go to the
device (ids, coordinates, velocities: 32 B/particle, pageable NumPy memory), the
per-snapshot plan is built on the host, the kernels run, and the apsis CSR comes
back and is written to the savefile.  The loader hands back prebuilt arrays (S
distinct snapshots, cycled), so its own cost is ~0.

value = particles of the timed snapshots / wall time of those snapshots (the first
snapshot, which only frames, and one warm-up comparison are excluded).

--device-loader: the loader returns torch device tensors (snapshots resident in HBM,
as a GPU-side reader or simulation would hand them over), so no H2D; what remains is
the driver's own per-snapshot cost: the host plan (OrbitEngine.prepare), the kernels,
the status read, the D2H of the apsis CSR and the savefile write.  The per-phase
host times are reported beside the wall time.

  python tools/bench_e2e.py [--particles 1e8] [--halos 10000] [--snapshots 6] [--device-loader]

--sharded (under torch.distributed.run, one rank per GPU; --backend gloo rehearses
several ranks on one GPU): the multi-GPU drop-in, track_orbits(..., engine=
ShardedEngine(EngineLocal(OrbitEngine()))).  --contract presharded (default): each
rank's loader returns its own ID range (--particles per rank, --scaling weak; or
--particles in total, --scaling strong); --contract whole: every rank is handed the
whole snapshot (device tensors) and the engine stripes + exchanges it.  Per-phase
host times of the sharded engine (prepare = shard + plan, launch, settle, the records'
gather to rank 0 and its wait) are reported per snapshot.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print('[bench_e2e]', *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--particles', type=float, default=1e8)
    ap.add_argument('--halos', type=int, default=10000)
    ap.add_argument('--snapshots', type=int, default=14, help='snapshots in the run')
    ap.add_argument('--warmup', type=int, default=4,
                    help='untimed leading snapshots (the first pinned host blocks are '
                         'page-locked then; later snapshots reuse them)')
    ap.add_argument('--distinct', type=int, default=3, help='distinct host snapshots (cycled)')
    ap.add_argument('--mode', default='pericentric')
    ap.add_argument('--device-loader', action='store_true',
                    help='the loader returns device tensors (no H2D)')
    ap.add_argument('--sharded', action='store_true', help='ShardedEngine over the ranks')
    ap.add_argument('--contract', default='presharded', choices=['presharded', 'whole'])
    ap.add_argument('--scaling', default='weak', choices=['weak', 'strong'])
    ap.add_argument('--backend', default='nccl')
    ap.add_argument('--profile-host', action='store_true',
                    help='cProfile of the driver (host functions by own time, to stderr)')
    ap.add_argument('--timeline', action='store_true',
                    help='GPU timeline per snapshot: k_step start/end and the records\' D2H '
                         '(timing events; the events themselves cost a few us)')
    args = ap.parse_args()
    import torch
    import orbitanalysis_amd  # noqa: F401
    from orbitanalysis_amd.synthetic_device import DevicePlummer
    from orbitanalysis_amd.track_orbits import track_orbits
    from orbitanalysis_amd.savefile import MemorySavefile
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0')) % max(torch.cuda.device_count(), 1)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    if args.sharded:
        import torch.distributed as dist
        if args.backend == 'gloo':
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=dev)
        args.device_loader = True
    per_rank = int(args.particles) if (args.scaling == 'weak' or not args.sharded) else \
        int(args.particles) // world
    if args.sharded and args.contract == 'presharded':
        gen = DevicePlummer(n_halos=args.halos, n_particles=per_rank, seed=0, rank=rank,
                            world=world, device=dev)
    else:
        gen = DevicePlummer(n_halos=args.halos, n_particles=per_rank, seed=0, device=dev)
    S = args.distinct
    host, cats = [], []
    t0 = time.perf_counter()
    for s in range(S):
        sn = gen.snapshot(s)
        if args.device_loader:
            h = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in sn.items()}
        else:
            h = {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in sn.items()}
        host.append(h)
        cats.append(gen.catalogue(s))
        del sn
    del gen
    torch.cuda.empty_cache()
    # per-phase host time of the driver's engine calls (tool-side instrumentation)
    from orbitanalysis_amd.engine import OrbitEngine
    phase = {'prepare': [], 'launch': [], 'settle': [], 'fetch': [], 'fetch_async': [],
             'wait': [], 'save': []}
    if args.sharded:
        phase.update({'shard_prepare': [], 'shard_settle': [], 'shard_fetch_async': [],
                      'shard_wait': []})

    def timed(name, fn):
        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            phase[name].append(time.perf_counter() - t)
            return r
        return w
    OrbitEngine.prepare = timed('prepare', OrbitEngine.prepare)
    kern_ev, host_launch = [], []
    if args.timeline:
        _launch = OrbitEngine.launch

        def launch_tl(self, pr, ws, prev=None, stream=None, step_events=None):
            if self.copy_events is None:
                self.copy_events = []
            if pr.compare and step_events is None:
                step_events = (torch.cuda.Event(enable_timing=True),
                               torch.cuda.Event(enable_timing=True))
                kern_ev.append(step_events)
                host_launch.append(time.perf_counter())
            return _launch(self, pr, ws, prev, stream, step_events)
        OrbitEngine.launch = launch_tl
    OrbitEngine.launch = timed('launch', OrbitEngine.launch)
    OrbitEngine.fetch = timed('fetch', OrbitEngine.fetch)
    OrbitEngine.fetch_async = timed('fetch_async', OrbitEngine.fetch_async)
    from orbitanalysis_amd import engine as E, track_orbits as TO
    _settle = OrbitEngine.settle

    def settle(self, res=None):
        # only the calls that wait (a pending step), not the no-op checks
        r = res if res is not None else self._pending
        if r is None or getattr(r, 'pending', None) is None:
            return _settle(self, res)
        t = time.perf_counter()
        out = _settle(self, res)
        phase['settle'].append(time.perf_counter() - t)
        return out
    OrbitEngine.settle = settle
    E.PendingFetch.wait = timed('wait', E.PendingFetch.wait)
    TO.save_to_file = timed('save', TO.save_to_file)
    engine = None
    if args.sharded:
        from orbitanalysis_amd import sharding as SH
        SH.ShardedEngine.prepare = timed('shard_prepare', SH.ShardedEngine.prepare)
        SH.ShardedEngine.fetch_async = timed('shard_fetch_async', SH.ShardedEngine.fetch_async)
        SH.ShardedFetch.wait = timed('shard_wait', SH.ShardedFetch.wait)
        _ssettle = SH.EngineLocal.settle

        def ssettle(self, lp):
            t = time.perf_counter()
            out = _ssettle(self, lp)
            phase['shard_settle'].append(time.perf_counter() - t)
            return out
        SH.EngineLocal.settle = ssettle
        engine = SH.ShardedEngine(SH.EngineLocal(OrbitEngine(mode=args.mode, device=dev)),
                                  presharded=args.contract == 'presharded')
        # rank 0's record placement timed (synchronised) per fetch: bytes per record
        # and merge ms in the output line
        engine.profile_fetch = True
        fstats = []
        _fa = SH.ShardedEngine.fetch_async

        def fa(self, res, ids_dtype):
            f = _fa(self, res, ids_dtype)
            if self.fetch_stats is not None:
                fstats.append(dict(self.fetch_stats))
            return f
        SH.ShardedEngine.fetch_async = fa
    if engine is None:
        engine = OrbitEngine(mode=args.mode, device=dev)
    log('setup %.1f s: %d host snapshots of %s particles' % (
        time.perf_counter() - t0, S, [len(h['ids']) for h in host]))

    stamps = {}

    def regions(snapshot_number, halo_ids):
        c, r, bv = cats[snapshot_number % S]
        return c[halo_ids], r[halo_ids], bv[halo_ids]

    def load_snapshot_data(snapshot_number, positions, radii):
        stamps[snapshot_number] = time.perf_counter()
        return dict(host[snapshot_number % S])

    class CountingSink(MemorySavefile):
        """The savefile interface with the write left out (SURVEY §8(d) excludes the
        HDF5 write): each group's arrays are counted and dropped, as an HDF5 writer
        drops them once written (nothing accumulates in host memory)."""

        def write_group(self, name, datasets):
            self.groups[name] = {k: int(np.asarray(v).size) for k, v in datasets.items()}

    n = args.snapshots
    sink = CountingSink()
    branches = np.tile(np.arange(args.halos), (n, 1))
    t_start = time.perf_counter()
    if args.sharded:
        dist.barrier()
    prof = None
    if args.profile_host:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    track_orbits(np.arange(n), branches, regions, load_snapshot_data, sink, mode=args.mode,
                 verbose=False, engine=engine)
    torch.cuda.synchronize()
    if prof is not None:
        prof.disable()
        import io
        import pstats
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats('tottime').print_stats(30)
        log('host profile (whole run, %d snapshots):\n%s' % (n, buf.getvalue()))
    t_end = time.perf_counter()
    # timed: snapshots W .. n-1 (from the loader call of snapshot W to the end)
    W = args.warmup
    timed = list(range(W, n))
    wall = t_end - stamps[W]
    units = sum(len(host[s % S]['ids']) for s in timed)
    if args.sharded:
        # whole-job rate: the slowest rank's wall, the units of every rank
        t = torch.tensor([wall, float(units if args.contract == 'presharded' or rank == 0 else 0)],
                         dtype=torch.float64, device=dev if args.backend != 'gloo' else 'cpu')
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        wall, units = float(t[0]), float(t[1])
        if rank != 0:
            dist.destroy_process_group()
            return
    n_apsis = sum(g['pericenter_IDs' if args.mode == 'pericentric' else 'apocenter_IDs']
                  for g in sink.groups.values())
    per = [stamps[s + 1] - stamps[s] for s in range(W, n - 1)] + [t_end - stamps[n - 1]]
    b = 32.0 * units / len(timed)
    res = {
        'metric': 'particle-snapshots/s (track_orbits end to end, %s loader)'
                  % ('device-tensor' if args.device_loader else 'host NumPy'),
        'value': units / wall, 'unit': 'particle-snapshots/s', 'n_gpus': world,
        'steps': len(timed), 'warmup': W, 'ms_per_step': wall / len(timed) * 1e3,
        'higher_is_better': True, 'dtype': 'f32', 'data': 'synthetic Plummer spheres, %s' % (
                    'device tensors' if args.device_loader else 'host NumPy'),
        'config': {'workload': 'BASELINE configs[2] shape: %d particles/snapshot, %d halos, f32, '
                               'public track_orbits, in-memory savefile' % (units // len(timed),
                                                                          args.halos),
                   'engine': ('ShardedEngine x%d (%s loader, %s scaling, %s)'
                              % (world, args.contract, args.scaling, args.backend))
                   if args.sharded else 'OrbitEngine'},
        'ms_per_snapshot': [round(p * 1e3, 2) for p in per],
        'ms_per_snapshot_median': round(float(np.median(per)) * 1e3, 3),
        # without the first timed interval (pinned blocks for the heavier pairs are
        # still being allocated) and the last (the drain: the final records' D2H)
        'ms_per_snapshot_steady_mean': round(float(np.mean(per[1:-1])) * 1e3, 3)
        if len(per) > 2 else None,
        'h2d_bytes_per_snapshot': 0.0 if args.device_loader else b,
        'host_ms_per_snapshot': {k: round(float(np.mean(v[W:])) * 1e3, 3) if len(v) > W else None
                                 for k, v in phase.items()},
        'host_ms_calls': {k: [round(x * 1e3, 2) for x in v] for k, v in phase.items() if v},
        'apsis_records': n_apsis,
        'total_wall_s': t_end - t_start,
    }
    if args.sharded and fstats:
        def med(k):
            v = [f[k] for f in fstats[W:] if k in f] or [f[k] for f in fstats if k in f]
            return float(np.median(v)) if v else None
        res['records_output'] = {
            'layout': fstats[-1]['layout'],
            'bytes_per_record': fstats[-1]['bytes_per_record'],
            'records_per_snapshot_median': med('records'),
            'own_records_per_snapshot_median': med('own_records'),
            'bytes_stored_by_this_rank_median': med('bytes_moved'),
            'place_ms_median': med('place_ms'),
            'note': 'every rank computes its records\' final positions (count scan: '
                    'presharded; bitmap rank over global previous rows: stripes) and stores '
                    'them into the shared page-locked host buffer (host_share); place_ms: '
                    'this rank\'s position computation + stores, synchronised'}
    if args.timeline and kern_ev:
        # GPU timeline relative to the first timed compare step's start: each step's
        # kernel window, the gap before it, and each records D2H window and its rate
        eng_obj = engine.local.engine if args.sharded else engine
        cev = eng_obj.copy_events or []
        t0e = kern_ev[0][0]
        ks = [(t0e.elapsed_time(a), t0e.elapsed_time(b)) for a, b in kern_ev]
        cs = [(t0e.elapsed_time(a), t0e.elapsed_time(b), n) for a, b, n in cev]
        res['timeline'] = {
            'kernel_ms': [round(b - a, 3) for a, b in ks],
            'gap_before_kernel_ms': [None] + [round(ks[i][0] - ks[i - 1][1], 3)
                                             for i in range(1, len(ks))],
            'd2h_ms': [round(b - a, 3) for a, b, _ in cs],
            'd2h_gbs': [round(n * 10 / max(b - a, 1e-6) / 1e6, 1) for a, b, n in cs],
            'd2h_start_after_kernel_end_ms': [round(cs[i][0] - ks[i][1], 3)
                                             for i in range(min(len(cs), len(ks)))],
        }
    print(json.dumps(res), flush=True)
    if args.sharded:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
