"""BASELINE.json configs[4] on one GPU: the track_orbits_onthefly stream with
double-buffered H2D.

Config 5 is 1e9 particles over 8 GPUs and 200 snapshots; one GPU's share is 1.25e8
particles per snapshot (float32, int64 IDs, periodic box).  Snapshots sit in pinned
host memory, as a loader that fills pinned buffers would leave them.  Each step
compares snapshot k with k-1:

  * a copy stream runs the H2D of snapshot k+1 (ids, coordinates, velocities:
    32 B/particle) into one of three device slots (k-1's IDs stay alive as the
    previous state);
  * the compute stream waits for snapshot k's copy, then runs the on-the-fly compare
    (`OnTheFly.run` with the carried frame state of k-1: one frame per snapshot) and
    brings every output to the host (apsis CSR, angle changes, entered/departed CSR).

value = particles of the timed steps / wall time (PCIe-inclusive, end to end).
Also reported: compute-only ms per step (HIP events), the H2D rate alone, and the
CPU oracle (the reference's per-call algorithm: both frames + compare) on a bounded
sample of halos with its apsis IDs checked against the GPU's.

  python tools/bench_onthefly.py [--particles 1.25e8] [--steps 6]

--sharded: the multi-GPU driver (``ShardedOnTheFly``) on every rank of a
torch.distributed run (``python -m torch.distributed.run ... tools/bench_onthefly.py
--sharded``; without a launcher, world 1).  Each rank holds only its block-aligned
stripe of every snapshot in pinned host memory (a striped reader's view of the
whole-snapshot contract), double-buffers that stripe's H2D on a copy stream, and runs
the sharded pipeline on it: owner all-to-all, join, apsis IDs and angle changes stored
by every rank into the shared host buffer, departed / entered rows merged on rank 0.  --particles is then the global snapshot size (configs[4]: 1e9 over 8
GPUs; the default 1.25e8 is one GPU's share).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PCIE_PEAK = 64.0        # GB/s per direction, PCIe 5.0 x16 (spec)


def log(*a):
    print('[bench_onthefly]', *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--particles', type=float, default=1.25e8)
    ap.add_argument('--per-halo', type=int, default=10000)
    ap.add_argument('--steps', type=int, default=12,
                    help='timed snapshots; the window also holds the last compare, which no '
                         'later H2D hides, so ms_per_step overstates the steady period by '
                         'about one compare / steps')
    ap.add_argument('--snapshots', type=int, default=3, help='distinct host snapshots (cycled)')
    ap.add_argument('--cpu-halos', type=int, default=150)
    ap.add_argument('--mode', default='pericentric')
    ap.add_argument('--sharded', action='store_true')
    ap.add_argument('--backend', default='nccl')
    ap.add_argument('--profile-host', action='store_true',
                    help='cProfile of the timed steps (host functions by own time, stderr)')
    args = ap.parse_args()
    import torch
    import orbitanalysis_amd  # noqa: F401
    from orbitanalysis_amd.synthetic_device import DevicePlummer
    from orbitanalysis_amd.track_orbits_onthefly import OnTheFly, ShardedOnTheFly
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0')) % max(torch.cuda.device_count(), 1)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    dist = None
    if args.sharded:
        import torch.distributed as dist
        if world == 1 and 'MASTER_ADDR' not in os.environ:
            os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT='29561')
        if args.backend == 'gloo':
            dist.init_process_group('gloo', rank=rank, world_size=world)
        else:
            dist.init_process_group('nccl', rank=rank, world_size=world, device_id=dev)
    nh = max(1, int(args.particles) // args.per_halo)
    gen = DevicePlummer(n_halos=nh, n_particles=int(args.particles), seed=5, device=dev)
    S = args.snapshots
    host, cats, offs, stripes, n_rows = [], [], [], [], []
    t0 = time.perf_counter()
    for s in range(S):
        sn = gen.snapshot(s)
        n = int(sn['ids'].numel())
        lo, hi = 0, n
        if args.sharded:
            from orbitanalysis_amd.sharding import my_stripe
            lo, hi = my_stripe(sn['region_offsets'], n)
        h = {k: torch.empty((hi - lo,) + tuple(sn[k].shape[1:]), dtype=sn[k].dtype,
                            pin_memory=True) for k in ('ids', 'coordinates', 'velocities')}
        for k in h:
            h[k].copy_(sn[k][lo:hi])
        host.append(h)
        stripes.append((lo, hi))
        n_rows.append(n)
        offs.append(np.asarray(sn['region_offsets'], dtype=np.int64))
        cats.append(gen.catalogue(s)[0])
        del sn
    box = gen.box
    del gen
    torch.cuda.empty_cache()
    log('setup %.1f s: %d halos, %s particles per snapshot, %d pinned host snapshots'
        % (time.perf_counter() - t0, nh, [int(h['ids'].numel()) for h in host], S))

    nmax = max(int(h['ids'].numel()) for h in host)
    slots = [{k: torch.empty((nmax,) + tuple(host[0][k].shape[1:]), dtype=host[0][k].dtype,
                             device=dev) for k in host[0]} for _ in range(3)]
    # the copy stream at high priority: HIP maps a process's streams onto
    # GPU_MAX_HW_QUEUES hardware queues (4 on the box) by priority, and with RCCL's
    # streams beside the compute stream a normal-priority copy stream shared the compute
    # stream's queue, so every sharded step waited behind the next snapshot's 70-ms H2D
    # (r04t: 127 ms per step; GPU_MAX_HW_QUEUES=8: 86 ms, r04v)
    cs = torch.cuda.Stream(device=dev, priority=-1)
    evs = {}

    def h2d(k):
        """Snapshot k (host copy k % S) into slot k % 3 on the copy stream."""
        src, dst = host[k % S], slots[k % 3]
        with torch.cuda.stream(cs):
            for key in src:
                n = src[key].shape[0]
                dst[key][:n].copy_(src[key], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cs)
        evs[k] = ev

    def snap_dict(k):
        m = int(host[k % S]['ids'].numel())
        n = n_rows[k % S]
        d = {key: slots[k % 3][key][:m] for key in host[0]}
        d.update(masses=1.0, box_size=box)
        if args.sharded:
            from orbitanalysis_amd.sharding import STRIPE
            d[STRIPE], d['n_rows'] = stripes[k % S], n
        o = offs[k % S]
        sl = np.stack([o, np.append(o[1:], n)], axis=1)
        return d, sl

    if args.sharded:
        from orbitanalysis_amd.engine import OrbitEngine
        otf = ShardedOnTheFly(OrbitEngine(mode=args.mode, device=dev))
    else:
        otf = OnTheFly(mode=args.mode)
    # H2D alone (copy-engine rate) on one snapshot, warm (the first copy into fresh
    # device memory is slower)
    for _ in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        h2d(0)
        evs[0].synchronize()
        h2d_s = time.perf_counter() - t
    h2d_bytes = sum(v.numel() * v.element_size() for v in host[0].values())
    log('H2D alone: %.1f ms for %.2f GB (%.1f GB/s)' % (h2d_s * 1e3, h2d_bytes / 1e9,
                                                     h2d_bytes / h2d_s / 1e9))
    # snapshot 0: frame only (its state is carried into step 1)
    h2d(1)
    torch.cuda.current_stream().wait_event(evs[0])
    d0, sl0 = snap_dict(0)
    if args.sharded:
        carried = None                          # step 1 frames snapshot 0 itself
    else:
        pp = otf._prepare(d0, sl0, cats[0], False)
        otf.eng.launch(pp, None)
        from orbitanalysis_amd.engine import SnapshotState
        from orbitanalysis_amd import _native as N
        bulk0 = pp.halos.cpu().numpy().view(N.HALO_DTYPE)['bulk'].astype(pp.plan.bulk)
        carried = (SnapshotState(ids=pp.snap['ids'], rhat=pp.rhat, meta=pp.meta,
                                 starts=pp.starts, counts=pp.counts, exists=np.arange(nh),
                                 plan=pp.plan), bulk0)
    total_steps = 1 + args.steps              # 1 warm-up step
    if args.sharded:                          # unperturbed per-phase host / stream times
        otf.timings, otf.timing_sync = {}, False
    comp_ms, units, outs = [], 0, None
    t_start = None
    prof = None
    for k in range(1, total_steps + 1):
        if k == 2 and args.profile_host:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        if k == 1:
            # the clock starts before snapshot 2's H2D is issued: the window holds the
            # H2Ds of every timed snapshot (2 .. total_steps), so a PCIe-bound stream
            # cannot read faster than its copies (starting at k == 2 left
            # snapshot 2's H2D outside, steps - 1 copies for steps snapshots)
            torch.cuda.synchronize()
            if dist is not None:
                dist.barrier()
            t_start = time.perf_counter()
        if k + 1 <= total_steps:
            h2d(k + 1)                         # overlaps this step's compare
        torch.cuda.current_stream().wait_event(evs[k])
        dk, slk = snap_dict(k)
        dp, slp = snap_dict(k - 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if carried is None:                    # sharded, first step: both snapshots
            outs = otf.run([dk, dp], [slk, slp], [cats[k % S], cats[(k - 1) % S]])
        else:
            outs = otf.run([dk, None], [slk, slp], [cats[k % S], cats[(k - 1) % S]],
                           carried=carried)
        e1.record()
        carried = otf.carry
        if k >= 2:
            e1.synchronize()
            comp_ms.append(e0.elapsed_time(e1))
            units += n_rows[k % S]
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_start
    if prof is not None:
        prof.disable()
        import io
        import pstats
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats('tottime').print_stats(30)
        log('host profile (%d timed steps):\n%s' % (total_steps - 1, buf.getvalue()))
    phases = None
    if args.sharded:
        # the timed steps' host and stream time per phase (medians), then an instrumented
        # pass: per-phase wall times of the sharded run (each boundary synchronises)
        phases = {p: float(np.median(v[1:])) for p, v in otf.timings.items() if len(v) > 1}
        otf.timings, otf.timing_sync = {}, True
        for k in range(total_steps + 1, total_steps + 3):
            h2d(k)
            torch.cuda.current_stream().wait_event(evs[k])
            dk, slk = snap_dict(k)
            _, slp = snap_dict(k - 1)
            otf.run([dk, None], [slk, slp], [cats[k % S], cats[(k - 1) % S]], carried=otf.carry)
        phases.update({p: float(np.median(v)) for p, v in otf.timings.items()})
        otf.timings = None
        log('sharded phases (ms, median of 2): %s' % phases)
    if dist is not None:
        nccl = dist.get_backend() == 'nccl'
        t = torch.tensor([wall], dtype=torch.float64, device=dev if nccl else 'cpu')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        if rank != 0:
            dist.destroy_process_group()
            return
    n_apsis = int(outs['apsis_offsets'][-1])

    # CPU oracle: the reference per-call algorithm (frames of both snapshots + compare)
    # on the first cpu_halos halos of the last step's pair
    from oracle import orbit_oracle as O
    k = total_steps
    ch = min(args.cpu_halos, nh)

    def host_snap(j):
        o = offs[j % S]
        e = int(o[ch]) if ch < nh else int(host[j % S]['ids'].numel())
        d = {key: host[j % S][key][:e].numpy() for key in host[0]}
        d.update(masses=1.0, box_size=box)
        sl = np.stack([o[:ch], np.append(o[1:ch], e)], axis=1)
        return d, sl
    hc, slc = host_snap(k)
    hp, slp = host_snap(k - 1)
    t = time.perf_counter()
    rc, vc, _ = O.onthefly_region_frame(hc, slc, cats[k % S][:ch])
    rp, vp, _ = O.onthefly_region_frame(hp, slp, cats[(k - 1) % S][:ch])
    want = O.onthefly_compare(hc['ids'], hp['ids'], vc, vp, rc, rp, slc, slp, args.mode)
    cdt = time.perf_counter() - t
    tag = args.mode[:8] + 'er'
    got = outs['apsis_ids'][:int(outs['apsis_offsets'][ch])]
    ok = bool(np.array_equal(want[tag + '_ids'], got))
    cpu_units = int(slc[-1][1])

    res = {
        'metric': 'particle-snapshots/s (track_orbits_onthefly stream, H2D inclusive)',
        'value': units / wall, 'unit': 'particle-snapshots/s', 'n_gpus': world,
        'driver': 'ShardedOnTheFly (stripe H2D + owner all-to-all + shared-buffer output stage)'
                  if args.sharded else 'OnTheFly (single GPU)',
        'steps': args.steps, 'warmup': 1, 'ms_per_step': wall / args.steps * 1e3,
        'timed_window': 'from before the H2D of the first timed snapshot (2) is issued to '
                        'the end of the last step: %d H2Ds and %d compares (the warm-up '
                        'compare of snapshot 1 overlaps snapshot 2\'s H2D)'
                        % (args.steps, args.steps + 1),
        'h2d_alone_ms': h2d_s * 1e3,
        'higher_is_better': True, 'dtype': 'f32', 'data': 'synthetic Plummer spheres, pinned host',
        'config': {'workload': 'BASELINE configs[4] per-GPU share: %d particles/snapshot, %d '
                               'halos, f32, box, double-buffered H2D on a copy stream, frame '
                               'state carried between snapshots' % (units // args.steps, nh)},
        'compute_ms_per_step': float(np.mean(comp_ms)),
        'compute_only_rate': units / (sum(comp_ms) * 1e-3),
        'sharded_phases_ms': phases,
        'apsis_last_step': n_apsis,
        'roofline': {'bound': 'pcie', 'achieved': h2d_bytes / h2d_s / 1e9, 'peak': PCIE_PEAK,
                     'unit': 'GB/s', 'frac': h2d_bytes / h2d_s / 1e9 / PCIE_PEAK,
                     'traffic': h2d_bytes, 'note': 'H2D of one snapshot alone, pinned host'},
        'cpu_baseline': {'value': cpu_units / cdt, 'unit': 'particle-snapshots/s', 'cores': 1,
                         'kind': 'port', 'sample': '%d of %d halos of the last pair, both '
                         'frames + compare, %.1f s; apsis IDs identical to the GPU: %s'
                         % (ch, nh, cdt, ok)},
    }
    print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
