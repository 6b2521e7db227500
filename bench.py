#!/usr/bin/env python
"""bench.py — particle-snapshots/s of the per-snapshot orbit-tagging hot path.

Workload (BASELINE.json configs[2], the metric's 1-GPU configuration): 1e8
particles per GPU in 1e4 halo region blocks, float32 coordinates/velocities with
float32 catalogue centres and bulk velocities, int64 IDs, periodic box, Hubble term
on.  A step = one snapshot of track_orbits' per-snapshot body on device-resident
inputs: fused frame + ID join + sign flip + angles (oa_step) and the apsis output
assembly (oa_compact); the host plan of each snapshot is built before the timing.
Multi-GPU: the product's ShardedEngine, particles sharded by ID range (every rank
generates its own range: presharded), one RCCL all-gather of the halo catalogue rows
per snapshot inside the timed step; --scaling weak (1e8 per GPU, default) or strong
(1e8 in total, configs[3]).

Prints ONE JSON line on rank 0 (contract in the task statement): value =
particle-snapshots/s over all ranks; roofline = algorithmic bytes of the oa_step
kernel / its HIP-event duration vs 8 TB/s; cpu_baseline = the CPU oracle (NumPy
restatement of the reference path, 1 core) timed on a bounded sample of the same
workload, with its apsis IDs checked against the GPU's for that sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'particle-snapshots/sec (peri/apo tagging), 1e8 particles, 1/2/4/8 GPUs'
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print('[bench]', *a, file=sys.stderr, flush=True)


def step_bytes(pr, n_prev, n_apsis, reads_only=False):
    """Algorithmic HBM bytes of one oa_step launch: every
    current particle reads id + x + v and writes its record; every previous
    particle reads id + record; every apsis writes id + f16 angle.  ``reads_only``:
    the bytes read."""
    p = pr.plan
    cur = p.ids.itemsize + 3 * p.coord.itemsize + 3 * p.vel.itemsize
    if p.mass is not None:
        cur += p.mass.itemsize
    prev = p.ids.itemsize + p.state_bytes
    if reads_only:
        return pr.n * cur + n_prev * prev
    return pr.n * (cur + p.state_bytes) + n_prev * prev + n_apsis * (p.ids.itemsize + 2)


def kernel_label(pr):
    """The kernels the oa_step HIP events bracket for this workload."""
    if pr.n_global and pr.part:
        return ('oa_step: k_part_scatter + k_part_join' +
                (' + k_step' if pr.n_small else ''))
    if pr.n_global:
        return 'oa_step: k_big_frame + k_big_join' + (' + k_step' if pr.n_small else '')
    return 'k_step'


def cpu_baseline(snap_cur, snap_prev, cat_cur, cat_prev, H, z, gpu_prev_angles,
                 gpu_ids, gpu_offs, n_halos, mode, workers):
    """Time the reference's per-halo path on the CPU (oracle/cpu_baseline.py, a child
    process that never touches the GPU) on the first ``n_halos`` blocks of the last
    timed snapshot pair: the reference's own join (setdiff1d/in1d/myin1d) on 1 core and
    over ``workers`` processes, and the oracle's searchsorted join on 1 core.  Returns
    the child's JSON plus whether its apsis IDs equal the GPU's for the sample."""
    import subprocess
    import tempfile

    def host(snap, k):
        offs = snap['region_offsets']
        end = int(offs[k]) if k < len(offs) else int(snap['ids'].numel())
        return ({key: snap[key][:end].cpu().numpy() for key in ('ids', 'coordinates', 'velocities')},
                np.append(offs[:k], end).astype(np.int64))

    cur, cb = host(snap_cur, n_halos)
    prv, pb = host(snap_prev, n_halos)
    tmp = '/dev/shm' if os.path.isdir('/dev/shm') else None
    with tempfile.TemporaryDirectory(dir=tmp) as td:
        path = os.path.join(td, 'sample.npz')
        np.savez(path, c_ids=cur['ids'], c_x=cur['coordinates'], c_v=cur['velocities'],
                 p_ids=prv['ids'], p_x=prv['coordinates'], p_v=prv['velocities'],
                 c_off=cb, p_off=pb, c_centre=cat_cur[0][:n_halos], c_bulk=cat_cur[2][:n_halos],
                 p_centre=cat_prev[0][:n_halos], p_bulk=cat_prev[2][:n_halos],
                 angles_prev=gpu_prev_angles[:pb[-1]], H=H, z=z, mode=mode,
                 mass=float(snap_cur['masses']), box=float(snap_cur['box_size']))
        ids_out = os.path.join(td, 'ids.npy')
        env = dict(os.environ, OMP_NUM_THREADS='1', OPENBLAS_NUM_THREADS='1', MKL_NUM_THREADS='1')
        r = subprocess.run([sys.executable, os.path.join(ROOT, 'oracle', 'cpu_baseline.py'), path,
                            '--workers', str(workers), '--ids-out', ids_out],
                           capture_output=True, text=True, env=env, timeout=900)
        if r.returncode != 0:
            raise RuntimeError('cpu baseline failed: %s' % r.stderr[-2000:])
        out = json.loads(r.stdout.strip().splitlines()[-1])
        want = np.load(ids_out)
    got = gpu_ids[:int(gpu_offs[n_halos])]
    out['identical'] = bool(np.array_equal(want, got))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--particles', type=float, default=1e8, help='per GPU')
    ap.add_argument('--halos', type=int, default=10000)
    ap.add_argument('--mode', default='pericentric')
    ap.add_argument('--dtype', default='float32', choices=['float32', 'float64'],
                    help='coordinates / velocities / catalogue dtype (configs[1] is float64)')
    ap.add_argument('--max-snapshots', type=int, default=40,
                    help='device memory guard: snapshots generated (steps + warmup + 1)')
    ap.add_argument('--cpu-halos', type=int, default=1500)
    ap.add_argument('--cpu-workers', type=int, default=0,
                    help='processes of the P-core CPU baseline (0: min(16, cpu_count): the '
                         'GPU box gives one GPU 16 host cores)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--scaling', default=None, choices=['weak', 'strong'],
                    help='strong (default for N > 1): --particles in total over the ranks, '
                         'BASELINE configs[3]; weak: --particles per GPU (configs[2] on every '
                         'rank).  N = 1: both are configs[2]')
    ap.add_argument('--ramp-steps', type=int, default=-1,
                    help='back-to-back launches of the warm-up steps before the W warm-up '
                         'steps proper, so the timed steps run at the steady GPU clock (-1: '
                         '30 per GPU-equivalent of work, i.e. 30 x N under strong scaling)')
    ap.add_argument('--no-output-stage', action='store_true',
                    help='N > 1: skip the second timed pass that includes the records\' '
                         'output stage (host_share.SharedRecordStage)')
    ap.add_argument('--sharded', action='store_true',
                    help='N = 1: drive the multi-GPU path (ShardedEngine, its per-snapshot '
                         'collectives at world 1) instead of OrbitEngine -- a probe of that '
                         'path\'s per-step overhead, not the headline')
    ap.add_argument('--backend', default='nccl',
                    help="collective backend for N > 1 ('gloo': rehearsal with several "
                         "ranks on one GPU; collectives go through host memory)")
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    if args.scaling is None:
        args.scaling = 'strong' if world > 1 else 'weak'
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    import torch
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    dist = None
    gloo = args.backend == 'gloo'
    cdev = torch.device('cpu') if gloo else dev           # where collective tensors live
    shard = world > 1 or args.sharded         # the ShardedEngine path
    if shard:
        import torch.distributed as dist
        if world == 1:
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            os.environ.setdefault('MASTER_PORT', '29571')
            os.environ.setdefault('RANK', '0')
            os.environ.setdefault('WORLD_SIZE', '1')
        if gloo:
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=dev)

    def barrier():
        if gloo:
            dist.barrier()
        else:
            dist.barrier(device_ids=[local])

    import orbitanalysis_amd  # noqa: F401
    from orbitanalysis_amd import _native
    from orbitanalysis_amd.engine import OrbitEngine, SnapshotState, layout_of, meta_angles
    from orbitanalysis_amd.synthetic_device import DevicePlummer
    from orbitanalysis_amd.utils import hubble_parameter

    t_setup = time.perf_counter()
    # weak: args.particles per GPU (configs[2] on every rank); strong: args.particles
    # in total, each rank holding one ID range (configs[3])
    per_rank = int(args.particles) if args.scaling == 'weak' else int(args.particles) // world
    gen = DevicePlummer(n_halos=args.halos, n_particles=per_rank, seed=0,
                        rank=rank, world=world, device=dev, dtype=args.dtype)
    # one snapshot per step, none reused: every timed pair is (s - 1, s) of one orbit
    S = args.steps + args.warmup + 1
    if S > args.max_snapshots:
        raise SystemExit('--steps + --warmup + 1 = %d snapshots > --max-snapshots %d'
                         % (S, args.max_snapshots))
    snaps, cats = [], []
    for s in range(S):
        snaps.append(gen.snapshot(s))
        cats.append(gen.catalogue(s))
        log('rank %d snapshot %d/%d: %d particles' % (rank, s + 1, S, snaps[-1]['ids'].numel()))
    cos = gen.cosmology
    H = hubble_parameter(cos['redshift'], cos['H0'], cos['Omega_m'], cos['Omega_L'])
    z = cos['redshift']
    exists = np.arange(args.halos)
    eng = OrbitEngine(mode=args.mode, device=dev)

    prep_s = []                               # host planning per compare step (untimed)
    if not shard:
        # snapshot 0: frame only (the reference's i == istart), outside the timing
        prep0 = eng.prepare(snaps[0], cats[0][0], cats[0][2], H, z, exists, False)
        eng.launch(prep0, None)
        chain = [(prep0, 0)]
        layout = layout_of(prep0, exists)
        for t in range(1, args.warmup + args.steps + 1):
            tp = time.perf_counter()
            pr = eng.prepare(snaps[t], cats[t][0], cats[t][2], H, z, exists, True,
                             prev_layout=layout)
            prep_s.append(time.perf_counter() - tp)
            chain.append((pr, t))
            # large halos: this step's bucket set is the next step's previous state
            layout = layout_of(pr, exists)
        preps = [c[0] for c in chain[1:]]
    else:
        # the product's multi-GPU path: ShardedEngine over this rank's ID range (the
        # generator hands every rank its own rows: presharded), one all-gather of the
        # halo catalogue rows per snapshot inside the timed launch
        from orbitanalysis_amd.sharding import ShardedEngine, EngineLocal
        seng = ShardedEngine(EngineLocal(eng), presharded=True)
        sp0 = seng.prepare(snaps[0], cats[0][0], cats[0][2], H, z, exists, False)
        seng.launch(sp0)
        chain = [(sp0, 0)]
        for t in range(1, args.warmup + args.steps + 1):
            tp = time.perf_counter()
            chain.append((seng.prepare(snaps[t], cats[t][0], cats[t][2], H, z, exists, True,
                                       prev=chain[-1][0]), t))
            prep_s.append(time.perf_counter() - tp)
        preps = [c[0].lp for c in chain[1:]]
    for p in preps:
        ws = eng.workspace(p)                 # grown to the largest step
    ws.status.zero_()
    log('setup %.1f s; items/step %d (large halos %d)'
        % (time.perf_counter() - t_setup, preps[0].n_small, preps[0].n_global))

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]

    def run(k, events=None, defer=False):
        pr, s = chain[k + 1]
        prev_pr, ps = chain[k]
        if shard:
            # defer: the drop-in driver's order -- the step's status is read (and the step
            # re-run on a re-plan or look-back timeout) by the fetch that settles it
            return seng.launch(pr, prev=prev_pr, step_events=events, check=defer, defer=defer)
        return eng.launch(pr, ws, SnapshotState.of(prev_pr, exists, ids=snaps[ps]['ids']),
                          step_events=events)

    # Clock ramp: after the host-side setup the GPU runs its first ~15 launches 5-25 %
    # slower (rocprof trace of this bench, profiles/r06/: 1.60 -> 1.40 ms per k_step over
    # 15 launches, then flat), longer than W = 5 warm-up steps cover.  The warm-up steps
    # are launched back to back first (each re-run writes the same outputs); the count is
    # fixed, so every rank issues the same collectives.
    ramp = args.ramp_steps if args.ramp_steps >= 0 else \
        30 * (world if args.scaling == 'strong' else 1)
    for i in range(ramp):
        run(i % max(args.warmup, 1))
    for k in range(args.warmup):
        run(k)
    torch.cuda.synchronize()
    if dist:
        barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        last_res = run(args.warmup + i, evs[i])
    t_issue = time.perf_counter() - t0          # the host's launch calls of the K steps
    torch.cuda.synchronize()
    if dist:
        barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    units = sum(preps[args.warmup + i].n for i in range(args.steps))
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        u = torch.tensor([units], dtype=torch.float64, device=cdev)
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
        units = float(u.item())
    status = int(ws.status[0].item())
    if status:
        raise RuntimeError('oa_step reported status %#x (table overflow) during the bench' % status)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    last = preps[-1]
    n_apsis = int(ws.total.item())

    # the records' gather to rank 0 and D2H of the last timed step (outside the timed
    # region, as the driver overlaps it with the next snapshot's step): ms per fetch,
    # the max over ranks, over 3 repetitions
    fetch = []
    fdt = snaps[0]['ids'].cpu().numpy().dtype
    for _ in range(3):
        if dist:
            barrier()
        torch.cuda.synchronize()
        tf = time.perf_counter()
        (seng if shard else eng).fetch_async(last_res, fdt).wait()
        if dist:
            barrier()
        fetch.append(time.perf_counter() - tf)
    fetch_ms = float(np.median(fetch)) * 1e3
    if dist:
        t = torch.tensor([fetch_ms], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        fetch_ms = float(t.item())

    # each timed step's own apsis count (its records' bytes): the steps are re-run
    # once, untimed, in order (each reads the state its predecessor wrote); N > 1: this
    # rank's own count (the roofline is rank 0's kernel)
    n_aps = []
    for i in range(args.steps):
        r_i = run(args.warmup + i)
        torch.cuda.synchronize()
        n_aps.append(int(ws.total.item()) if not shard else int(r_i.lp.res.total.item()))

    # N > 1: the same K steps again with the output stage of the drop-in driver
    # (track_orbits' pipelined order: step s launched, then the records of s - 1 start
    # towards the host, then those of s - 2 are waited for), every rank storing its own
    # records into the shared host buffer (host_share.SharedRecordStage); timed as the
    # compute pass.  value stays the compute pass (as at N = 1, where the records' D2H is
    # outside the timed region too); this pass is reported beside it.
    stage = None
    if world > 1 and not args.no_output_stage:
        from orbitanalysis_amd.host_share import SharedRecordStage
        seng._stage = SharedRecordStage(seng.group, seng.rank, seng.world, seng.ROOT, timeout=120)
        if not seng._stage.probe(eng.lib, cdev, True):
            stage = {'skipped': 'a rank could not page-lock a shared-memory segment'}
    if world > 1 and not args.no_output_stage and stage is None:
        seng.profile_fetch = False
        pend, moved = [], []
        for i in range(2):                        # warm: maps and registers the slots
            seng.fetch_async(run(i, defer=True), fdt).wait()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        prev_res = None
        for i in range(args.steps):
            r_i = run(args.warmup + i, defer=True)
            if prev_res is not None:
                pend.append(seng.fetch_async(prev_res, fdt))
            if len(pend) > 1:
                got = pend.pop(0)
                got.wait()
                moved.append(got.moved)
            prev_res = r_i
        pend.append(seng.fetch_async(prev_res, fdt))
        for f in pend:
            f.wait()
            moved.append(f.moved)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        e2e = time.perf_counter() - t1
        t = torch.tensor([e2e], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        e2e = float(t.item())
        mv = torch.tensor([float(np.mean(moved))], dtype=torch.float64, device=cdev)
        allmv = [torch.zeros_like(mv) for _ in range(world)]
        dist.all_gather(allmv, mv)
        stage = {'e2e_value': units / e2e, 'e2e_ms_per_step': e2e / args.steps * 1e3,
                 'bytes_stored_per_step_by_rank': [float(x.item()) for x in allmv],
                 'note': 'the K compare steps again, each followed (pipelined as track_orbits '
                         'does) by its records\' move to the host: every rank stores its own '
                         'records at their final positions in one page-locked host buffer all '
                         'ranks map (host_share.SharedRecordStage), rank 0 moves only its own '
                         'and waits for the others; max over ranks'}
        log('output stage: %.3f ms per step (compute only %.3f); bytes stored per rank %s'
            % (stage['e2e_ms_per_step'], elapsed / args.steps * 1e3,
               stage['bytes_stored_per_step_by_rank']))
    bytes_launch = float(np.mean([step_bytes(preps[args.warmup + i], preps[args.warmup + i].n_prev,
                                             n_aps[i]) for i in range(args.steps)]))
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    log('elapsed %.4f s for %d steps; k_step %.3f ms; %.1f GB/s; apsis %d'
        % (elapsed, args.steps, kern_ms, achieved, n_apsis))

    traffic, counters = None, None
    for name in ('pmc_k_step.json', 'pmc_part.json'):
        pmc = os.path.join(ROOT, 'profiles', name)
        if traffic is not None or not os.path.exists(pmc):
            continue
        with open(pmc) as f:
            pj = json.load(f)
        # only for the workload the counters were collected on
        if (pj.get('particles'), pj.get('halos'), pj.get('n_gpus', 1)) == \
                (per_rank, args.halos, 1):
            traffic = pj.get('hbm_bytes_per_launch')
            counters = {'source': 'profiles/' + name,
                        'fetch_size_bytes': pj.get('fetch_size_bytes'),
                        'write_size_bytes': pj.get('write_size_bytes'),
                        'width_calibration': pj.get('width_calibration'),
                        'traffic_over_algorithmic': traffic / bytes_launch if traffic else None}
    # §8(d): read-only bytes against the peak (the reads alone, per launch)
    read_launch = float(np.mean([step_bytes(preps[args.warmup + i], preps[args.warmup + i].n_prev,
                                            0, reads_only=True) for i in range(args.steps)]))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        pr_last, s_last = chain[-1]
        prev_pr, s_prev = chain[-2]
        ang_prev = meta_angles(prev_pr.meta)
        offs = ws.offsets[:int(last.has_prog.sum()) + 1].cpu().numpy()
        gids = ws.out_ids[:n_apsis].cpu().numpy()
        nh = min(args.cpu_halos, args.halos)
        ncpu = os.cpu_count() or 1
        workers = args.cpu_workers or min(16, ncpu)
        cb = cpu_baseline(snaps[s_last], snaps[s_prev], cats[s_last], cats[s_prev],
                          H, z, ang_prev, gids, offs, nh, args.mode, workers)
        pc, r1, p1 = cb['ref_pcore'], cb['ref_1core'], cb['port_1core']
        cpu = {'value': pc['rate'], 'unit': 'particle-snapshots/s', 'cores': workers,
               'kind': 'port',
               'sample': '%d of %d halos (%d particles) of the last timed snapshot pair; the '
                         "reference's per-halo path restated (region_frame, setdiff1d/in1d/"
                         'myin1d join, calc_angles) with the halos split over %d processes '
                         '(host has %d CPUs; the box allots one GPU 16), %.2f s; apsis IDs '
                         'identical to the GPU: %s' % (nh, args.halos, cb['particles'], workers,
                                                       ncpu, pc['seconds'], cb['identical']),
               'single_core': {'value': r1['rate'], 'seconds': r1['seconds'],
                               'algorithm': 'reference join (setdiff1d + in1d + myin1d)'},
               'single_core_searchsorted': {'value': p1['rate'], 'seconds': p1['seconds'],
                                            'algorithm': 'oracle join (argsort + searchsorted)'},
               'host_cpus': ncpu,
               'cores_note': ('P = min(16, os.cpu_count()): os.cpu_count() reports the whole '
                              'host (%d CPUs) but the GPU box allots one GPU 16 host cores, so '
                              'a pool of os.cpu_count() processes would time-share those 16 '
                              '(--cpu-workers overrides)' % ncpu)}
        log('cpu baseline: %d procs %.3e/s, 1 core %.3e/s (searchsorted join %.3e/s), parity %s'
            % (workers, pc['rate'], r1['rate'], p1['rate'], cb['identical']))

    if rank == 0:
        out = {
            'metric': METRIC, 'value': units / elapsed, 'unit': 'particle-snapshots/s',
            'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'warmup_note': 'the W warm-up steps are preceded by %d back-to-back launches of '
                           'the same warm-up steps (GPU clock ramp after the host-side '
                           'setup); the timed region is exactly the K steps' % ramp,
            'ms_per_step': elapsed / args.steps * 1e3, 'higher_is_better': True,
            'scaling': args.scaling, 'vs_baseline': None,
            'dtype': last.plan.coord.name.replace('float', 'f'),
            'data': 'synthetic: %d Plummer spheres (device-generated, AHW sampling, leapfrog '
                    'orbits), region cut r<4a, per-snapshot shuffled blocks, int64 randperm IDs'
                    % args.halos,
            'config': {'workload': 'BASELINE configs[%d]: %.0e particles%s, %d halos, %s '
                                   'coords/vels/centres, catalogue bulk velocities, periodic '
                                   'box, Hubble term, %s'
                                   % ((3 if args.scaling == 'strong' else 2)
                                      if args.dtype == 'float32' else 1, args.particles,
                                      '/GPU' if args.scaling == 'weak' else ' in total',
                                      args.halos, last.plan.coord.name.replace('float', 'f'),
                                      args.mode),
                       'particles_per_step_per_gpu': int(last.n),
                       'halos': args.halos, 'work_items': int(last.n_small),
                       'large_halos': int(last.n_global),
                       'parallelism': 'id-range shards x%d (ShardedEngine, presharded; one '
                                      'catalogue all-gather per snapshot)' % world
                                      if shard else 'single GPU',
                       'timed_region': 'the device launches of K compare steps (frame, join, '
                                       'sign test, angles, compaction) on inputs resident in '
                                       'HBM; the host planning of each step (prepare: halo '
                                       'table, item plan, partition plan) runs before the '
                                       'timed region and is excluded, see host_prepare_ms',
                       'host_prepare_ms': float(np.median(prep_s)) * 1e3,
                       'host_launch_ms': t_issue / args.steps * 1e3,
                       'fetch_ms': fetch_ms,
                       'fetch_note': 'records of one step moved to the host for rank 0 '
                                     '(N = 1: one D2H; N > 1: every rank stores its own '
                                     'records into the shared host buffer), outside the '
                                     'timed region (the driver overlaps it with the next '
                                     'step); max over ranks',
                       'output_stage': stage,
                       'weak_scaling_config': 'bench.py --scaling weak: configs[2] (1e8 '
                                              'particles) on every rank'
                                              if world > 1 else None},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS,
                         'traffic': traffic, 'kernel': kernel_label(last), 'kernel_ms': kern_ms,
                         'alg_bytes_per_launch': bytes_launch,
                         'alg_read_bytes_per_launch': read_launch,
                         'read_only_achieved': read_launch / (kern_ms * 1e-3) / 1e9,
                         'read_only_frac': read_launch / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         'counters': counters},
            'cpu_baseline': cpu,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
