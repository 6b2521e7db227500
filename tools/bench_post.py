"""Benchmarks of SURVEY §8(f) rows f3/f4 on one MI355X (device-resident inputs), each
with its HBM roofline and the CPU oracle timed on a bounded sample beside it.

  python tools/bench_post.py [--which collate,central,mainprog] [--scale 1.0]

Prints one JSON line per workload:
* collate  — Apsides.collate_apsides at config-3 scale: 1e4 halos, ~5e6 apsis records
             per snapshot (5 % of 1e8), IDs drawn from 1e4-particle halo pools, f16
             angles, pi/4 cut, 10 snapshots; unit = apsis records/s; algorithmic bytes
             per snapshot = 10 B per record + 16 B per old state element read + 16 B
             per merged element written.
* central  — get_central_particle_ids over 1e8 float32 particles in 1e4 blocks, n=100,
             periodic box; unit = particles/s; algorithmic bytes = 12 B per particle.
* mainprog — find_main_progenitors: 1e8 int64 halo members in 1e4 halos, 1e4 tracked
             blocks of 100 central IDs; unit = halo members/s; algorithmic bytes = 8 B
             per member + 8 B per tracked ID.
Timing: HIP events on the launch stream around the device calls only; the kernels'
share is cross-checked with rocprofv3 --kernel-trace --stats (profiles/).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PEAK = 8000.0


def log(*a):
    print('[bench_post]', *a, file=sys.stderr, flush=True)


def _pmc(which):
    """HBM bytes per call of a workload's kernels from profiles/pmc_post.json
    (tools/pmc_post.sh over this bench at scale 1), or None."""
    p = os.path.join(ROOT, 'profiles', 'pmc_post.json')
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f).get('per_call', {}).get(which)


def roof(bytes_, ms, which=None, scale=1.0):
    gbs = bytes_ / (ms * 1e-3) / 1e9
    t = _pmc(which) if which and scale == 1.0 else None
    return {'bound': 'hbm', 'achieved': gbs, 'peak': PEAK, 'unit': 'GB/s', 'frac': gbs / PEAK,
            'traffic': t, 'traffic_over_algorithmic': t / bytes_ if t else None}


def make_track_groups(rng, n_halos, n_snap, rec_per_halo, pool):
    """Synthetic track_orbits output groups (the collate input)."""
    groups = {}
    for s in range(1, n_snap + 1):
        lens = rng.poisson(rec_per_halo, n_halos)
        h = np.repeat(np.arange(n_halos), lens)
        ids = h.astype(np.int64) * pool + rng.integers(0, pool, h.size)
        ang = rng.uniform(0, 6.3, h.size).astype(np.float16)
        g = {'region_offsets': np.concatenate([[0], np.cumsum(lens)]),
             'pericenter_IDs': ids, 'angles': ang, 'halo_IDs': np.arange(n_halos),
             'region_radii': np.ones(n_halos), 'region_positions': np.zeros((n_halos, 3)),
             'bulk_velocities': np.zeros((n_halos, 3))}
        if s != n_snap:
            g['final_descendant_IDs'] = np.arange(n_halos)
        groups['snapshot_%03d' % s] = g
    return groups


def bench_collate(scale, cpu_halos):
    import torch
    from orbitanalysis_amd import _native as N
    from orbitanalysis_amd.postprocessing import _CollateState, _dev
    from oracle import post_oracle as PO
    rng = np.random.default_rng(5)
    nh, ns = int(1e4 * scale), 10
    groups = make_track_groups(rng, nh, ns, 500, 10000)
    lib = N.load(require_device=True)
    dev = torch.device('cuda', 0)
    f16 = np.arange(65536, dtype=np.uint16).view(np.float16)
    lut_d = _dev((np.nan_to_num(f16.astype(np.float64), nan=-1) > np.pi / 4).astype(np.uint8), dev)
    inputs = []
    for g in sorted(groups):
        d = groups[g]
        off = d['region_offsets']
        inputs.append((_dev(d['pericenter_IDs'], dev), _dev(d['angles'], dev),
                       off[:-1].astype(np.int64), np.diff(off).astype(np.int64)))
    torch.cuda.synchronize()
    state = _CollateState(nh, dev)
    events, n_old, n_rec, n_new = [], [], [], []
    for ids_d, ang_d, so, sc in inputs:
        n_old.append(state.total)
        state.merge(lib, ids_d, 0, 1, ang_d, lut_d, so, sc, events=events)
        n_rec.append(int(sc.sum()))
        n_new.append(state.total)
    torch.cuda.synchronize()
    ms = [e0.elapsed_time(e1) for e0, e1 in events]
    # snapshot 1 starts from an empty state; report the steady snapshots 2..ns
    tot_ms = sum(ms[1:])
    bytes_ = sum(10 * r + 16 * o + 16 * n for r, o, n in zip(n_rec[1:], n_old[1:], n_new[1:]))
    recs = sum(n_rec[1:])
    # CPU oracle on the first cpu_halos halos of every snapshot
    sub = {}
    for g, d in groups.items():
        off = d['region_offsets']
        e = int(off[cpu_halos])
        sub[g] = dict(d, region_offsets=off[:cpu_halos + 1], pericenter_IDs=d['pericenter_IDs'][:e],
                      angles=d['angles'][:e], halo_IDs=d['halo_IDs'][:cpu_halos])
        if 'final_descendant_IDs' in d:
            sub[g]['final_descendant_IDs'] = d['final_descendant_IDs'][:cpu_halos]
        for k in ('region_radii', 'region_positions', 'bulk_velocities'):
            sub[g][k] = d[k][:cpu_halos]
    t0 = time.perf_counter()
    want = PO.collate_apsides(sub, {'mode': 'pericentric'})
    cdt = time.perf_counter() - t0
    crec = sum(int(sub[g]['region_offsets'][-1]) for g in sorted(sub)[1:])
    # parity on the sample: the device state restricted to those halos
    off = state.off.cpu().numpy()
    keys = state.keys[:state.total].cpu().numpy().view(np.uint64) ^ np.uint64(1 << 63)
    ok = np.array_equal(keys[:off[cpu_halos]].view(np.int64),
                        want['snapshot_%03d' % ns]['particle_IDs'])
    return {'metric': 'apsis records/s (collate_apsides)', 'value': recs / (tot_ms * 1e-3),
            'unit': 'records/s', 'ms_per_snapshot': tot_ms / (ns - 1), 'dtype': 'int64',
            'config': {'workload': 'f3 collate: %d halos, ~%d records/snapshot, %d snapshots, '
                       'pi/4 cut' % (nh, recs // (ns - 1), ns), 'state_final': n_new[-1]},
            'roofline': dict(roof(bytes_ / (ns - 1), tot_ms / (ns - 1), 'collate', scale),
                             kernel='oa_collate_step'),
            'cpu_baseline': {'value': crec / cdt, 'unit': 'records/s', 'cores': 1, 'kind': 'port',
                             'sample': '%d of %d halos, all %d snapshots, %.1f s; final particle '
                                       'IDs identical to the GPU: %s' % (cpu_halos, nh, ns, cdt, ok)}}


def bench_central(scale, cpu_halos, reps=5):
    import torch
    from orbitanalysis_amd.progenitors import CentralIds
    from oracle import post_oracle as PO
    rng = np.random.default_rng(6)
    nh, per = int(1e4 * scale), 10000
    n = nh * per
    centres = rng.uniform(0, 100, (nh, 3)).astype(np.float32)
    x = (np.repeat(centres, per, axis=0) + rng.normal(0, 1, (n, 3)).astype(np.float32)) % np.float32(100)
    snap = {'ids': rng.permutation(n).astype(np.int64), 'coordinates': x.astype(np.float32),
            'region_offsets': np.arange(nh, dtype=np.int64) * per, 'box_size': 100.0}
    c = CentralIds(snap, centres, 100)
    c.launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        c.launch()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    got, _ = c.result()
    sub = {'ids': snap['ids'][:cpu_halos * per], 'coordinates': x[:cpu_halos * per],
           'region_offsets': snap['region_offsets'][:cpu_halos], 'box_size': 100.0}
    t0 = time.perf_counter()
    want, _ = PO.get_central_particle_ids(sub, centres[:cpu_halos], 100)
    cdt = time.perf_counter() - t0
    ok = np.array_equal(want, got[:cpu_halos * 100])
    return {'metric': 'particles/s (get_central_particle_ids, n=100)', 'value': n / (ms * 1e-3),
            'unit': 'particles/s', 'ms_per_call': ms, 'dtype': 'f32',
            'config': {'workload': 'f4 central IDs: %d particles f32 in %d blocks, n=100, box'
                       % (n, nh)},
            'roofline': dict(roof(12.0 * n, ms, 'central', scale), kernel='k_central'),
            'cpu_baseline': {'value': cpu_halos * per / cdt, 'unit': 'particles/s', 'cores': 1,
                             'kind': 'port', 'sample': '%d of %d blocks, %.1f s; IDs identical '
                             'to the GPU: %s' % (cpu_halos, nh, cdt, ok)}}


def bench_mainprog(scale, cpu_blocks, reps=5):
    import torch
    from orbitanalysis_amd.progenitors import MainProgenitors
    from oracle import post_oracle as PO
    rng = np.random.default_rng(7)
    nh, per = int(1e4 * scale), 10000
    n = nh * per
    hp = rng.permutation(n).astype(np.int64)
    ho = np.arange(nh, dtype=np.int64) * per
    # each descendant tracks 100 IDs: 70 from one progenitor halo, 30 from others / absent
    nb = nh
    main = rng.integers(0, nh, nb)
    idx = (main[:, None] * per + rng.integers(0, per, (nb, 70))).ravel()
    other = rng.integers(0, n + n // 10, nb * 30)
    tp = np.concatenate([hp[idx].reshape(nb, 70),
                         np.where(other < n, hp[np.minimum(other, n - 1)], other).reshape(nb, 30)],
                        axis=1).ravel()
    to = np.arange(nb, dtype=np.int64) * 100
    m = MainProgenitors(hp, ho, tp, to)
    m.launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        m.launch()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    got = m.result()
    # CPU oracle on a bounded sample: the first cpu_blocks tracked blocks against all members
    t0 = time.perf_counter()
    want = PO.find_main_progenitors(hp, ho, tp[:cpu_blocks * 100], to[:cpu_blocks])
    cdt = time.perf_counter() - t0
    ok = [int(v) for v in want] == [int(v) for v in got[:cpu_blocks]]
    return {'metric': 'halo members/s (find_main_progenitors)', 'value': n / (ms * 1e-3),
            'unit': 'members/s', 'ms_per_call': ms, 'dtype': 'int64',
            'config': {'workload': 'f4 main progenitors: %d int64 members in %d halos, %d tracked '
                       'blocks of 100' % (n, nh, nb)},
            'roofline': dict(roof(8.0 * n + 8.0 * len(tp), ms, 'mainprog', scale),
                             kernel='k_mp_probe'),
            'cpu_baseline': {'value': n / cdt, 'unit': 'members/s', 'cores': 1, 'kind': 'port',
                             'sample': 'all %d members, first %d tracked blocks, %.1f s; results '
                             'identical to the GPU: %s' % (n, cpu_blocks, cdt, ok)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--which', default='collate,central,mainprog')
    ap.add_argument('--scale', type=float, default=1.0)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    for w in args.which.split(','):
        t0 = time.time()
        if w == 'collate':
            r = bench_collate(args.scale, 300)
        elif w == 'central':
            r = bench_central(args.scale, 100)
        elif w == 'mainprog':
            r = bench_mainprog(args.scale, 1000)
        else:
            raise SystemExit('unknown workload ' + w)
        log(w, 'done in %.1f s' % (time.time() - t0))
        print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
