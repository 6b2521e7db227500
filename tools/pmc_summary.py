#!/usr/bin/env python3
"""Reduce the rocprofv3 --pmc passes of tools/pmc.sh to profiles/pmc_k_step.json.

HBM bytes per k_step launch, following MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE come from the L2's fabric requests.  The guide calibrates 16-B-per-lane
streams (FETCH_SIZE = 1/2 of the bytes read, WRITE_SIZE exact) and leaves other widths
to the user; tools/ubench/fetch_cal.hip measured every width k_step uses (buffer loads
of 4, 8, 12 and 16 B per lane, stores of 4, 12 and 16 B, nt bit, 2 GiB each:
profiles/fetch_cal.json): FETCH_SIZE reads 1/2 of the bytes at every load width
(factors 1.9999-2.0000) and WRITE_SIZE reads the bytes at every store width
(0.998-0.999).  So

    hbm_bytes_per_launch = f_load * FETCH_SIZE + f_store * WRITE_SIZE

with the calibrated factors (2 and 1: the guide's rule, now measured for these widths).

Round 1-5 scaled FETCH_SIZE by the frame-only launch's ratio (k = 2.57), which is not
a clean calibration: snapshot 0's arrays were written by the generator just before
that launch, so part of its reads came from the Infinity Cache and fewer requests
reached the counters.  `frame_calibrated_bytes` keeps that figure for comparison.

usage: pmc_summary.py PMC_DIR N_FRAME_ONLY [OUT_JSON]
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d, n0 = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles', 'pmc_k_step.json')
    per = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, 'p*', '**', '*counter_collection.csv'), recursive=True)):
        for r in csv.DictReader(open(f)):
            if 'k_step' not in r['Kernel_Name']:
                continue
            c = per[(os.path.relpath(f, d).split(os.sep)[0], int(r['Dispatch_Id']))]
            c[r['Counter_Name']] = c.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    # one row per dispatch, counters merged across passes by dispatch order
    passes = collections.defaultdict(list)
    for (p, disp), c in sorted(per.items()):
        passes[p].append(c)
    n = min(len(v) for v in passes.values())
    disp = [dict() for _ in range(n)]
    for p, rows in passes.items():
        for i in range(n):
            disp[i].update(rows[i])
    frame, cmp_ = disp[0], disp[1:]
    mean = {c: sum(x[c] for x in cmp_) / len(cmp_) for c in cmp_[0]}
    fetch0 = frame['FETCH_SIZE'] * 1024.0
    k = n0 * 32.0 / fetch0
    fetch = mean['FETCH_SIZE'] * 1024.0
    write = mean['WRITE_SIZE'] * 1024.0
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cal = json.load(open(os.path.join(root, 'profiles', 'fetch_cal.json')))
    f_load = sum(v['factor'] for v in cal['load'].values()) / len(cal['load'])
    f_store = sum(v['factor'] for v in cal['store'].values()) / len(cal['store'])
    res = {
        'kernel': 'k_step<float,float,float,8,compare>',
        'workload': 'bench.py defaults (1e8 particles, 1e4 halos, f32)',
        'particles': 100000000, 'halos': 10000, 'n_gpus': 1,
        'dispatches': {'frame_only': 1, 'compared': len(cmp_)},
        'calibration': {'frame_only_particles': n0, 'frame_only_read_bytes': n0 * 32,
                        'frame_only_fetch_size_bytes': fetch0, 'k': k,
                        'frame_only_write_size_bytes': frame['WRITE_SIZE'] * 1024.0,
                        'frame_only_write_expected': n0 * 16},
        'fetch_size_bytes': fetch, 'write_size_bytes': write,
        'width_calibration': {'source': 'profiles/fetch_cal.json', 'load_factor': f_load,
                              'store_factor': f_store},
        'hbm_bytes_per_launch': f_load * fetch + f_store * write,
        'hbm_read_bytes_per_launch': f_load * fetch,
        'guide_rule_bytes': 2.0 * fetch + write,
        'frame_calibrated_bytes': k * fetch + write,
        'counters_mean_compared': mean,
        'counters_frame_only': frame,
    }
    w = mean.get('SQ_WAVE_CYCLES')
    if w:
        res['sq_fractions'] = {c: mean[c] / w for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY',
                                                        'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU')
                               if c in mean}
    with open(out, 'w') as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k_: res[k_] for k_ in ('hbm_bytes_per_launch', 'guide_rule_bytes',
                                              'fetch_size_bytes', 'write_size_bytes')}))
    print('k =', k)


if __name__ == '__main__':
    main()
