#!/usr/bin/env python3
"""Per-dispatch k_step durations from a rocprofv3 --kernel-trace of bench.py, split into
the bench's phases by dispatch order: ramp + warm-up launches, the K timed steps, then
the untimed re-run that reads each step's apsis count.

bench.py launches, in order: R ramp launches, W warm-up steps, K timed steps, K re-runs
(N = 1).  The timed window's average is the rocprof figure comparable with the bench
line's HIP-event ``kernel_ms`` (the whole-trace average of rocprof --stats also holds the
clock ramp after the host-side setup).

usage: trace_window.py TRACE_DIR_OR_CSV RAMP WARMUP STEPS [OUT_JSON]
"""
import csv
import glob
import json
import os
import sys


def main():
    src, ramp, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    f = src if src.endswith('.csv') else glob.glob(os.path.join(src, '**', '*kernel_trace.csv'),
                                                   recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f))
            if 'k_step<' in r['Kernel_Name'] and ', true, false, true' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows]
    a = ramp + warm
    timed = d[a:a + steps]
    res = {'source': os.path.relpath(f), 'kernel': rows[0]['Kernel_Name'] if rows else None,
           'dispatches': len(d), 'ramp_plus_warmup': a, 'timed': len(timed),
           'timed_mean_ms': sum(timed) / len(timed) if timed else None,
           'timed_min_ms': min(timed) if timed else None,
           'timed_max_ms': max(timed) if timed else None,
           'all_mean_ms': sum(d) / len(d) if d else None,
           'first_ramp_ms': d[:5], 'durations_ms': [round(x, 4) for x in d]}
    if len(sys.argv) > 5:
        with open(sys.argv[5], 'w') as fo:
            json.dump(res, fo, indent=1)
        # the timed window in rocprofv3's kernel_stats.csv columns (one row)
        if timed:
            ns = [int(round(x * 1e6)) for x in timed]
            with open(os.path.splitext(sys.argv[5])[0] + '_kernel_stats_timed.csv', 'w') as fo:
                w = csv.writer(fo, quoting=csv.QUOTE_NONNUMERIC)
                w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'MinNs', 'MaxNs',
                            'Window'])
                w.writerow([res['kernel'], len(ns), sum(ns), sum(ns) / len(ns), min(ns), max(ns),
                            'dispatches %d..%d of %d (after %d ramp + warm-up launches)'
                            % (a, a + len(ns) - 1, len(d), a)])
    print(json.dumps({k: v for k, v in res.items() if k != 'durations_ms'}))


if __name__ == '__main__':
    main()
