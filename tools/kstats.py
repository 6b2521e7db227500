"""Summarise rocprofv3 kernel_stats.csv files: the hot-path kernels' calls and mean
durations.   python tools/kstats.py <dir-or-csv>..."""
import csv
import glob
import os
import sys

KEYS = ('k_step', 'k_big', 'k_part', 'k_gather', 'k_scan', 'k_bulk', 'k_central', 'k_mp', 'k_collate',
        'k_retro', 'fillBuffer')
for arg in sys.argv[1:]:
    files = [arg] if arg.endswith('.csv') else glob.glob(os.path.join(arg, '**', '*kernel_stats.csv'),
                                                          recursive=True)
    for f in files:
        print('==', f)
        for r in csv.DictReader(open(f)):
            n = r['Name']
            if any(k in n for k in KEYS):
                short = n.replace('void (anonymous namespace)::', '').split('(')[0]
                print('  %-58s calls %5s  avg %9.1f us  total %9.1f us' % (
                    short[:58], r['Calls'], float(r['AverageNs']) / 1e3, float(r['TotalDurationNs']) / 1e3))
