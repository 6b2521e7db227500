"""Print the median, per-snapshot times and the D2H / kernel timeline of bench_e2e JSON
files (one per argument)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    t = d.get('timeline', {})
    print(f, 'median', d['ms_per_snapshot_median'], 'per snapshot', d['ms_per_snapshot'])
    print('  kernel_ms', t.get('kernel_ms'))
    print('  gap_ms   ', t.get('gap_before_kernel_ms'))
    print('  d2h_ms   ', t.get('d2h_ms'))
