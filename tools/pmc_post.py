#!/usr/bin/env python3
"""Reduce tools/pmc_post.sh's counter passes to per-kernel HBM bytes per dispatch.

HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE: tools/ubench/fetch_cal.hip measured FETCH_SIZE
at 1/2 of the bytes for every streaming load width and WRITE_SIZE exact for every store
width on gfx950 (profiles/fetch_cal.json).  Collation (bench_post.py: 10 snapshots, one
k_collate_rank / k_collate_offsets / k_collate_place round each) skips the first
snapshot's round, as the bench's figures do (it starts from an empty state).

usage: pmc_post.py PMC_DIR OUT_JSON
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def per_dispatch(d, counter):
    rows = collections.OrderedDict()
    for f in glob.glob(os.path.join(d, counter, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r'(k_collate_\w+|k_central\w*|k_mp_\w+)', r['Kernel_Name'])
            if not m:
                continue
            key = (int(r['Dispatch_Id']), m.group(1))
            rows[key] = rows.get(key, 0.0) + float(r['Counter_Value']) * 1024.0
    return sorted(rows.items())


def main():
    d, out = sys.argv[1], sys.argv[2]
    fetch, write = per_dispatch(d, 'FETCH_SIZE'), per_dispatch(d, 'WRITE_SIZE')
    res = {'rule': '2 x FETCH_SIZE + WRITE_SIZE (profiles/fetch_cal.json)', 'kernels': {}}
    for name in sorted({k[1] for k, _ in fetch}):
        fv = [v for (i, k), v in fetch if k == name]
        wv = [v for (i, k), v in write if k == name]
        skip = 1 if name.startswith('k_collate') else 0      # snapshot 1: empty state
        fv, wv = fv[skip:], wv[skip:]
        n = min(len(fv), len(wv))
        if not n:
            continue
        f = sum(fv[:n]) / n
        w = sum(wv[:n]) / n
        res['kernels'][name] = {'dispatches': n, 'fetch_size_bytes': f, 'write_size_bytes': w,
                                'hbm_bytes_per_dispatch': 2 * f + w}
    k = res['kernels']
    res['per_call'] = {
        'collate': sum(v['hbm_bytes_per_dispatch'] for n_, v in k.items() if n_.startswith('k_collate')),
        'central': sum(v['hbm_bytes_per_dispatch'] for n_, v in k.items() if n_.startswith('k_central')),
        'mainprog': sum(v['hbm_bytes_per_dispatch'] for n_, v in k.items() if n_.startswith('k_mp_')),
    }
    with open(out, 'w') as fo:
        json.dump(res, fo, indent=1, sort_keys=True)
    print(json.dumps(res['per_call']))
    for n_, v in sorted(k.items()):
        print('%-22s n=%3d  fetch %.3e  write %.3e  hbm %.3e' % (n_, v['dispatches'], v['fetch_size_bytes'],
                                                                v['write_size_bytes'], v['hbm_bytes_per_dispatch']))


if __name__ == '__main__':
    main()
