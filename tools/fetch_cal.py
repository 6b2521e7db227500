#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE correction per access width, from tools/ubench/fetch_cal
under rocprofv3 --pmc (tools/gpu.sh step ``cal``).

Each calibration kernel streams a known byte count with one load (or store) width;
factor[w] = known bytes / counter bytes (counter KB x 1024).  MI355X_MICROARCH.md
§HBM gives 2.0 for 16-B loads and 1.0 for 16-B stores; the other widths are what this
measures.  ``traffic_of`` applies the factors to a kernel whose bytes per width are
known (k_step: tools/pmc_summary.py).

usage: fetch_cal.py CAL_DIR PROGRAM_STDOUT > fetch_cal.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def counters(d):
    """{(kernel, width): counter bytes} from every counter_collection.csv under d."""
    per = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r'k_cal_(load|store)<(\d)>', r['Kernel_Name'])
            if m:
                per[(m.group(1), m.group(2), r['Counter_Name'])] += float(r['Counter_Value'])
    return per


def traffic_of(bytes_by_width, factors):
    """True bytes estimated from a counter value whose accesses have these byte counts
    per width: the counter a mix of widths reports is sum(b_w / f_w); scaling the
    measured counter by sum(b_w) / sum(b_w / f_w) gives the mix's true bytes."""
    alg = sum(bytes_by_width.values())
    expect = sum(b / factors[w] for w, b in bytes_by_width.items())
    return alg / expect


def main():
    d, out = sys.argv[1], sys.argv[2]
    known = None
    for line in open(out):
        if line.startswith('{"load_bytes"'):
            known = json.loads(line)
    per = counters(d)
    res = {'source': 'tools/ubench/fetch_cal.hip: 2 GiB streamed per kernel, one width each, '
                     'buffer loads/stores with the nt bit (k_step\'s shapes)',
           'load': {}, 'store': {}}
    for (kind, w, c), v in sorted(per.items()):
        if (kind, c) not in (('load', 'FETCH_SIZE'), ('store', 'WRITE_SIZE')):
            continue
        b = known['%s_bytes' % kind][w]
        res[kind]['dword_x%s' % w] = {'bytes': b, 'counter_bytes': v * 1024.0,
                                      'factor': b / (v * 1024.0)}
    json.dump(res, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == '__main__':
    main()
