"""Readers for the §8(f) golden fixtures (g9_collate, g10_progenitors; written by
tools/gen_golden.py from the reference itself)."""
import json

import numpy as np

from golden_util import load


def _param(text):
    """Collate parameters were stored as repr()s: keep their exact Python/NumPy type,
    which decides NumPy's comparison dtype for ``angles > angle_cut``."""
    if text.startswith("<class 'numpy."):
        return getattr(np, text.split('.')[1].rstrip("'>"))
    return eval(text, {'np': np, '__builtins__': {}})


def collate_runs():
    """[(case, tag, input groups, attrs, collate kwargs, final-counts kwargs|None, want)]."""
    fix = load('g9_collate')
    meta = json.loads(str(fix['meta_json']))
    runs = []
    for case, recs in meta.items():
        groups, attrs = {}, {'mode': str(fix['%s/in/attr/mode' % case])}
        pre = case + '/in/snapshot_'
        for k in fix.files:
            if k.startswith(pre):
                g, d = k[len(case) + 4:].split('/')
                groups.setdefault(g, {})[d] = fix[k]
        for r in recs:
            tag = r['tag']
            kw = {}
            if 'angle_cut' in r:
                kw['angle_cut'] = _param(r['angle_cut'])
            if 'data_type' in r:
                kw['data_type'] = _param(r['data_type'])
            if 'snapshot_number' in r:
                kw['snapshot_number'] = r['snapshot_number']
            hk = '%s/%s/halo_ids' % (case, tag)
            if hk in fix.files:
                kw['halo_ids'] = fix[hk]
            fkw = None
            if r.get('final_counts'):
                fkw = {}
                if 'final_snapshot_numbers' in r:
                    fkw['snapshot_numbers'] = r['final_snapshot_numbers']
            want = {}
            opre = '%s/%s/out/' % (case, tag)
            for k in fix.files:
                if k.startswith(opre):
                    g, d = k[len(opre):].split('/')
                    want.setdefault(g, {})[d] = fix[k]
            runs.append((case, tag, groups, attrs, kw, fkw, want))
    return runs


def central_cases():
    fix = load('g10_progenitors')
    meta = json.loads(str(fix['meta_json']))
    out = []
    for name in sorted({k.split('/')[1] for k in fix.files if k.startswith('central/')}):
        pre = 'central/%s/' % name
        snap = {k: fix[pre + k] for k in ('ids', 'coordinates', 'region_offsets')}
        if pre + 'box_size' in fix.files:
            b = fix[pre + 'box_size']
            snap['box_size'] = [float(v) for v in b] if meta[name + '/box_is_list'] else \
                (float(b) if b.ndim == 0 else b)
        out.append((name, snap, fix[pre + 'halo_positions'], meta[name + '/n'],
                    fix[pre + 'out_ids'], fix[pre + 'out_offsets']))
    return out


def mainprog_cases():
    fix = load('g10_progenitors')
    out = []
    for name in ('i64', 'i32'):
        pre = 'mainprog/%s/' % name
        out.append((name, fix[pre + 'halo_pids'], fix[pre + 'halo_offsets'],
                    fix[pre + 'tracked_pids'], fix[pre + 'tracked_offsets'], fix[pre + 'out']))
    return out
