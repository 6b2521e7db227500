"""Helpers shared by the golden-vector tests (fixtures from tools/gen_golden.py)."""
import json
import os

import numpy as np

from conftest import GOLDEN


def load(name):
    return np.load(os.path.join(GOLDEN, name + '.npz'))


def universe(fix):
    from orbitanalysis_amd.synthetic import PlummerSnapshots
    meta = json.loads(str(fix['meta_json']))
    g = dict(meta['gen'])
    for k in ('dtype', 'centre_dtype'):
        if k in g:
            g[k] = np.dtype(g[k])
    u = PlummerSnapshots(**g)
    assert u.input_digest() == str(fix['input_sha256']), 'synthetic generator drifted'
    return u, meta


def groups(fix, prefix=''):
    """{group: {dataset: array}} for keys 'prefix' + 'snapshot_XXX/name'."""
    out = {}
    for k in fix.files:
        if not k.startswith(prefix + 'snapshot_'):
            continue
        g, d = k[len(prefix):].split('/')
        out.setdefault(g, {})[d] = fix[k]
    return out


def assert_same(a, b, what=''):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    assert a.dtype == b.dtype, (what, a.dtype, b.dtype)
    if a.dtype.kind == 'f':
        same = (a == b) | (np.isnan(a) & np.isnan(b))
        assert same.all(), (what, int((~same).sum()), 'mismatches')
    else:
        assert np.array_equal(a, b), what


def assert_groups_equal(got, want):
    assert sorted(got) == sorted(want), (sorted(got), sorted(want))
    for g in want:
        assert sorted(got[g]) == sorted(want[g]), (g, sorted(got[g]), sorted(want[g]))
        for d in want[g]:
            assert_same(got[g][d], want[g][d], g + '/' + d)


# f16 apsis angles compared against reference fixtures in this session, and how many
# differ by one f16 ulp (numpy's arccos is not correctly rounded); conftest prints the
# total at the end of the run and writes it to gpurun_out/angle_mismatch.json
ANGLE_TALLY = {'angles': 0, 'mismatch': 0}

# on-the-fly / module-level angle changes (float32 or float64 arccos) compared against the
# reference's in this session: ulp distance -> count; conftest prints the histogram and
# writes gpurun_out/angle_change_ulps.json.  The bound is the observed maximum.
CHANGE_TALLY = {}
CHANGE_ULP_MAX = 2
# the same split by the dtype arccos ran in ({'float32': {ulps: count}, ...}), and per
# dtype the largest relative error |v - w| / |w| (north_star: 1e-10 for float64)
CHANGE_TALLY_DT = {}
CHANGE_REL_MAX = {}


def check_changes(v, w, dtype, where):
    """Angle changes ``v`` vs the reference's ``w``: NaN where it is NaN, elsewhere within
    CHANGE_ULP_MAX ulps of ``dtype`` (the dtype arccos ran in), tallied by distance."""
    v, w = np.asarray(v), np.asarray(w)
    nan = np.isnan(w)
    assert np.array_equal(np.isnan(v), nan), where
    dt = np.dtype(dtype)
    a, b = v[~nan].astype(dt), w[~nan].astype(dt)
    assert np.all(b >= 0) and np.all(a >= 0), where          # arccos range: bits are monotone
    it = np.int32 if dt.itemsize == 4 else np.int64
    d = np.abs(a.view(it).astype(np.int64) - b.view(it).astype(np.int64))
    per = CHANGE_TALLY_DT.setdefault(dt.name, {})
    for k, c in zip(*np.unique(d, return_counts=True)):
        CHANGE_TALLY[int(k)] = CHANGE_TALLY.get(int(k), 0) + int(c)
        per[int(k)] = per.get(int(k), 0) + int(c)
    nz = b != 0
    if nz.any():
        rel = float(np.max(np.abs(a[nz].astype(np.float64) - b[nz].astype(np.float64)) /
                           np.abs(b[nz].astype(np.float64))))
        CHANGE_REL_MAX[dt.name] = max(CHANGE_REL_MAX.get(dt.name, 0.0), rel)
    assert d.max(initial=0) <= CHANGE_ULP_MAX, (where, int(d.max(initial=0)))
    if dt == np.float64:
        # north_star: float64 values within 1e-10 relative of the reference's
        assert not nz.any() or CHANGE_REL_MAX[dt.name] <= 1e-10, (where, CHANGE_REL_MAX)

