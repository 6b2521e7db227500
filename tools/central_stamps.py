"""Diagnostic: k_central per-phase timeline (needs the -DOA_STAMPS=1 build, e.g.
ORBIT_HIP_LIB=nbody-orbit-analysis_amd/variants/lib_stamps.so), on bench_post's central
workload (1e8 f32 particles in 1e4 Gaussian blocks, n = 100, periodic box)."""
import os
import sys
import ctypes
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import orbitanalysis_amd  # noqa
from orbitanalysis_amd import _native as N
from orbitanalysis_amd.progenitors import CentralIds

rng = np.random.default_rng(6)
nh, per = int(os.environ.get('NHALO', 10000)), 10000
n = nh * per
centres = rng.uniform(0, 100, (nh, 3)).astype(np.float32)
x = (np.repeat(centres, per, axis=0) + rng.normal(0, 1, (n, 3)).astype(np.float32)) % np.float32(100)
snap = {'ids': rng.permutation(n).astype(np.int64), 'coordinates': x.astype(np.float32),
        'region_offsets': np.arange(nh, dtype=np.int64) * per, 'box_size': 100.0}
c = CentralIds(snap, centres, 100)
for _ in range(3):
    c.launch()
torch.cuda.synchronize()
lib = N.load()
f = lib.oa_debug_central_stamps
buf = np.zeros(nh * 8, dtype=np.uint64)
assert f(buf.ctypes.data, buf.size) > 0, 'not a stamps build'
t = buf.reshape(nh, 8).astype(np.float64) * 0.01          # 100 MHz -> us
t -= t[:, 0].min()
names = ['loads+keys', 'minmax', 'hist', 'scan', 'select', 'rank', 'output']
for i, nm in enumerate(names):
    d = t[:, i + 1] - t[:, i]
    print('%-10s mean %6.2f  p50 %6.2f  p90 %6.2f us' % (nm, d.mean(), *np.percentile(d, [50, 90])))
d = t[:, 7] - t[:, 0]
print('total      mean %6.2f us; span %.1f us' % (d.mean(), t[:, 7].max()))
