"""Diagnostic: per-work-group timeline of the partitioned large-halo kernels
(k_part_scatter, k_part_join) on configs[1] (needs the -DOA_STAMPS=1 build:
ORBIT_HIP_LIB=nbody-orbit-analysis_amd/variants/lib_stamps.so)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import orbitanalysis_amd  # noqa
from orbitanalysis_amd.engine import OrbitEngine
from orbitanalysis_amd.synthetic_device import DevicePlummer
from orbitanalysis_amd.utils import hubble_parameter

n = float(os.environ.get('NPART', 1e7)); nh = int(os.environ.get('NHALO', 100))
gen = DevicePlummer(n_halos=nh, n_particles=int(n), dtype='float64')
cos = gen.cosmology
H = hubble_parameter(cos['redshift'], cos['H0'], cos['Omega_m'], cos['Omega_L'])
ex = np.arange(nh)
eng = OrbitEngine()
for s in range(3):
    c = gen.catalogue(s)
    eng.step(gen.snapshot(s), c[0], c[2], H, cos['redshift'], ex, s > 0)
torch.cuda.synchronize()
for which, name in ((1, 'k_part_scatter'), (0, 'k_part_join')):
    k = 8
    buf = np.zeros((1 << 16) * k, dtype=np.uint64)
    got = eng.lib.oa_debug_part_stamps(which, buf.ctypes.data, buf.size)
    assert got > 0, 'not a stamps build'
    t = buf.reshape(-1, k).astype(np.float64)
    t = t[t[:, 0] > 0]
    e = 7 if which else 5
    # rows of the last launch only (an earlier, larger launch leaves stale rows): work-group
    # 0 is in every launch and starts first
    t = t[(t[:, 0] >= t[0, 0] - 500) & (t[:, e] > 0)]
    if which == 0:
        t = t[t[:, 6] > 0]
    t = (t - t[:, :1].min()) / 100.0                       # 100 MHz -> us
    print('%s: %d work-groups, span %.1f us, mean duration %.2f us' % (
        name, len(t), t[:, e].max(), (t[:, e] - t[:, 0]).mean()))
    if which == 0:
        phases = (('loads+clear+bar', 0, 1), ('insert+bar', 1, 2), ('walks+bar', 2, 3),
                  ('lookup chunk 0', 3, 4), ('lookups rest', 4, 6), ('records+state words', 6, 5))
    else:
        # the work-group's first sub-chunk (sub-chunks with halos on the large path only)
        phases = (('sub0 loads+frame', 0, 1), ('count barrier', 1, 2), ('atomics+scan', 2, 3),
                  ('stage+bar', 3, 4), ('copy-out+bar', 4, 5), ('rest of chunk', 5, 7))
        t = t[(t[:, 1] > 0) & (t[:, 5] >= t[:, 1])]
    for nm, a, b in phases:
        d = t[:, b] - t[:, a]
        print('  %-20s mean %6.2f p50 %6.2f p90 %6.2f us' % (nm, d.mean(), *np.percentile(d, [50, 90])))
    # concurrency: work-groups alive over time (start stamp 0 .. end stamp)
    ev = np.concatenate([np.stack([t[:, 0], np.ones(len(t))], 1), np.stack([t[:, e], -np.ones(len(t))], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    alive = np.cumsum(ev[:, 1])
    dt = np.diff(ev[:, 0], append=ev[-1, 0])
    print('  alive: max %d, time-weighted mean %.1f; starts p10/p50/p90 %.1f/%.1f/%.1f us' % (
        alive.max(), (alive * dt).sum() / max(dt.sum(), 1e-9), *np.percentile(t[:, 0], [10, 50, 90])))
