"""Diagnostic: per-work-group phase timeline of one oa_step (needs the -DOA_STAMPS=1
build, e.g. ORBIT_HIP_LIB=nbody-orbit-analysis_amd/variants/lib_stamps.so)."""
import os
import sys
import ctypes
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import orbitanalysis_amd  # noqa
from orbitanalysis_amd import _native as N
from orbitanalysis_amd.engine import OrbitEngine
from orbitanalysis_amd.synthetic_device import DevicePlummer
from orbitanalysis_amd.utils import hubble_parameter

n = float(os.environ.get('NPART', 1e8)); nh = int(os.environ.get('NHALO', 10000))
gen = DevicePlummer(n_halos=nh, n_particles=int(n))
s0, s1 = gen.snapshot(0), gen.snapshot(1)
c0, c1 = gen.catalogue(0), gen.catalogue(1)
cos = gen.cosmology
H = hubble_parameter(cos['redshift'], cos['H0'], cos['Omega_m'], cos['Omega_L'])
z = cos['redshift']
ex = np.arange(nh)
eng = OrbitEngine()
p0 = eng.prepare(s0, c0[0], c0[2], H, z, ex, False)
eng.launch(p0, None)
from orbitanalysis_amd.engine import SnapshotState, layout_of
p1 = eng.prepare(s1, c1[0], c1[2], H, z, ex, True, prev_layout=layout_of(p0, ex))
ws = eng.workspace(p1)
st0 = SnapshotState.of(p0, ex)
for rep in range(3):
    eng.launch(p1, ws, st0)
torch.cuda.synchronize()
ni = len(p1.items)
nw = eng.lib.oa_build_info(0) // 64
NP = 9                                            # STAMP_NP in orbit_hip.hip
sn = NP + 3 * nw + 1
buf = np.zeros(ni * sn, dtype=np.uint64)
got = eng.lib.oa_debug_stamps(buf.ctypes.data, buf.size)
assert got > 0, 'not a stamps build'
tw = buf.reshape(ni, sn).astype(np.float64) * 10.0 / 1000.0   # 100 MHz -> us
tw -= tw[:, 0].min()
t = tw[:, [0, 1, 8, 2, 3, 4, 5, 6, 7]]           # stamps in phase order
w1, w2, w3 = (tw[:, NP + j:NP + 3 * nw:3] for j in range(3))  # per-wave loop ends
for name, w in (('wave skew phase1 end', w1), ('wave skew phase2a end', w2),
                ('wave skew phase2b end', w3)):
    d = w.max(1) - w.min(1)
    m = w.max(1) - w.mean(1)
    print('%-22s max-min mean %6.2f p90 %6.2f | max-mean mean %6.2f us'
          % (name, d.mean(), np.percentile(d, 90), m.mean()))
start, end = t[:, 0], t[:, 8]
print('items', ni, 'kernel span %.1f us' % (end.max()))
for name, a, b in (('phase0', 0, 1), ('phase1(t0)', 1, 2), ('2a-issue+bar', 2, 3),
                   ('walks+bar', 3, 4), ('phase2a(t0)', 4, 5), ('stage+bar', 5, 6),
                   ('phase2b(t0)', 6, 7), ('phase3+', 7, 8), ('total', 0, 8)):
    d = t[:, b] - t[:, a]
    print('%-12s mean %7.2f  p10 %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f us'
          % (name, d.mean(), *np.percentile(d, [10, 50, 90]), d.max()))
dg = buf.reshape(ni, sn)[:, -1]
npend, chain, nst = dg & 0xFFFFF, (dg >> 20) & 0xFFFFF, dg >> 40
for name, v in (('deferred inserts', npend), ('longest walk', chain), ('stashed', nst)):
    print('%-17s mean %8.1f  p50 %6d  p90 %6d  max %6d' % (name, v.mean(), np.percentile(v, 50),
                                                          np.percentile(v, 90), v.max()))
ts = np.linspace(0, end.max(), 12)
print('alive:', [int(((start <= x) & (end > x)).sum()) for x in ts])
# tail: busy fraction of the 256 CUs over the span, and the stretch at the end where
# fewer than 240 items are alive (the last dispatch round's quantisation + skew)
busy = (end - start).sum() / (256 * end.max())
grid = np.linspace(0, end.max(), 2000)
alive = np.array([int(((start <= x) & (end > x)).sum()) for x in grid])
low = np.nonzero(alive[len(grid) // 2:] < 240)[0]
t_low = grid[len(grid) // 2 + low[0]] if len(low) else end.max()
print('busy %.4f of 256 CUs over the span; tail (<240 alive) %.1f us, its idle %.1f CU-us '
      '(%.2f %% of span), last start %.1f us' % (
          busy, end.max() - t_low,
          ((256 - alive[grid >= t_low]) * (grid[1] - grid[0])).sum(),
          100 * ((256 - alive[grid >= t_low]) * (grid[1] - grid[0])).sum() / (256 * end.max()),
          start.max()))
# dispatch gap: the k-th work-group to start after the first 256 takes the CU the k-th
# one to end released (in order), so start[256 + k] - end_sorted[k] estimates the time a
# CU sits between two items
ss, es = np.sort(start), np.sort(end)
if ni > 256:
    g = ss[256:] - es[:ni - 256]
    print('dispatch gap mean %.2f p10 %.2f p50 %.2f p90 %.2f us; first-round start spread %.2f us'
          % (g.mean(), *np.percentile(g, [10, 50, 90]), ss[255] - ss[0]))
