"""Diagnostic: k_collate_rank per-phase timeline of the last launch (needs the
-DOA_STAMPS=2 build, e.g. ORBIT_HIP_LIB=nbody-orbit-analysis_amd/variants/lib_rstamps.so),
on bench_post's collate workload (1e4 halos, ~5e6 records per snapshot, 10 snapshots)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import orbitanalysis_amd  # noqa
from orbitanalysis_amd import _native as N
from orbitanalysis_amd.postprocessing import _CollateState, _dev
from tools.bench_post import make_track_groups

rng = np.random.default_rng(5)
nh, ns = 10000, int(os.environ.get('NSNAP', 10))
groups = make_track_groups(rng, nh, ns, 500, 10000)
lib = N.load(require_device=True)
dev = torch.device('cuda', 0)
f16 = np.arange(65536, dtype=np.uint16).view(np.float16)
lut_d = _dev((np.nan_to_num(f16.astype(np.float64), nan=-1) > np.pi / 4).astype(np.uint8), dev)
state = _CollateState(nh, dev)
for g in sorted(groups):
    d = groups[g]
    off = d['region_offsets']
    state.merge(lib, _dev(d['pericenter_IDs'], dev), 0, 1, _dev(d['angles'], dev), lut_d,
                off[:-1].astype(np.int64), np.diff(off).astype(np.int64))
torch.cuda.synchronize()
buf = np.zeros(nh * 8, dtype=np.uint64)
assert lib.oa_debug_central_stamps(buf.ctypes.data, buf.size) > 0, 'not a stamps build'
t = buf.reshape(nh, 8).astype(np.float64) * 0.01          # 100 MHz -> us
t -= t[:, 0].min()
print('state before the last snapshot: %d elements' % state.total)
names = ['offsets+records', 'sort', 'rle', 'old tiles', 'scan+writes']
for i, nm in enumerate(names):
    d = t[:, i + 1] - t[:, i]
    print('%-16s mean %6.2f  p50 %6.2f  p90 %6.2f us' % (nm, d.mean(), *np.percentile(d, [50, 90])))
d = t[:, 5] - t[:, 0]
print('total            mean %6.2f us; span %.1f us; mean concurrency %.0f work-groups'
      % (d.mean(), t[:, 5].max(), d.sum() / t[:, 5].max()))
