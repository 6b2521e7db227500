"""Drop-in ``get_central_particle_ids`` / ``find_main_progenitors``
(orbitanalysis/progenitors.py:5-117): the producer of ``main_branches`` for the
orbit path, on the device.

* ``get_central_particle_ids``: one work-group per region block recentres, takes the
  float64 radius with the reference's expression tree and selects the n nearest by an
  MSB-first radix select plus an LDS sort of the survivors (``oa_central_ids``)
  instead of a full ``argsort`` per block.  Ties in radius are broken by block
  position (NumPy's introsort leaves their order unspecified).
* ``find_main_progenitors``: hash tables in HBM replace ``np.unique`` /
  ``in1d(kind='table')`` / ``myin1d`` (their IDs need not fit a dense table), and a
  per-block LDS tally replaces the per-block ``np.unique(return_counts)`` + argmax
  (``oa_main_progenitors``).  Precondition as in the reference: ``halo_pids`` values
  are unique (``myin1d``) and ``halo_offsets`` start at 0.

Inputs are host NumPy arrays (the reference's interface); results return as NumPy.
No CPU fallback: without the library or a device these calls raise.
"""
import ctypes

import numpy as np

from . import _native as N
from .postprocessing import _dev, _ptr, _host, _id_kind


def _device():
    import torch
    N.load(require_device=True)
    return torch.device('cuda', torch.cuda.current_device())


def _stream(dev):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _box_plan(box, dx_dtype):
    """Per-dim (wrap in float64?, bs, bs/2) exactly as recenter_coordinates evaluates
    ``position[:, dim] > bs/2`` and ``position[...] -= bs`` (utils.py:24-33)."""
    if isinstance(box, (float, np.floating, int, np.integer)):
        box = box * np.ones(3)
    probe = np.zeros(1, dtype=dx_dtype)
    plan = []
    for bs in box:
        wdt = (probe - bs).dtype                      # NumPy promotion (weak Python scalars)
        half = bs / 2
        plan.append((wdt == np.float64, float(np.asarray(bs).astype(wdt)),
                     float(np.asarray(half).astype(wdt))))
    if len(plan) > 3:
        raise ValueError('box_size has more than 3 dimensions')
    return plan


class CentralIds:
    """One ``oa_central_ids`` invocation with its inputs resident on the device
    (built once; ``launch`` may be repeated, e.g. by the benchmark)."""

    def __init__(self, snapshot, halo_positions, n=100):
        import torch
        ids = np.asarray(snapshot['ids'])
        x = np.asarray(snapshot['coordinates'])
        offsets = np.append(np.asarray(snapshot['region_offsets'], dtype=np.int64), len(ids))
        nh = len(offsets) - 1
        if nh == 0:
            raise ValueError('need at least one array to concatenate')
        if len(halo_positions) < nh:
            raise ValueError('fewer halo positions (%d) than region blocks (%d)'
                             % (len(halo_positions), nh))
        n = int(n)
        if n < 0:
            raise NotImplementedError('negative n (argsort(...)[:n] slicing) is not supported')
        if x.dtype not in (np.float32, np.float64):
            raise NotImplementedError('coordinates must be float32 or float64')
        if ids.dtype.itemsize not in (4, 8):
            raise NotImplementedError('IDs must be 4- or 8-byte integers')
        dx_dtype = (x[:1] - halo_positions[0]).dtype
        if dx_dtype not in (np.float32, np.float64):
            raise NotImplementedError('coordinates - positions dtype %s' % dx_dtype)
        lens = np.minimum(np.diff(offsets), n)
        if lens.max(initial=0) > N.CENTRAL_MAX_N:
            raise NotImplementedError('n > %d central particles per halo' % N.CENTRAL_MAX_N)
        out_off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        self.total = int(lens.sum())
        self.lens = lens
        self.id_dtype = ids.dtype
        self.n_particles = len(ids)
        self.lib = N.load(require_device=True)
        self.dev = dev = _device()
        pos = np.asarray([np.asarray(halo_positions[k], dtype=np.float64) for k in range(nh)])
        plan = _box_plan(snapshot['box_size'], dx_dtype) if 'box_size' in snapshot else []
        # every device buffer is held by self until the kernel has run; the radius-key
        # scratch is touched only by blocks the register fast path cannot take
        self.x_d, self.ids_d = _dev(x, dev), _dev(ids, dev)
        self.scratch = torch.empty(max(len(ids), 1), dtype=torch.int64, device=dev)
        self.out = torch.empty(max(self.total * ids.itemsize // 4, 1), dtype=torch.int32, device=dev)
        self.pos_d, self.off_d, self.oo_d = _dev(pos, dev), _dev(offsets, dev), _dev(out_off, dev)
        a = N.CentralArgs(coords=_ptr(self.x_d), coord_f64=int(x.dtype == np.float64),
                          dx_f64=int(dx_dtype == np.float64), positions=_ptr(self.pos_d),
                          ids=_ptr(self.ids_d), id_bytes=ids.itemsize, n_halos=nh,
                          offsets=_ptr(self.off_d), out_offsets=_ptr(self.oo_d),
                          n=int(lens.max(initial=0)), n_box_dims=len(plan),
                          scratch=_ptr(self.scratch), out_ids=_ptr(self.out))
        for d, (w64, bs, half) in enumerate(plan):
            a.wrap_f64[d], a.box[d], a.half[d] = int(w64), bs, half
        self.args = a

    def launch(self):
        N.check(self.lib.oa_central_ids(ctypes.byref(self.args), _stream(self.dev)),
                'oa_central_ids')

    def result(self):
        t = self.total
        central = self.out.cpu().numpy().view(self.id_dtype)[:t] if t else np.zeros(0, self.id_dtype)
        return central, np.cumsum(np.concatenate([[0], self.lens]))[:-1].astype(np.int64)


def get_central_particle_ids(snapshot, halo_positions, n=100):
    """IDs of the n closest particles to each halo centre, arranged in blocks, and
    the block offsets (reference docstring: progenitors.py:7-36)."""
    c = CentralIds(snapshot, halo_positions, n)
    c.launch()
    return c.result()


class MainProgenitors:
    """One ``oa_main_progenitors`` invocation with its inputs resident on the device."""

    def __init__(self, halo_pids, halo_offsets, tracked_pids, tracked_offsets):
        import torch
        hp = np.asarray(halo_pids)
        tp = np.asarray(tracked_pids)
        ho = np.asarray(halo_offsets, dtype=np.int64)
        if len(ho) == 0:
            raise IndexError('halo_offsets is empty')
        to = np.asarray(tracked_offsets, dtype=np.int64)
        nb = len(to)
        if nb == 0:
            raise IndexError('tracked_offsets is empty')
        to_full = np.append(to, len(tp)).astype(np.int64)
        hk = _id_kind(hp.dtype, 'halo particle ID')
        tk = _id_kind(tp.dtype, 'tracked particle ID')
        if N.ID_KIND[np.dtype(np.uint64)] in (hk, tk):
            raise NotImplementedError('uint64 IDs (compared as float64 by in1d) are not supported')
        self.lib = lib = N.load(require_device=True)
        self.dev = dev = _device()
        self.nb = nb
        self.n_halo_pids, self.n_tracked = len(hp), len(tp)
        self.ws = torch.empty(lib.oa_mainprog_workspace_bytes(len(hp), len(tp)) // 8 + 1,
                              dtype=torch.int64, device=dev)
        self.res = torch.empty(nb, dtype=torch.int64, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.hp_d, self.tp_d = _dev(hp, dev), _dev(tp, dev)
        self.ho_d, self.to_d = _dev(ho, dev), _dev(to_full, dev)
        self.args = N.MainProgArgs(
            halo_pids=_ptr(self.hp_d), halo_kind=hk, n_halo_pids=len(hp),
            halo_offsets=_ptr(self.ho_d), n_halos=len(ho), tracked=_ptr(self.tp_d),
            tracked_kind=tk, n_tracked=len(tp), tracked_offsets=_ptr(self.to_d), n_blocks=nb,
            max_block=int(np.diff(to_full).max(initial=0)), tab_keys=_ptr(self.ws),
            result=_ptr(self.res), status=_ptr(self.status))

    def launch(self):
        N.check(self.lib.oa_main_progenitors(ctypes.byref(self.args), _stream(self.dev)),
                'oa_main_progenitors')

    def result(self):
        flags = int(self.status.item())
        if flags & N.POST_SENTINEL:
            raise ValueError('an ID equals INT64_MIN, the hash tables\' empty marker')
        if flags & N.POST_OVERFLOW:
            raise RuntimeError('a tracked block spans more distinct halos than its tally holds')
        r = _host(self.res, self.nb, np.int64)
        return [np.int64(v) if v >= 0 else -1 for v in r]


def find_main_progenitors(halo_pids, halo_offsets, tracked_pids, tracked_offsets):
    """Main progenitor (halo number in ``halo_offsets`` order, or -1) of every tracked
    block, by plurality of its central particles (progenitors.py:59-117)."""
    m = MainProgenitors(halo_pids, halo_offsets, tracked_pids, tracked_offsets)
    m.launch()
    return m.result()
