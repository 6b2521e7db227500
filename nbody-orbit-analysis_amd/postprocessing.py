"""Drop-in ``Apsides`` (orbitanalysis/postprocessing.py:8-240): collation of the
orbit path's apsis records into per-halo orbit counts, on the device.

The reference rebuilds every halo's cumulative apsis-ID list with ``np.append`` and
re-runs ``np.unique(return_counts=True)`` on all of it at every snapshot
(postprocessing.py:121-141), an O(S^2) host loop.  Here each collated halo keeps its
sorted-unique (ID, count) list in HBM; a snapshot's kept records are sorted per halo
in LDS and merged in (``oa_collate_step``, csrc/orbit_post.hip), so a snapshot costs
one pass over the state plus the new records.  ``save_final_apsis_counts`` is one
binary-search lookup per element (``oa_retro_counts``).

Files: ``filename`` / ``savefile`` / ``collated_file`` may be HDF5 paths (h5py, as the
reference) or in-memory savefile objects (``savefile.MemorySavefile``).  Halo-sized
bookkeeping (``intersect1d`` / ``myin1d`` of halo ID lists, offsets) stays on the host
like the reference's; every per-particle operation runs in the HIP kernels.  There is
no CPU fallback: without the library or a device these calls raise.
"""
import ctypes
import time

import contextlib

import numpy as np

from . import _native as N
from .utils import myin1d


# ------------------------------------------------------------------ file access
class _H5Store:
    """An HDF5 file opened per access, as the reference opens it (postprocessing.py:
    14, :89, :145, :198): a destination ('a') is created by its first group write,
    not before."""

    def __init__(self, path, mode):
        import h5py
        self._h5py = h5py
        self.path = path
        self.mode = mode
        self._attrs = None
        if mode in ('r', 'r+'):
            self.attrs                    # a missing file fails here, as the reference's open

    @property
    def attrs(self):
        if self._attrs is None:
            with self._h5py.File(self.path, 'r') as hf:
                self._attrs = {k: hf.attrs[k] for k in hf.attrs.keys()}
        return self._attrs

    def group_names(self):
        with self._h5py.File(self.path, 'r') as hf:
            return list(hf.keys())

    def read(self, g, d):
        with self._h5py.File(self.path, 'r') as hf:
            return hf[g][d][:]

    def has(self, g, d):
        with self._h5py.File(self.path, 'r') as hf:
            return d in hf[g]

    def create_group(self, name, datasets):
        with self._h5py.File(self.path, 'a') as hf:
            grp = hf.create_group(name)
            for k, v in datasets.items():
                grp.create_dataset(k, data=v)

    @contextlib.contextmanager
    def session(self):
        """One 'r+' open held across a run of reads and dataset writes, as the
        reference's save_final_apsis_counts holds one (postprocessing.py:196-240): each
        dataset is in the file as soon as it is computed, so an error part-way leaves the
        earlier snapshots' datasets written, as the reference's does."""
        with self._h5py.File(self.path, 'r+') as hf:
            yield _H5Session(hf)


class _H5Session:
    """Reads and dataset writes through one open h5py file (_H5Store.session)."""

    def __init__(self, hf):
        self.hf = hf

    def group_names(self):
        return list(self.hf.keys())

    def read(self, g, d):
        return self.hf[g][d][:]

    def add_dataset(self, g, d, arr):
        self.hf[g].create_dataset(d, data=arr)


class _MemStore:
    def __init__(self, obj):
        self.obj = obj
        self.attrs = obj.attrs

    def group_names(self):
        return sorted(self.obj.groups)

    def read(self, g, d):
        return self.obj.groups[g][d]

    def has(self, g, d):
        return d in self.obj.groups[g]

    def create_group(self, name, datasets):
        self.obj.write_group(name, datasets)

    @contextlib.contextmanager
    def session(self):
        yield self

    def add_dataset(self, g, d, arr):
        grp = self.obj.groups[g]
        if d in grp:
            raise ValueError('dataset %s/%s exists' % (g, d))
        grp[d] = np.asarray(arr)


def _store(f, mode='r'):
    if f is None:
        raise TypeError('a savefile (path or savefile object) is required')
    if isinstance(f, (str, bytes)) or hasattr(f, '__fspath__'):
        return _H5Store(str(f), mode)
    if hasattr(f, 'groups') and hasattr(f, 'attrs'):
        return _MemStore(f)
    raise TypeError('savefile must be a path or a savefile object with groups/attrs')


# ------------------------------------------------------------------ device helpers
def _torch():
    import torch
    return torch


_TORCH_VIEW = {1: np.int8, 2: np.int16, 4: np.int32, 8: np.int64}


def _dev(arr, device):
    """Host array -> device tensor of the same bytes (uint dtypes travel as int views)."""
    torch = _torch()
    a = np.ascontiguousarray(arr)
    if a.dtype.kind in 'ub' or a.dtype == np.float16:
        a = a.view(_TORCH_VIEW[a.dtype.itemsize])
    if a.size == 0:
        return torch.empty(1, dtype=torch.int64, device=device)
    return torch.from_numpy(a).to(device)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _host(t, n, dtype):
    """First n elements of a device tensor as a numpy array of dtype (same itemsize)."""
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return t[:n].cpu().numpy().view(dtype)


def _id_kind(dt, what):
    dt = np.dtype(dt)
    if dt not in N.ID_KIND:
        raise NotImplementedError('%s dtype %s: supported ID dtypes are int64, uint64, '
                                  'int32 and uint32' % (what, dt))
    return N.ID_KIND[dt]


class _CollateState:
    """Cumulative per-halo sorted-unique (key, count) lists in HBM (CSR)."""

    def __init__(self, n_halos, device):
        torch = _torch()
        self.torch = torch
        self.device = device
        self.n = n_halos
        self.off = torch.zeros(n_halos + 1, dtype=torch.int64, device=device)
        self.off_h = np.zeros(n_halos + 1, dtype=np.int64)
        self.keys = torch.empty(1, dtype=torch.int64, device=device)
        self.cnt = torch.empty(1, dtype=torch.int64, device=device)
        self.total = 0

    def merge(self, lib, ids_d, in_kind, key_signed, angles_d, lut_d, src_off, src_cnt,
              events=None):
        """Merge one snapshot's kept apsis IDs into the state (rounds of at most
        COLLATE_CHUNK records per halo, one oa_collate_step each).  ``events``: optional
        list that receives a (start, end) HIP-event pair around every oa_collate_step."""
        torch = self.torch
        dev = self.device
        ch = N.COLLATE_CHUNK
        rounds = int(-(-int(src_cnt.max(initial=0)) // ch))
        src_off_d = _dev(src_off, dev)
        src_cnt_d = _dev(src_cnt, dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        for r in range(rounds):
            chunk = np.clip(src_cnt - r * ch, 0, ch).astype(np.int64)
            # LDS sized to this round's largest chunk (several work-groups share a CU)
            lds_keys = 64
            while lds_keys < int(chunk.max(initial=0)):
                lds_keys <<= 1
            if int(np.diff(self.off_h).max(initial=0)) + ch >= 2 ** 31:
                raise NotImplementedError('a collated halo of 2^31 or more particle IDs')
            base = np.concatenate([[0], np.cumsum(chunk)[:-1]]).astype(np.int64)
            cap = int(chunk.sum())
            i32 = dict(dtype=torch.int32, device=dev)
            w_keys = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
            w_cnt, w_lb, w_fp = (torch.empty(max(cap, 1), **i32) for _ in range(3))
            w_ulen, w_found = (torch.empty(self.n, **i32) for _ in range(2))
            new_off = torch.empty(self.n + 1, dtype=torch.int64, device=dev)
            new_keys = torch.empty(max(self.total + cap, 1), dtype=torch.int64, device=dev)
            new_cnt = torch.empty(max(self.total + cap, 1), dtype=torch.int64, device=dev)
            base_d = _dev(base, dev)
            a = N.CollateArgs(
                n_halos=self.n, in_kind=in_kind, key_signed=key_signed, chunk_start=r * ch,
                lds_keys=lds_keys, apsis_ids=_ptr(ids_d), angles=_ptr(angles_d),
                keep_lut=_ptr(lut_d), src_off=_ptr(src_off_d), src_cnt=_ptr(src_cnt_d),
                new_base=_ptr(base_d), old_keys=_ptr(self.keys), old_cnt=_ptr(self.cnt),
                old_off=_ptr(self.off), n_old=self.total, n_new_cap=cap, w_keys=_ptr(w_keys),
                w_cnt=_ptr(w_cnt), w_lb=_ptr(w_lb), w_fp=_ptr(w_fp), w_ulen=_ptr(w_ulen),
                w_found=_ptr(w_found), new_off=_ptr(new_off), new_keys=_ptr(new_keys),
                new_cnt=_ptr(new_cnt), status=_ptr(status))
            if events is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            N.check(lib.oa_collate_step(ctypes.byref(a), ctypes.c_void_p(st)), 'oa_collate_step')
            if events is not None:
                e1.record()
                events.append((e0, e1))
            self.off, self.keys, self.cnt = new_off, new_keys, new_cnt
            self.off_h = new_off.cpu().numpy()
            self.total = int(self.off_h[-1])
        if rounds and int(status.item()) & N.POST_BOUNDS:
            raise N.NativeError('oa_collate_step: a merged position fell outside its halo '
                                '(OA_POST_BOUNDS): inconsistent collation workspace')

    def lengths(self):
        return np.diff(self.off_h)

    def export(self, lib, key_signed, out_dtype):
        torch = self.torch
        st = torch.cuda.current_stream(self.device).cuda_stream
        n = self.total
        out = torch.empty(max(n * np.dtype(out_dtype).itemsize // 4, 1), dtype=torch.int32,
                          device=self.device)
        N.check(lib.oa_keys_to_ids(_ptr(self.keys), n, key_signed, _id_kind(out_dtype, 'output'),
                                   _ptr(out), ctypes.c_void_p(st)), 'oa_keys_to_ids')
        ids = out.cpu().numpy().view(out_dtype)[:n] if n else np.zeros(0, dtype=out_dtype)
        cnt = _host(self.cnt, n, np.int64)
        return ids, cnt


class Apsides:
    """Collate per-snapshot apsis records (reference: postprocessing.py:8-28)."""

    def __init__(self, filename, device=None):
        self.filename = filename
        st = _store(filename, 'r')
        skeys = st.group_names()
        self.snapshot_numbers = np.array([int(k.split('_')[1]) for k in skeys])
        self.final_halo_ids = st.read(skeys[-1], 'halo_IDs')
        self.mode = st.attrs['mode']
        if 'box_size' in st.attrs:
            self.box_size = st.attrs['box_size']
        self._device = device

    def _dev(self):
        torch = _torch()
        N.load(require_device=True)
        return torch.device(self._device) if self._device is not None else \
            torch.device('cuda', torch.cuda.current_device())

    def collate_apsides(self, halo_ids=None, snapshot_number=None, angle_cut=np.pi / 4,
                        save_final_counts=False, data_type=None, savefile=None, verbose=True):
        """Complete set of orbiting particle IDs and their counts at each snapshot,
        subject to an angle cut (reference docstring: postprocessing.py:34-62)."""
        if verbose:
            t_start = time.time()
        if halo_ids is None:
            halo_ids = self.final_halo_ids
        elif len(np.intersect1d(self.final_halo_ids, halo_ids)) < len(halo_ids):
            self.missing_halo_ids = np.setdiff1d(halo_ids, self.final_halo_ids)
            raise ValueError(
                "The input halo ID list contains IDs of halos (at z=0) "
                "that have not been processed. Refer to the final row of "
                "the `main_branches` attribute to see all IDs (at z=0) "
                "that have been processed.")
        halo_ids = np.asarray(halo_ids)
        if snapshot_number is None:
            sind = len(self.snapshot_numbers) - 1
        else:
            sind = np.argwhere(self.snapshot_numbers == snapshot_number).flatten()[0]

        lib = N.load(require_device=True)
        dev = self._dev()
        src = _store(self.filename, 'r')
        dst = _store(savefile, 'a')
        tag = '{}er'.format(self.mode[:-3])
        f16 = np.arange(65536, dtype=np.uint16).view(np.float16)
        with np.errstate(invalid='ignore'):
            lut_d = _dev((f16 > angle_cut).astype(np.uint8), dev)    # NumPy's own comparison dtype
        state = None
        out_dtype = None
        n_j = len(halo_ids)
        for s in self.snapshot_numbers[:sind + 1]:
            g = 'snapshot_{}'.format('%0.3d' % s)
            halo_ids_current = src.read(g, 'halo_IDs')
            if s != self.snapshot_numbers[-1]:
                halo_ids_final = src.read(g, 'final_descendant_IDs')
            else:
                halo_ids_final = halo_ids_current
            common = np.intersect1d(halo_ids_final, halo_ids)
            hinds1 = myin1d(halo_ids_final, common)
            hinds2 = myin1d(halo_ids, common)
            ids = src.read(g, tag + '_IDs')
            if len(ids) == 0:
                continue
            if state is None:
                out_dtype = np.dtype(ids.dtype if data_type is None else data_type)
                state = _CollateState(n_j, dev)
            if len(hinds2):
                out_dtype = np.result_type(out_dtype, ids.dtype)          # np.append promotion
            if out_dtype.kind not in 'iu':
                raise NotImplementedError('collated ID dtype %s is not an integer type' % out_dtype)
            angles = src.read(g, 'angles')
            if angles.dtype != np.float16:
                raise NotImplementedError('angles must be float16 (the track_orbits layout)')
            hoff = src.read(g, 'region_offsets').astype(np.int64)
            src_off = np.zeros(n_j, dtype=np.int64)
            src_cnt = np.zeros(n_j, dtype=np.int64)
            src_off[hinds2] = hoff[hinds1]
            src_cnt[hinds2] = hoff[np.asarray(hinds1) + 1] - hoff[hinds1]
            key_signed = 1 if out_dtype.kind == 'i' else 0
            ids_d, ang_d = _dev(ids, dev), _dev(angles, dev)
            state.merge(lib, ids_d, _id_kind(ids.dtype, 'apsis ID'), key_signed, ang_d, lut_d,
                        src_off, src_cnt)
            lens_all = state.lengths()
            present = set(int(b) for b in hinds2)
            lens = [int(lens_all[i]) for i in range(n_j) if i in present]
            pids, counts = state.export(lib, key_signed, out_dtype)
            d = {'particle_IDs': pids,
                 '{}_counts'.format(tag): counts,
                 'halo_offsets': np.cumsum([0] + lens)[:-1]}
            if s != self.snapshot_numbers[-1]:
                d['final_descendant_IDs'] = halo_ids_final[hinds1]
            d['halo_IDs'] = halo_ids_current[hinds1]
            d['halo_positions'] = src.read(g, 'region_positions')[hinds1]
            d['halo_velocities'] = src.read(g, 'bulk_velocities')[hinds1]
            d['region_radii'] = src.read(g, 'region_radii')[hinds1]
            dst.create_group('snapshot_{}'.format('%03d' % s), d)
            if verbose:
                print('Snapshot {} collated'.format('%03d' % s))
        if save_final_counts:
            self.save_final_apsis_counts(savefile, verbose=verbose)
        if verbose:
            print('{}ers collated in {} s'.format(self.mode[:-3], round(time.time() - t_start, 3)))
        return

    def save_final_apsis_counts(self, collated_file, snapshot_numbers=None, verbose=True):
        """Save the orbit counts the particles at each snapshot will have by the final
        snapshot (reference docstring: postprocessing.py:179-193)."""
        lib = N.load(require_device=True)
        dev = self._dev()
        torch = _torch()
        with _store(collated_file, 'r+').session() as st:
            self._final_counts(st, lib, dev, torch, snapshot_numbers, verbose)

    def _final_counts(self, st, lib, dev, torch, snapshot_numbers, verbose):
        """save_final_apsis_counts inside one open store session: each snapshot's
        counts are computed on the device and written before the next one's."""
        tag = '{}er'.format(self.mode[:-3])
        skeys = np.array(st.group_names())
        ids_final = st.read(skeys[-1], 'particle_IDs')
        counts_final = st.read(skeys[-1], tag + '_counts').astype(np.int64)
        halo_ids = st.read(skeys[-1], 'halo_IDs')
        offsets_final = np.append(st.read(skeys[-1], 'halo_offsets'), len(ids_final)).astype(np.int64)
        if snapshot_numbers is None:
            skeys_ = skeys[:-1]
        else:
            snap_nums = np.array([int(k.split('_')[-1]) for k in skeys])
            skeys_ = skeys[np.where(np.isin(snap_nums, snapshot_numbers))[0]]
        kind = _id_kind(ids_final.dtype, 'particle ID')
        fin_d = _dev(ids_final, dev)
        foff_d = _dev(offsets_final, dev)
        fcnt_d = _dev(counts_final, dev)
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        for skey in skeys_:
            ids = st.read(skey, 'particle_IDs')
            if ids.dtype != ids_final.dtype:
                raise NotImplementedError('particle ID dtype differs between snapshots')
            desc_ids = st.read(skey, 'final_descendant_IDs')
            offsets = np.append(st.read(skey, 'halo_offsets'), len(ids)).astype(np.int64)
            hinds = np.asarray(myin1d(halo_ids, desc_ids), dtype=np.int64)
            n = len(ids)
            out = torch.zeros(max(n, 1), dtype=torch.float64, device=dev)
            status = torch.zeros(1, dtype=torch.int32, device=dev)
            n_seg = min(len(hinds), len(offsets) - 1)
            # device copies held in locals: a temporary's memory would return to the
            # caching allocator (and be reused) before the kernel runs
            ids_d, off_d, hinds_d = _dev(ids, dev), _dev(offsets, dev), _dev(hinds, dev)
            N.check(lib.oa_retro_counts(_ptr(ids_d), kind, n, _ptr(off_d),
                                        _ptr(hinds_d), n_seg, _ptr(fin_d), _ptr(foff_d),
                                        _ptr(fcnt_d), _ptr(out), _ptr(status), stream),
                    'oa_retro_counts')
            if int(status.item()) & N.POST_MISSING:
                raise ValueError('%s: particle IDs absent from the final snapshot\'s halo '
                                 '(shape mismatch in the reference)' % skey)
            st.add_dataset(skey, '{}_counts_final'.format(tag), _host(out, n, np.float64))
            if verbose:
                print('Final counts saved for {} {}'.format(*(skey.split('_'))))
