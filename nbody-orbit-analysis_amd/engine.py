"""Device engine for the per-snapshot orbit-tagging path.

One ``OrbitEngine`` owns the previous snapshot's device state (IDs, particle
records {r̂, sign(v_r), f16 angle}, block table) and turns each new snapshot into
exactly three stream-ordered native calls:

    oa_bulk_velocity  (only when the catalogue gives no bulk velocity)
    oa_step           fused region_frame + ID join + sign flip + angles
    oa_compact        apsis records in the reference's output order

Host work per snapshot is O(n_halos) table building (no per-particle Python).
Reference behaviour mirrored: track_orbits.py:104-240 (per-snapshot body),
:247-290 (frame), :293-327 (compare), :330-351 (angles), :199-227 (assembly).
"""
import ctypes
import math
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from . import _native as N

F32, F64 = np.dtype(np.float32), np.dtype(np.float64)
# LDS table sizes per work-group item, by r̂ dtype.  One item's LDS is
# the header + max(8-byte cuckoo slots + 2 B/entry insert list, 3 r̂ components per
# entry) + 1 B/entry of signs, within the CU's 160 KB (the table and the r̂ arrays
# overlay each other):
#   float32 r̂: 11776 entries, 16960 slots (load <= 0.69)
#   float64 r̂:  6144 entries, 16896 slots (load <= 0.36)
DEFAULT_ENTRIES = {False: 11776, True: 6144}
DEFAULT_SLOTS = {False: 16960, True: 16896}

_TORCH_FROM_NP = {
    np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
    np.dtype(np.int32): torch.int32, np.dtype(np.uint32): torch.int32,
    np.dtype(np.int64): torch.int64, np.dtype(np.uint64): torch.int64,
    np.dtype(np.float16): torch.float16, np.dtype(np.int16): torch.int16,
    np.dtype(np.uint16): torch.int16,
}
_NP_FROM_TORCH = {torch.float32: F32, torch.float64: F64, torch.int32: np.dtype(np.int32),
                  torch.int64: np.dtype(np.int64), torch.float16: np.dtype(np.float16)}


def np_dtype(x):
    if isinstance(x, torch.Tensor):
        return _NP_FROM_TORCH[x.dtype]
    if isinstance(x, np.ndarray):
        return x.dtype
    return np.asarray(x).dtype


def is_array(x):
    return isinstance(x, (np.ndarray, torch.Tensor))


# ---------------------------------------------------------------- dtype plan
@dataclass
class DtypePlan:
    """NumPy's promotion results for the reference expression tree of one snapshot
    (track_orbits.py:254-288), evaluated on 1-row samples of the real dtypes."""
    coord: np.dtype
    vel: np.dtype
    dx: np.dtype            # x - centre, and r̂
    vb: np.dtype            # v - bulk
    wrap_f64: bool          # recenter arithmetic in float64
    box: tuple = ()         # per-dimension box lengths (float64 values)
    ids: np.dtype = np.dtype(np.int64)
    bulk: np.dtype = F64    # bulk-velocity result dtype
    mass: Optional[np.dtype] = None

    @property
    def state_bytes(self):
        """Bytes of carried state per particle: r̂ (3 x dx dtype) + meta word."""
        return 3 * self.dx.itemsize + 4

    @property
    def torch_dx(self):
        return torch.float64 if self.dx == F64 else torch.float32


def plan_dtypes(snapshot, centre, bulk_cat, H, z):
    coord, vel = np_dtype(snapshot['coordinates']), np_dtype(snapshot['velocities'])
    for name, dt in (('coordinates', coord), ('velocities', vel)):
        if dt not in (F32, F64):
            raise NotImplementedError('%s dtype %s: the device path supports float32/float64'
                                      % (name, dt))
    ids = np_dtype(snapshot['ids'])
    if ids.kind not in 'iu' or ids.itemsize not in (4, 8):
        raise NotImplementedError('ids dtype %s: the device path supports 32/64-bit integers' % ids)
    x1 = np.zeros((1, 3), coord)
    v1 = np.zeros((1, 3), vel)
    c = np.zeros(3, dtype=np.asarray(centre).dtype)
    dx = x1 - c
    if dx.dtype not in (F32, F64):
        raise NotImplementedError('x - centre dtype %s unsupported' % dx.dtype)
    wrap_f64, box = dx.dtype == F64, ()
    if 'box_size' in snapshot:
        bs = snapshot['box_size']
        if isinstance(bs, (float, np.floating, int, np.integer)):
            bs = np.float64(bs) * np.ones(3)          # utils.py:25-26
        elems = list(bs)
        if len(elems) > 3:
            raise ValueError('box_size has more than 3 dimensions')
        kinds = {(dx[:, 0] - e).dtype for e in elems}
        if len(kinds) != 1 or next(iter(kinds)) not in (F32, F64):
            raise NotImplementedError('mixed/unsupported box_size dtypes %s' % kinds)
        wrap_f64 = next(iter(kinds)) == F64
        box = tuple(float(e) for e in elems)
    masses = snapshot['masses']
    mass = None
    if bulk_cat is not None:
        bulk = np.asarray(bulk_cat).dtype
    elif is_array(masses):
        mass = np_dtype(masses)
        if mass not in (F32, F64):
            raise NotImplementedError('masses dtype %s unsupported' % mass)
        m1 = np.ones(1, mass)
        bulk = (np.sum(m1[:, None] * v1, axis=0) / np.sum(m1)).dtype
    else:
        bulk = np.mean(v1, axis=0).dtype
    vb = (v1 - np.zeros(3, bulk)).dtype
    hterm = (H * dx) / (1 + z)
    w = vb.type(0) + hterm
    if hterm.dtype != F64 or w.dtype != F64 or vb not in (F32, F64):
        raise NotImplementedError('Hubble term dtype %s: the device path needs a float64 H '
                                  '(hubble_parameter of Python floats)' % hterm.dtype)
    return DtypePlan(coord=coord, vel=vel, dx=dx.dtype, vb=vb, wrap_f64=bool(wrap_f64),
                     box=box, ids=ids, bulk=bulk, mass=mass)


# ---------------------------------------------------------------- items
GCHUNK = 4096                  # particles per work-group chunk of a large halo


def plan_items(cur_cnt, prev_cnt, entries, hmax=128, out_slot=None, max_pv=None, slots=None,
               cur_off=None):
    """Work-group items of one snapshot, planned by the library's host
    function ``oa_plan_items`` (O(n_halos) C++; no per-halo Python).

    Consecutive halos whose current blocks fit one LDS table (<= ``entries``
    particles, <= ``hmax`` halos, <= ``max_pv`` padded progenitor positions) are
    packed greedily into *items* (k_step).  A halo beyond those limits becomes a
    *global* item: joined through its own table in global memory by as many
    work-groups as it has chunks (k_big_frame / k_big_join).

    Returns (items, global_items, scratch): ITEM_DTYPE arrays (``slot0`` set from
    ``out_slot`` when given) and the apsis-scratch size (one 64-slot segment per
    progenitor row, global items after the packed ones).  An item's ``n_pv`` counts
    its progenitor rows of 64 virtual positions: every progenitor block is padded to
    whole rows, so a row of k_step's phase 2 lies in one block."""
    out, k, n, scratch = _plan(cur_cnt, prev_cnt, entries, hmax, out_slot, max_pv, slots, cur_off)
    return out[:k], out[k:n], scratch


def _plan(cur_cnt, prev_cnt, entries, hmax, out_slot, max_pv, slots, cur_off):
    """oa_plan_items into one ITEM_DTYPE buffer: (items, n_small, n, scratch), the
    packed items first (no copies: prepare uploads items[:n] as they are)."""
    lib = N.load()
    cur = np.ascontiguousarray(cur_cnt, dtype=np.int64)
    prev = np.ascontiguousarray(prev_cnt, dtype=np.int64)
    nh = len(cur)
    off = np.ascontiguousarray(np.concatenate([[0], np.cumsum(cur)[:-1]]) if cur_off is None
                               else cur_off, dtype=np.int64)
    if slots is None:
        slots = 2 * int(entries) + 64
    osl = None if out_slot is None else np.ascontiguousarray(out_slot, dtype=np.int64)
    if max_pv is None:
        max_pv = lib.oa_build_info(3) * lib.oa_build_info(0)
    out = np.empty(max(nh, 1), dtype=N.ITEM_DTYPE)       # every planned row is written
    n_small, scratch = ctypes.c_int64(0), ctypes.c_int64(0)
    n = lib.oa_plan_items(off.ctypes.data, cur.ctypes.data, prev.ctypes.data,
                          None if osl is None else osl.ctypes.data, nh, int(entries),
                          int(slots), int(hmax), int(max_pv), out.ctypes.data, len(out),
                          ctypes.byref(n_small), ctypes.byref(scratch))
    if n < 0:
        raise ValueError(lib.oa_last_error().decode())
    return out, n_small.value, n, int(scratch.value)


def plan_global(glob, cur_cnt, prev_cnt, first_index, compare):
    """Chunk lists and table layout of the global items (k_big_frame / k_big_join),
    vectorised: (item, start, count) chunks of GCHUNK particles of every large halo's
    current block (and, when comparing, of its previous block), and one linear-probing
    table per halo with a power-of-two capacity >= 2 n (load <= 0.5; a 0.7 load, small
    enough for the Infinity Cache, measured slower: 2.26 vs 1.65 ms for configs[1])."""
    h = np.asarray(glob['h0'], dtype=np.int64)
    gi = first_index + np.arange(len(h), dtype=np.int64)

    def chunks(n):
        k = (n + GCHUNK - 1) // GCHUNK
        rep = np.repeat(np.arange(len(n)), k)
        st = (np.arange(k.sum()) - np.repeat(np.cumsum(k) - k, k)) * GCHUNK
        return np.stack([gi[rep], st, np.minimum(GCHUNK, n[rep] - st)], axis=1).astype(np.int64)

    n1 = np.asarray(cur_cnt, dtype=np.int64)[h]
    n2 = np.maximum(np.asarray(prev_cnt, dtype=np.int64)[h], 0) if compare else np.zeros_like(n1)
    two_n = np.maximum(2 * n1, 1)
    cap = np.maximum(64, np.left_shift(1, np.ceil(np.log2(two_n)).astype(np.int64)))
    cap = np.where(cap < two_n, cap * 2, cap)            # guard float rounding
    tab = np.stack([np.cumsum(cap) - cap, cap], axis=1).astype(np.int64).reshape(-1, 2)
    return chunks(n1).reshape(-1, 3), chunks(n2).reshape(-1, 3), tab, int(cap.sum())


# compare steps with packed items only write their records at their final offsets
# from k_step (oa_step_args.direct: decoupled look-back over items), so the step needs
# no oa_compact; ORBIT_DIRECT=0 keeps scratch + oa_compact
DIRECT = os.environ.get('ORBIT_DIRECT', '1') != '0'

PART_FILL = 0.9      # mean fill of a large-halo partition's LDS table at most (k_part_join)


def _pow2_ceil(x):
    x = np.maximum(np.asarray(x, dtype=np.int64), 1)
    return np.left_shift(1, np.ceil(np.log2(x)).astype(np.int64))


def _pow2_floor(x):
    x = np.maximum(np.asarray(x, dtype=np.int64), 1)
    return np.left_shift(1, np.floor(np.log2(x)).astype(np.int64))


# partitions per large halo at least (a power of two): as many as one XCD's CUs run join
# work-groups at once, so an XCD works on one halo at a time
PART_SPREAD = int(_pow2_ceil(int(os.environ.get('ORBIT_PART_SPREAD', 32))))
GPART_W = 16         # int64 per gpart row (orbit_hip.h)


def _gfield(items, name, n):
    """An item-table field as int64 (zeros when a test's stand-in table lacks it)."""
    try:
        return np.asarray(items[name], dtype=np.int64)
    except (KeyError, ValueError):
        return np.zeros(n, dtype=np.int64)


def plan_part(glob, cur_cnt, prev_cnt, part_e, kmax, prev_idx=None, prev_sets=None, n_xcd=8,
              key4=False, td_f64=None):
    """Partition layout of the global items for the partitioned large-halo path
    (k_part_scatter / k_part_join), vectorised.

    A halo with a progenitor block gets K = a power of two >= C / (0.9 part_e) (and
    >= PART_SPREAD) hash partitions of its IDs: a partition's current count is binomial
    with mean <= 0.9 part_e, so the LDS capacity is many standard deviations away (an
    overflow is reported by the kernel and the snapshot re-runs on the global-table
    path).  Its current state goes into the step's current bucket set (part_e entries
    per partition).  Its previous state comes from the previous step's set when that
    step bucketed the progenitor block (``prev_sets``, indexed by the previous
    snapshot's halo number ``prev_idx``; any K: both are powers of two), else from a
    fresh previous set scattered from the position-order state (mean + 8 sqrt(mean) + 64
    entries per partition).  A previous set is inherited only when its keys have the
    step's width (``key4``: 4-byte low words) and r̂ in the step's dtype (``td_f64``).  plist (and its descriptor rows, prow) deals the partitions to the 8 XCDs
    in contiguous runs (work-group b runs on XCD b % 8), so one halo's partitions share
    an L2.  The counters (pcnt) are the current set's, the fresh previous set's, then
    one record counter per previous-block chunk (gchunk2 row, GCHUNK positions; gpart[8]
    is the item's first).  Returns None when no halo needs the join or one needs more
    than ``kmax`` partitions."""
    h = np.asarray(glob['h0'], dtype=np.int64)
    c = np.asarray(cur_cnt, dtype=np.int64)[h]
    p = np.maximum(np.asarray(prev_cnt, dtype=np.int64)[h], 0)
    # the spread floor scales with the halo (one partition per ~1024 particles, a power
    # of two <= PART_SPREAD): a halo just past the item budget gets a few partitions, not
    # PART_SPREAD * part_e entries
    floor = np.minimum(PART_SPREAD, _pow2_floor(np.maximum(c // 1024, 1)))
    K = np.maximum(_pow2_ceil(-(-c // int(part_e * PART_FILL))), floor)
    K = np.where(p > 0, K, 0).astype(np.int64)
    nk = int(K.sum())
    if nk == 0 or K.max() > kmax:
        return None
    ng = len(h)
    gpart = np.zeros((ng, GPART_W), dtype=np.int64)
    gpart[:, 0] = (np.cumsum(K) - K) * int(part_e)
    gpart[:, 1] = K
    gpart[:, 2] = np.cumsum(K) - K
    inh = np.zeros(ng, dtype=bool)
    if prev_sets is not None and prev_idx is not None:
        pc = np.asarray(prev_idx, dtype=np.int64)[h]
        ok = (pc >= 0) & (K > 0) & (bool(prev_sets.key4) == bool(key4))
        if td_f64 is not None:
            ok &= bool(prev_sets.td_f64) == bool(td_f64)
        pk = np.where(ok, prev_sets.K[np.maximum(pc, 0)], 0)
        inh = ok & (pk > 0)
        gpart[inh, 3] = 1
        gpart[inh, 4] = prev_sets.base[pc[inh]]
        gpart[inh, 5] = pk[inh]
        gpart[inh, 6] = int(prev_sets.cap)
        gpart[inh, 7] = prev_sets.cbase[pc[inh]]
    fresh = (K > 0) & ~inh
    mean = p / np.maximum(K, 1)
    cap2 = np.where(fresh, np.ceil(mean + 8 * np.sqrt(mean) + 64), 0).astype(np.int64)
    fsz = np.where(fresh, K * cap2, 0)
    fk = np.where(fresh, K, 0)
    gpart[fresh, 4] = (np.cumsum(fsz) - fsz)[fresh]
    gpart[fresh, 5] = K[fresh]
    gpart[fresh, 6] = cap2[fresh]
    gpart[fresh, 7] = nk + (np.cumsum(fk) - fk)[fresh]
    # record counters: one per previous-block chunk, in gchunk2 row order (plan_global)
    nrow = -(-p // GCHUNK)
    rc0 = nk + int(fk.sum())
    gpart[:, 8] = rc0 + np.cumsum(nrow) - nrow
    g = np.repeat(np.arange(ng), K)
    pp = np.arange(nk) - np.repeat(np.cumsum(K) - K, K)
    per = -(-nk // n_xcd)
    b = np.arange(per * n_xcd)
    idx = (b % n_xcd) * per + b // n_xcd
    okb = idx < nk
    plist = np.zeros((len(b), 2), dtype=np.int32)
    plist[:, 0] = -1
    plist[okb, 0], plist[okb, 1] = g[idx[okb]], pp[idx[okb]]
    # the join's per-work-group descriptor rows (oa_step_args.prow): the item's gpart row,
    # the partition, the item, its scratch base, record chunks and output slot
    gg = g[idx[okb]]
    prow = np.zeros((len(b), GPART_W), dtype=np.int64)
    prow[:, 10] = -1
    prow[okb, :9] = gpart[gg, :9]
    prow[okb, 9], prow[okb, 10] = pp[idx[okb]], gg
    prow[okb, 11] = _gfield(glob, 'scratch_off', ng)[gg]
    prow[okb, 12] = -(-p[gg] // GCHUNK)
    prow[okb, 13] = _gfield(glob, 'slot0', ng)[gg]
    return dict(gpart=gpart, plist=plist, prow=prow, n_cur=nk * int(part_e), n_prev=int(fsz.sum()),
                n_pcnt=rc0 + int(nrow.sum()), rc0=rc0, kmax=int(K.max()), K=K, inherited=inh,
                h=h)


def retry_plan(pr, st):
    """(entries, part) of the re-run of a step whose kernels reported status ``st``:
    a full LDS table halves the items (at the floor every halo takes the global-table
    path, which keys on the full 64-bit ID); an overflowing large-halo partition
    moves the large halos to the global-table path.  (A direct-records look-back
    timeout re-runs the same plan: OrbitEngine.note_status switches direct records
    off.)"""
    from . import _native as N
    if st & N.STATUS_PLAN:
        raise RuntimeError('oa_step: an item exceeds the kernel limits (planner bug)')
    e = pr.entries
    # a partition overflow or a large-halo ID outside the 4-byte keys' high word: the
    # re-run takes the global tables (OrbitEngine.note_status keeps 8-byte keys after)
    part = pr.part and not (st & (N.STATUS_PART_OVERFLOW | N.STATUS_PART_KEYS))
    if st & N.STATUS_TABLE_OVERFLOW:
        e = 0 if e <= 256 else max(256, e // 2)
        # smaller items turn more (and smaller) halos into global items: those take the
        # global tables, sized by each halo, not partitions of part_e entries each
        part = False
    return e, part


def items_single(items):
    """oa_step_args.items_single: 1 when every packed item holds one halo, so oa_step
    launches k_step's one-halo specialisation (ORBIT_SINGLE=0 keeps the general kernel,
    for A/B runs); 0 for any other plan."""
    if len(items) == 0 or os.environ.get('ORBIT_SINGLE', '1') == '0':
        return 0
    return int(bool(np.all(np.asarray(items['h1']) - np.asarray(items['h0']) == 1)))


def set_item_slots(items, out_slot):
    """items['slot0'] = the first output slot among each item's halos [h0, h1), or -1
    (k_gather_items then needs no serial walk over the halo table)."""
    if len(items) == 0:
        return
    nh = len(out_slot)
    has = np.asarray(out_slot) >= 0
    # next halo index >= j with a slot (nh if none)
    nxt = np.full(nh + 1, nh, dtype=np.int64)
    idx = np.where(has, np.arange(nh), nh)
    nxt[:nh] = np.minimum.accumulate(idx[::-1])[::-1]
    first = nxt[items['h0']]
    items['slot0'] = np.where(first < items['h1'], np.asarray(out_slot)[np.minimum(first, nh - 1)], -1)


def check_angles_in(angles_in, n):
    """Checkpoint angles restored on resume must cover the snapshot exactly: the
    kernels read one per particle, and the reference fails on the mismatch too
    (track_orbits.py:229-232 -> calc_angles :342)."""
    if angles_in is not None and len(angles_in) != n:
        raise ValueError('checkpoint angles have %d entries for a snapshot of %d particles'
                         % (len(angles_in), n))


def to_device(x, device, dtype=None):
    """numpy/torch array -> contiguous device tensor (bit-preserving for uint)."""
    if isinstance(x, torch.Tensor):
        t = x
    else:
        a = np.ascontiguousarray(x)
        if dtype is not None:
            a = a.astype(dtype, copy=False)
        if a.dtype.kind == 'u':
            a = a.view(a.dtype.str.replace('u', 'i'))
        t = torch.from_numpy(a)
    return t.to(device, non_blocking=False).contiguous()


class _Staging:
    """Page-locked staging blocks for the host tables of a step (halo table, item plan,
    partition rows): the host fills a block and a kernel on the current stream pulls it
    into device memory (``oa_copy_bytes``).  A copy-engine DMA would queue behind the
    records D2H of an earlier step (track_orbits' pipeline: ~2.3 ms on a heavy pair) and
    hold this step's launch behind it (``profiles/r06/e2e_timeline_*``).  A block is
    reused once the event recorded after its pull has completed."""
    blocks = []

    @classmethod
    def upload(cls, a, device):
        import mmap
        lib = N.load(require_device=True)
        n = int(a.nbytes)
        stream = torch.cuda.current_stream(device)
        blk = next((b for b in cls.blocks
                    if b['cap'] >= n and (b['ev'] is None or b['ev'].query())), None)
        if blk is None:
            cap = max(1 << 20, 1 << max(n - 1, 1).bit_length())
            mm = mmap.mmap(-1, cap)
            arr = np.frombuffer(mm, dtype=np.uint8)
            dev = ctypes.c_void_p()
            N.check(lib.oa_host_register(ctypes.c_void_p(arr.ctypes.data), cap,
                                         ctypes.byref(dev)), 'oa_host_register')
            blk = dict(mm=mm, arr=arr, cap=cap, dev=dev.value, ev=None)
            cls.blocks.append(blk)
        blk['arr'][:n] = a.reshape(-1).view(np.uint8)
        out = torch.empty(n, dtype=torch.uint8, device=device)
        N.check(lib.oa_copy_bytes(ctypes.c_void_p(blk['dev']), ctypes.c_void_p(out.data_ptr()),
                                  n, ctypes.c_void_p(stream.cuda_stream)), 'oa_copy_bytes')
        ev = torch.cuda.Event()
        ev.record(stream)
        blk['ev'] = ev
        return out


# set while an engine with ``table_pull`` prepares a step (OrbitEngine.prepare)
_TABLE_PULL = [False]


def _upload(a, device):
    """Host table -> device tensor of bytes, asynchronous on the current stream.

    Two routes.  A DMA from a page-locked block of torch's caching host allocator (the
    allocator keeps the block until the copy has run) -- the default.  Or, while an
    engine with ``table_pull`` prepares (the pipelined batch driver), ``_Staging``: a
    page-locked block pulled by a kernel.  The batch driver keeps the copy engine busy
    with records D2H, behind which a DMA upload would wait; the on-the-fly stream keeps
    the link's host-to-device direction busy with snapshots, which a kernel's reads
    would have to share."""
    a = np.ascontiguousarray(a)
    if _TABLE_PULL[0]:
        return _Staging.upload(a, device)
    h = torch.empty(a.nbytes, dtype=torch.uint8, pin_memory=True)
    h.numpy()[:] = a.reshape(-1).view(np.uint8)
    return h.to(device, non_blocking=True)


def _up(a, device):
    """``_upload`` of a typed host array: a device tensor of the same dtype and shape.
    (A pageable ``torch.from_numpy(a).to(dev)`` would wait for the stream's queued
    kernels, which a deferred step is still running.)"""
    a = np.ascontiguousarray(a)
    dt = torch.from_numpy(a[:0].reshape(-1)).dtype
    if a.nbytes == 0:
        return torch.empty(a.shape, dtype=dt, device=device)
    return _upload(a, device).view(dt).reshape(a.shape)


_PIN_GRAIN = 1 << 22
N_WS = 3                       # compare-step workspaces in rotation (OrbitEngine)


def _pinned(n, dtype):
    """A page-locked host tensor of n elements from torch's caching host allocator, the
    block rounded up to a power of two (>= 4 MiB): snapshots' record counts differ, and
    a block that fits the next request is reused instead of page-locking a new one
    (that, not the DMA, is what held the D2H of the records to ~20 GB/s; a 4-MiB grain
    still page-locked a new block whenever the count crossed one, ~3-7 ms each)."""
    itemsize = torch.empty(0, dtype=dtype).element_size()
    nb = max(1 << max(int(n) * itemsize - 1, 1).bit_length(), _PIN_GRAIN)
    return torch.empty(nb // itemsize, dtype=dtype, pin_memory=True)[:n]


class PendingFetch:
    """Records on their way to the host (OrbitEngine.fetch_async)."""

    def __init__(self, done, h_off, h_ids, h_ang, ids_dtype):
        self.done, self.h_off, self.h_ids, self.h_ang = done, h_off, h_ids, h_ang
        self.ids_dtype = ids_dtype

    def wait(self):
        self.done.synchronize()
        offsets = self.h_off.numpy()
        if self.h_ids is None:
            return offsets, np.zeros(0, dtype=self.ids_dtype), np.zeros(0, dtype=np.float16)
        return offsets, ids_as(self.h_ids.numpy(), self.ids_dtype), \
            self.h_ang.numpy().view(np.float16)


def ids_as(raw, ids_dtype):
    """Records' IDs (the workspace's integer width) in the previous snapshot's ID dtype,
    the dtype of the reference's ids_prev_[apsis_inds] (track_orbits.py:315-316): a
    widened previous state (int32 -> int64 between snapshots) narrows back exactly."""
    ids_dtype = np.dtype(ids_dtype)
    if raw.dtype.itemsize == ids_dtype.itemsize:
        return raw.view(ids_dtype)
    return raw.view(np.dtype('%s%d' % (ids_dtype.kind, raw.dtype.itemsize))).astype(ids_dtype)


def meta_angles(meta):
    """float16 angles held in the low half of device meta words -> host array."""
    return (meta & 0xFFFF).cpu().numpy().astype(np.uint16).view(np.float16)


def _ptr(t):
    return None if t is None else t.data_ptr()


@dataclass
class BucketSet:
    """One step's state of its partitioned large halos, by hash partition (k_part_*,
    orbit_hip.h): per entry the ID, position | sign << 30, state word and r̂; part_e
    entries per partition.  Per halo of that step: K (0: not bucketed), base entry and
    first counter.  The position-order state arrays of those halos are not written
    (OrbitEngine.unbucket restores them on demand); ``restored`` marks halos done."""
    key: torch.Tensor
    pos: torch.Tensor
    meta: torch.Tensor
    rh: torch.Tensor
    cnt: torch.Tensor
    K: np.ndarray
    base: np.ndarray
    cbase: np.ndarray
    cap: int
    td_f64: bool
    key4: bool = False                  # keys are the IDs' low words (oa_step_args.part_key4)
    restored: Optional[np.ndarray] = None


@dataclass
class SnapshotState:
    """Device state a snapshot leaves for the next one (track_orbits.py:234-240)."""
    ids: torch.Tensor
    rhat: torch.Tensor
    meta: torch.Tensor
    starts: np.ndarray
    counts: np.ndarray
    exists: np.ndarray
    plan: DtypePlan
    buckets: Optional[BucketSet] = None

    @classmethod
    def of(cls, pr, exists, ids=None):
        """The state a prepared (and launched) step leaves for the next one."""
        return cls(ids=pr.snap['ids'] if ids is None else ids, rhat=pr.rhat, meta=pr.meta,
                   starts=pr.starts, counts=pr.counts, exists=np.asarray(exists), plan=pr.plan,
                   buckets=pr.buckets)

    def layout(self):
        """The ``prev_layout`` of the next step's ``prepare``."""
        return (self.starts, self.counts, self.exists, self.plan, self.ids.numel(), self.buckets)


def layout_of(pr, exists):
    """``prev_layout`` for the step after the prepared step ``pr`` (bench / tools)."""
    return (pr.starts, pr.counts, np.asarray(exists), pr.plan, pr.n, pr.buckets)


@dataclass
class StepResult:
    """A compare step's records.  They live in one of the engine's N_WS workspaces and
    are valid until the step N_WS later reuses it: ``fetch`` / ``fetch_async`` of an
    older result raise instead of returning another snapshot's records."""
    n_slots: int
    has_prog: np.ndarray                       # bool per current halo
    offsets: Optional[torch.Tensor] = None     # device int64 [n_slots+1]
    apsis_ids: Optional[torch.Tensor] = None   # device, capacity >= total
    apsis_ang: Optional[torch.Tensor] = None   # device int16 (f16 bits)
    total: Optional[torch.Tensor] = None       # device int64 scalar
    halos: Optional[torch.Tensor] = None       # device halo table (bulk written on device)
    apsis_pos: Optional[torch.Tensor] = None   # device int32 previous-state rows (optional)
    extra: dict = field(default_factory=dict)
    ws: object = None                          # the workspace holding the records
    gen: int = 0                               # its launch count when they were written
    done: object = None                        # event after its kernels (compare steps)
    pending: object = None                     # (ctx, prep) until OrbitEngine.settle
    ws_idx: int = 0                            # which of the engine's workspaces

    def check_fresh(self):
        if self.ws is not None and self.ws.gen != self.gen:
            raise RuntimeError('StepResult is stale: its workspace was reused by a later '
                               'step (fetch a result before N_WS later steps ran)')


@dataclass
class PreparedStep:
    """Everything one snapshot step needs on the device, built by OrbitEngine.prepare."""
    plan: DtypePlan
    n: int
    starts: np.ndarray
    counts: np.ndarray
    has_prog: np.ndarray
    items: np.ndarray              # packed items, then global (large-halo) items
    n_small: int
    scratch: int
    compare: bool
    n_prev: int = 0
    entries: int = 0               # per-item particle budget the plan used
    part: bool = False             # large halos on the partitioned path (k_part_*)
    halos: Optional[torch.Tensor] = None
    d_items: Optional[torch.Tensor] = None
    glob: dict = field(default_factory=dict)       # device chunk lists / tables
    rhat: Optional[torch.Tensor] = None
    meta: Optional[torch.Tensor] = None
    angles_in: Optional[torch.Tensor] = None
    halo_list: Optional[torch.Tensor] = None
    bulk_computed: bool = False
    buckets: Optional['BucketSet'] = None          # this step's current bucket set
    unbucket_prev: Optional[np.ndarray] = None     # previous halos to restore first
    snap: dict = field(default_factory=dict)
    args: N.StepArgs = field(default_factory=N.StepArgs)
    cargs: N.CompactArgs = field(default_factory=N.CompactArgs)

    @property
    def n_global(self):
        return len(self.items) - self.n_small


class _HostWords:
    """Page-locked host words the device stores into (``oa_post_status``): registered
    pages of 16-byte slots (status int32 at +0, record count int64 at +8), one slot per
    workspace, returned to the page's free list when the workspace goes."""
    PAGE = 4096
    pages = []

    @classmethod
    def take(cls, lib):
        for pg in cls.pages:
            if pg['free']:
                return pg, pg['free'].pop()
        import mmap
        mm = mmap.mmap(-1, cls.PAGE)
        arr = np.frombuffer(mm, dtype=np.uint8)
        dev = ctypes.c_void_p()
        N.check(lib.oa_host_register(ctypes.c_void_p(arr.ctypes.data), cls.PAGE,
                                     ctypes.byref(dev)), 'oa_host_register')
        pg = dict(mm=mm, arr=arr, dev=dev.value, free=list(range(cls.PAGE // 16 - 1, -1, -1)))
        cls.pages.append(pg)
        return pg, pg['free'].pop()


class Workspace:
    """Scratch of compare steps, kept by the engine and grown on demand (capacities are
    high-water marks, so a steady stream of snapshots allocates nothing)."""

    FIELDS = ('scratch', 'n_prev', 'n_slots', 'n_items')

    def __init__(self, device, id_torch_dtype, scratch, n_prev, n_slots, n_items,
                 positions=False):
        def e(n, dt):
            return torch.empty(max(int(n), 1), dtype=dt, device=device)
        self.device, self.id_dtype, self.positions = device, id_torch_dtype, bool(positions)
        self.cap = dict(scratch=int(scratch), n_prev=int(n_prev), n_slots=int(n_slots),
                        n_items=int(n_items))
        self.scratch_ids = e(scratch, id_torch_dtype)
        self.scratch_ang = e(scratch, torch.int16)
        self.seg_count = e(scratch // 64 + 1, torch.uint8)
        self.halo_count = e(n_slots, torch.int32)
        self.item_count = e(n_items, torch.int32)
        self.status = e(1, torch.int32)
        self.gen = 0                        # launches that wrote this workspace
        self.offsets = e(n_slots + 1, torch.int64)
        self.out_ids = e(n_prev, id_torch_dtype)
        self.out_ang = e(n_prev, torch.int16)
        self.total = e(1, torch.int64)
        # apsis records' previous-state indices (the sharded driver's merge key)
        self.scratch_pos = e(scratch, torch.int32) if positions else None
        self.out_pos = e(n_prev, torch.int32) if positions else None
        self.status.zero_()
        # the status word and record count of the last launch, stored into page-locked
        # host words by a kernel behind the step (post_status): OrbitEngine.settle reads
        # them after the step's event, with no stream sync and no copy engine in between
        self.h_status = np.zeros(1, np.int32)
        self.h_total = np.zeros(1, np.int64)
        self._hw = None
        self.copy_done = None               # event after the last D2H of its records
        self.scratch_rk = None              # partitioned halos' record positions (rk())
        self.lookback, self.lb_epoch = None, 0  # direct records' item words (lookback())

    def post_status(self, lib, stream):
        """Queue the status word and record count to the host words on ``stream``
        (``oa_post_status``).  A D2H copy there would wait for the copy engine, which
        may still be moving an earlier step's records (track_orbits' pipeline), and
        hold the host's settle, and so the next launch, behind it."""
        if self._hw is None:
            import weakref
            pg, k = _HostWords.take(lib)
            self._hw = (pg['dev'] + 16 * k, pg['arr'])
            self.h_status = pg['arr'][16 * k:16 * k + 4].view(np.int32)
            self.h_total = pg['arr'][16 * k + 8:16 * k + 16].view(np.int64)
            weakref.finalize(self, pg['free'].append, k)
        dev = self._hw[0]
        N.check(lib.oa_post_status(ctypes.c_void_p(self.status.data_ptr()),
                                   ctypes.c_void_p(self.total.data_ptr()),
                                   ctypes.c_void_p(dev), ctypes.c_void_p(dev + 8),
                                   ctypes.c_void_p(stream.cuda_stream)), 'oa_post_status')

    @staticmethod
    def need(pr):
        return dict(scratch=pr.scratch, n_prev=pr.n_prev, n_slots=int(pr.has_prog.sum()),
                    n_items=len(pr.items))

    @classmethod
    def for_step(cls, pr, device):
        dt = torch.int64 if pr.plan.ids.itemsize == 8 else torch.int32
        return cls(device, dt, **cls.need(pr))

    def fits(self, pr, positions=False):
        dt = torch.int64 if pr.plan.ids.itemsize == 8 else torch.int32
        return dt == self.id_dtype and self.positions >= bool(positions) and \
            all(self.cap[k] >= v for k, v in self.need(pr).items())

    def reset(self, n_slots):
        """Per-launch zeroing (the status word accumulates: callers clear it)."""
        self.halo_count[:max(n_slots, 1)].zero_()

    def lookback_words(self, n):
        """(pointer, epoch) of the direct records' look-back words for a launch of ``n``
        items: kept between launches and tagged per launch (oa_step_args.lb_epoch), so
        they are zeroed only when the buffer grows or the 16-bit epoch would repeat."""
        if self.lookback is None or self.lookback.numel() < n or self.lb_epoch >= 0xFFFF:
            if self.lookback is None or self.lookback.numel() < n:
                self.lookback = torch.zeros(max(int(n), 1), dtype=torch.int64, device=self.device)
            else:
                self.lookback.zero_()
            self.lb_epoch = 0
        self.lb_epoch += 1
        return self.lookback.data_ptr(), self.lb_epoch

    def rk(self):
        """Per apsis-scratch slot, the position of a partitioned halo's record in its
        previous-block chunk (oa_step_args.scratch_rk), allocated on first use."""
        n = self.cap['scratch']
        if self.scratch_rk is None or self.scratch_rk.numel() < n:
            self.scratch_rk = torch.empty(max(n, 1), dtype=torch.int16, device=self.device)
        return self.scratch_rk.data_ptr()


class OrbitEngine:
    """Per-snapshot device pipeline with carried state (see module docstring)."""

    def __init__(self, mode='pericentric', device=None, lds_entries=None, lds_slots=None,
                 hmax=None):
        if mode not in N.MODE:
            raise ValueError("Orbit detection mode not recognized. Please specify either "
                             "'pericentric' or 'apocentric'.")
        self.lib = N.load(require_device=True)
        self.device = torch.device(device if device is not None else 'cuda')
        self.mode = mode
        env = os.environ.get
        # LDS table sizes: one item fills one CU's 160 KB; the defaults
        # depend on the r̂ dtype, an explicit value applies to both
        self.entries_cfg = int(lds_entries or env('ORBIT_LDS_ENTRIES', 0)) or None
        self.slots_cfg = int(lds_slots or env('ORBIT_LDS_SLOTS', 0)) or None
        self.hmax = min(int(hmax or env('ORBIT_HMAX', 1 << 30)), self.lib.oa_build_info(1))
        self.max_pv = self.lib.oa_build_info(3) * self.lib.oa_build_info(0)
        self.max_lds = self.lib.oa_max_lds_bytes()
        for f64 in (False, True):
            self.table_sizes(f64)                   # validates the LDS budget
        self.prev: Optional[SnapshotState] = None
        # N_WS compare-step workspaces, in rotation between snapshots (step): a snapshot's
        # records can still be on their way to the host (fetch_async) while the next
        # snapshots' kernels write the others; with three, the D2H of step s - 1 has two
        # steps' time before step s + 2 reuses its workspace (a copy slower than one
        # step no longer holds the next kernel back)
        self._wss = [None] * N_WS
        self._wsi = 0
        self._pending = None                # a deferred step not yet settled (step)
        # apsis records also carry their previous-state row (ShardedEngine's merge)
        self.emit_positions = False
        # large halos of compare steps: hash partitions joined in LDS (k_part_*);
        # ORBIT_PART=0 keeps them on the per-halo global tables (k_big_*)
        self.part_large = env('ORBIT_PART', '1') != '0'
        # partition capacity: 4096 entries in 6144 slots (~74 KB of LDS: two join
        # work-groups per CU); at most oa_build_info(4)
        self.part_e = min(int(env('ORBIT_PART_ENTRIES', 4096)), self.lib.oa_build_info(4))
        self.part_slots = int(env('ORBIT_PART_SLOTS', 0)) or self.part_e + self.part_e // 2
        self.part_kmax = self.lib.oa_build_info(5)
        if self.lib.oa_build_info(7) != GCHUNK:
            raise N.NativeUnavailable('record chunk %d != engine.GCHUNK %d'
                                      % (self.lib.oa_build_info(7), GCHUNK))
        # 4-byte bucket keys (the IDs' low words) while every large-halo ID's high word
        # is 0; a step that meets another one re-runs and the engine keeps 8-byte keys
        self.part_key4 = env('ORBIT_PART_KEY4', '1') != '0'
        # packed-only compare steps write their records from k_step (direct records)
        self.direct = DIRECT
        # direct records' look-back poll bound (0: the library default); tests set 1 to
        # force OA_STATUS_LOOKBACK and the re-run through oa_compact
        self.lb_spin_max = 0
        # per-step tables pulled by a kernel instead of a DMA (_upload); the pipelined
        # batch driver sets it for its run
        self.table_pull = False
        # diagnostics (tools/bench_e2e.py --timeline): a list collecting (start, end) timing
        # events of each fetch_async's copies on the copy stream; None: off
        self.copy_events = None

    def _advance_ws(self):
        """The current workspace index, then rotate to the next one."""
        i = self._wsi
        self._wsi = (self._wsi + 1) % len(self._wss)
        return i

    def note_status(self, st):
        """Run-wide switches a step's status word turns off before its re-run."""
        if st & N.STATUS_LOOKBACK:
            self.direct = False
        if st & N.STATUS_PART_KEYS:
            self.part_key4 = False

    def table_sizes(self, dx_f64, entries=None):
        """(entries, slots) of one k_step item for a float32 / float64 r̂."""
        e = int(entries or self.entries_cfg or DEFAULT_ENTRIES[bool(dx_f64)])
        s = int(self.slots_cfg or max(DEFAULT_SLOTS[bool(dx_f64)], e + 1))
        need = self.lib.oa_step_lds_bytes(e, s, int(bool(dx_f64)))
        if need > self.max_lds:
            raise ValueError('LDS table (%d entries, %d slots, %s r̂) needs %d bytes > device '
                             'limit %d' % (e, s, 'float64' if dx_f64 else 'float32', need,
                                           self.max_lds))
        return e, s

    @property
    def entries(self):
        return self.table_sizes(False)[0]

    @property
    def _ws(self):
        return self._wss[self._wsi]

    def workspace(self, pr, idx=None):
        """The engine's current compare-step workspace (or workspace ``idx``), grown to
        fit ``pr``."""
        idx = self._wsi if idx is None else idx
        ws = self._wss[idx]
        if ws is None or not ws.fits(pr, self.emit_positions):
            old = ws.cap if ws is not None else {}
            need = Workspace.need(pr)
            cap = {k: max(need[k], old.get(k, 0)) for k in need}
            dt = torch.int64 if pr.plan.ids.itemsize == 8 else torch.int32
            nws = Workspace(self.device, dt, positions=self.emit_positions, **cap)
            if ws is not None:
                nws.gen, nws.copy_done = ws.gen, ws.copy_done
                nws.lookback, nws.lb_epoch = ws.lookback, ws.lb_epoch
            ws = self._wss[idx] = nws
        return ws

    def reset(self):
        self.settle()
        self.prev = None

    # ------------------------------------------------------------------ tables
    def build_tables(self, snapshot, centres, bulk_cat, exists, compare, prev_layout=None,
                     entries=None, slots=None):
        n = int(snapshot['ids'].numel()) if isinstance(snapshot['ids'], torch.Tensor) \
            else len(snapshot['ids'])
        starts = np.ascontiguousarray(np.asarray(snapshot["region_offsets"], dtype=np.int64).reshape(-1))
        ends = np.append(starts[1:], n)
        counts = ends - starts
        nh = len(starts)
        if nh != len(exists):
            raise ValueError('region_offsets has %d blocks for %d halos' % (nh, len(exists)))
        if nh and (np.any(counts < 0) or starts[0] < 0 or ends[-1] > n):
            raise ValueError('region_offsets must be non-decreasing block starts within [0, N]')
        # columns first (contiguous), then the 96-byte rows in one host pass (C++)
        prev_off = np.zeros(nh, dtype=np.int64)
        prev_cnt = np.full(nh, -1, dtype=np.int64)
        out_slot = np.full(nh, -1, dtype=np.int64)
        has_prog = np.zeros(nh, dtype=bool)
        prev_idx = np.full(nh, -1, dtype=np.int64)     # the progenitor's previous halo number
        if compare:
            p_starts, p_counts, pe = prev_layout[0], prev_layout[1], np.asarray(prev_layout[2])
            if len(pe) == nh and np.array_equal(pe, exists):
                # the same halos as the previous snapshot (the usual case): no search
                prev_off[:] = p_starts
                prev_cnt[:] = p_counts
                out_slot[:] = prev_idx[:] = np.arange(nh)
                has_prog[:] = True
            elif len(pe):
                p = np.searchsorted(pe, exists)
                pc = np.minimum(p, len(pe) - 1)
                has_prog = (p < len(pe)) & (pe[pc] == exists)
                prev_off[has_prog] = p_starts[p[has_prog]]
                prev_cnt[has_prog] = p_counts[p[has_prog]]
                out_slot[has_prog] = np.arange(int(has_prog.sum()))
                prev_idx[has_prog] = p[has_prog]
        cen = np.ascontiguousarray(centres, dtype=np.float64).reshape(nh, 3)
        blk = None if bulk_cat is None else \
            np.ascontiguousarray(bulk_cat, dtype=np.float64).reshape(nh, 3)
        halos = np.empty(nh, dtype=N.HALO_DTYPE)
        if nh:
            N.check(self.lib.oa_build_halos(starts.ctypes.data, counts.ctypes.data,
                                            prev_off.ctypes.data, prev_cnt.ctypes.data,
                                            out_slot.ctypes.data, cen.ctypes.data,
                                            None if blk is None else blk.ctypes.data, nh,
                                            halos.ctypes.data), 'oa_build_halos')
        buf, k, n_it, scratch = _plan(counts, prev_cnt, entries, self.hmax, out_slot,
                                      self.max_pv, slots, starts)
        self._prev_idx = prev_idx
        return halos, buf[:n_it], k, scratch, starts, counts, has_prog

    # ------------------------------------------------------------------ step
    def step(self, snapshot, centres, bulk_cat, H, z, exists, compare, angles_in=None,
             angles_layout=None, defer=False):
        """Process one snapshot.  ``compare`` is the reference's ``i > istart``.
        ``angles_layout``: the row layout a resumed checkpoint was written in (None:
        the snapshot's own rows, the only layout a single GPU reads).

        ``defer``: return without waiting for the kernels.  The step's status word (an
        LDS table overflow asks for a re-planned re-run) is then checked by ``settle``:
        the next ``step`` does it after planning its own snapshot on the host, so that
        planning overlaps this snapshot's kernels; ``fetch*``, ``angles`` and
        ``bulk_velocities`` settle first too.  A re-run replaces the step's records and
        state in place (same workspace), exactly as the synchronous path would have."""
        exists = np.asarray(exists)
        if angles_in is not None and angles_layout is not None:
            from .sharding import check_layout
            check_layout(angles_layout, None)
        if compare and self.prev is None:
            raise RuntimeError('compare step without a previous snapshot')
        dev = self.device
        snap = dict(snapshot)
        for k in ('ids', 'coordinates', 'velocities'):
            snap[k] = to_device(snapshot[k], dev)
        if is_array(snapshot['masses']):
            snap['masses'] = to_device(snapshot['masses'], dev)
        ctx = dict(snap=snap, centres=centres, bulk_cat=bulk_cat, H=H, z=z, exists=exists,
                   compare=compare, angles_in=angles_in, plan_src=snapshot,
                   prev=self.prev if compare else None)
        prep = self._prepare_ctx(ctx, None, True)
        if self._pending is not None and self.settle(self._pending):
            # the previous step was re-planned: its layout / bucket sets changed
            ctx['prev'] = self.prev if compare else None
            prep = self._prepare_ctx(ctx, None, True)
        if defer:
            res = self._launch_ctx(ctx, prep)
            if compare:
                res.pending = (ctx, prep)
                self._pending = res
        else:
            res, prep = self._run_ctx(ctx, prep)
        self._set_prev(ctx, prep)
        if compare:
            self._advance_ws()              # the next snapshot writes the next workspace
        return res

    def _prepare_ctx(self, ctx, entries, part):
        p = ctx['prev']
        layout = None if p is None else p.layout()
        return self.prepare(ctx['snap'], ctx['centres'], ctx['bulk_cat'], ctx['H'], ctx['z'],
                            ctx['exists'], ctx['compare'], angles_in=ctx['angles_in'],
                            plan_src=ctx['plan_src'], prev_layout=layout, entries=entries,
                            part=part)

    def _launch_ctx(self, ctx, prep, idx=None):
        """Launch a prepared step into workspace ``idx`` (default: the current one); a
        compare step also queues the copy of its status word and record count to
        page-locked host memory behind an event."""
        if not ctx['compare']:
            return self.launch(prep, None)
        idx = self._wsi if idx is None else idx
        ws = self.workspace(prep, idx)
        ws.status.zero_()
        if ws.copy_done is not None:
            # the records of the last step in this workspace may still be crossing PCIe
            torch.cuda.current_stream(self.device).wait_event(ws.copy_done)
            ws.copy_done = None
        res = self.launch(prep, ws, prev=ctx['prev'])
        res.ws_idx = idx
        ws.post_status(self.lib, torch.cuda.current_stream(self.device))
        res.done = torch.cuda.Event()
        res.done.record(torch.cuda.current_stream(self.device))
        return res

    def _run_ctx(self, ctx, prep, res=None):
        """Launch, wait, and re-plan until the kernels report no overflow."""
        idx = res.ws_idx if res is not None else None
        for attempt in range(10):
            r = self._launch_ctx(ctx, prep, idx)
            if not ctx['compare']:
                return r, prep
            r.done.synchronize()
            st = int(r.ws.h_status[0])
            if not st:
                if res is not None:          # the deferred result object, now re-filled
                    res.__dict__.update({k: v for k, v in r.__dict__.items()})
                    r = res
                r.pending = None
                return r, prep
            self.note_status(st)
            prep = self._prepare_ctx(ctx, *retry_plan(prep, st))
        raise RuntimeError('LDS hash tables kept overflowing')

    def _set_prev(self, ctx, prep):
        self.prev = SnapshotState.of(prep, ctx['exists'], ids=ctx['snap']['ids'])

    def step_ready(self, res):
        """Without waiting: None while a step's kernels run, else whether its records
        are final (False: its kernels asked for a re-planned re-run).  Error paths use
        it to avoid blocking on, or launching more work after, a failure."""
        if res.done is not None and not res.done.query():
            return None
        if getattr(res, 'pending', None) is not None:
            return not int(res.ws.h_status[0])
        return True

    def settle(self, res=None):
        """Wait for a deferred step (default: the pending one) and re-run it if its
        kernels reported an overflow.  Returns True when it was re-run (its state
        replaced).  Only the engine's latest step can be pending."""
        res = self._pending if res is None else res
        if res is None or getattr(res, 'pending', None) is None:
            return False
        ctx, prep = res.pending
        res.done.synchronize()
        if not int(res.ws.h_status[0]):
            res.pending = None
            if self._pending is res:
                self._pending = None
            return False
        self._pending = None
        st = int(res.ws.h_status[0])
        self.note_status(st)
        _, prep = self._run_ctx(ctx, self._prepare_ctx(ctx, *retry_plan(prep, st)), res=res)
        self._set_prev(ctx, prep)
        return True

    def prepare(self, *args, **kw):
        """Host half of a step (``_prepare``), its table uploads routed by ``table_pull``
        (``_upload``)."""
        old = _TABLE_PULL[0]
        _TABLE_PULL[0] = bool(self.table_pull)
        try:
            return self._prepare(*args, **kw)
        finally:
            _TABLE_PULL[0] = old

    def _prepare(self, snap, centres, bulk_cat, H, z, exists, compare, angles_in=None,
                 plan_src=None, prev_layout=None, entries=None, part=True):
        """Host half of a step: dtype plan, halo/item tables, device uploads.

        ``snap`` holds device tensors for ids/coordinates/velocities(/masses);
        ``prev_layout`` (starts, counts, exists, plan) defaults to the engine state.
        ``entries`` overrides the per-item particle budget of the plan (0: every halo
        on the large-halo path); ``part`` = False keeps large halos on the global-table
        path (k_big_*) instead of the partitioned one (k_part_*)."""
        dev = self.device
        exists = np.asarray(exists)
        plan = plan_dtypes(plan_src if plan_src is not None else snap,
                           centres[0] if len(centres) else np.zeros(3),
                           None if bulk_cat is None else bulk_cat[0], H, z)
        if prev_layout is None and compare:
            prev_layout = self.prev.layout()
        prev_sets = prev_layout[5] if compare and len(prev_layout) > 5 else None
        if compare:
            # a snapshot whose r̂ or ID dtype is wider than the previous one's compares in
            # the wider dtype, as NumPy promotes (launch widens the previous state); a
            # narrower one would need the previous state in two dtypes at once
            pplan = prev_layout[3]
            if np.dtype(plan.dx).itemsize < np.dtype(pplan.dx).itemsize:
                raise NotImplementedError('r̂ dtype narrowed between snapshots (%s -> %s)'
                                          % (pplan.dx, plan.dx))
            if plan.ids.itemsize < pplan.ids.itemsize:
                raise NotImplementedError('ids dtype narrowed between snapshots (%s -> %s)'
                                          % (pplan.ids, plan.ids))
        n = snap['ids'].numel()
        if snap['coordinates'].numel() != 3 * n or snap['velocities'].numel() != 3 * n:
            raise ValueError('coordinates/velocities must be (N, 3) with N = len(ids)')
        if not compare:
            check_angles_in(angles_in, n)
        lds_e, lds_s = self.table_sizes(plan.dx == F64)
        plan_e = lds_e if entries is None else min(int(entries), lds_e)
        halos, all_items, n_small, scratch, starts, counts, has_prog = self.build_tables(
            snap, centres, bulk_cat, exists, compare, prev_layout, plan_e, lds_s)
        prev_idx = self._prev_idx
        items, glob = all_items[:n_small], all_items[n_small:]
        pr = PreparedStep(plan=plan, n=n, starts=starts, counts=counts, has_prog=has_prog,
                          items=all_items, n_small=n_small, scratch=scratch,
                          compare=bool(compare), n_prev=prev_layout[4] if compare else 0,
                          entries=plan_e)
        pr.halos = _upload(halos.view(np.uint8), dev)
        pr.d_items = _upload(all_items.view(np.uint8), dev)
        if len(glob):
            ch1, ch2, tab, total = plan_global(glob, counts, halos['prev_cnt'], len(items),
                                               compare)
            g = pr.glob
            g['ch1'] = _up(ch1, dev)
            g['ch2'] = _up(ch2, dev) if len(ch2) else None
            g['tab'] = _up(tab, dev)
            g['total'] = total
            pl = None
            if compare and part and self.part_large:
                key4 = self.part_key4 or plan.ids.itemsize == 4
                pl = plan_part(glob, counts, halos['prev_cnt'], self.part_e, self.part_kmax,
                               prev_idx, prev_sets, key4=key4, td_f64=plan.dx == F64)
            if pl is not None:
                pr.part = True
                i32, i64 = torch.int32, torch.int64
                g['prow'] = _up(pl['prow'].reshape(-1), dev)
                g['gpart'] = _up(pl['gpart'].reshape(-1), dev)
                # this step's current bucket set: the next step's previous state
                kt = i32 if key4 else i64
                g['key4'] = key4
                g['pkey_cur'] = torch.empty(pl['n_cur'], dtype=kt, device=dev)
                g['ppos_cur'] = torch.empty(pl['n_cur'], dtype=i32, device=dev)
                g['pmeta_cur'] = torch.empty(pl['n_cur'], dtype=i32, device=dev)
                g['prh_cur'] = torch.empty(3 * pl['n_cur'], dtype=plan.torch_dx, device=dev)
                g['pkey_prev'] = torch.empty(max(pl['n_prev'], 1), dtype=kt, device=dev)
                g['ppos_prev'] = torch.empty(max(pl['n_prev'], 1), dtype=i32, device=dev)
                g['pmeta_prev'] = torch.empty(max(pl['n_prev'], 1), dtype=i32, device=dev)
                g['prh_prev'] = torch.empty(3 * max(pl['n_prev'], 1), dtype=plan.torch_dx,
                                            device=dev)
                g['pcnt'] = torch.empty(pl['n_pcnt'], dtype=i32, device=dev)
                g['rc0'] = pl['rc0']
                g['n_parts'], g['kmax'] = len(pl['plist']), pl['kmax']
                nh = len(halos)
                K = np.zeros(nh, np.int64)
                K[pl['h']] = pl['K']
                base = np.full(nh, -1, np.int64)
                base[pl['h']] = pl['gpart'][:, 0]
                cbase = np.zeros(nh, np.int64)
                cbase[pl['h']] = pl['gpart'][:, 2]
                pr.buckets = BucketSet(key=g['pkey_cur'], pos=g['ppos_cur'], meta=g['pmeta_cur'],
                                       rh=g['prh_cur'], cnt=g['pcnt'], K=K, base=base,
                                       cbase=cbase, cap=self.part_e, td_f64=plan.dx == F64,
                                       key4=key4)
                if prev_sets is not None and pl['inherited'].any():
                    g['inherit'] = prev_sets           # keeps the previous set alive
                    # the scatter reads only the previous chunks of fresh sets
                    gi = np.asarray(ch2[:, 0], dtype=np.int64) - len(items)
                    ch3 = ch2[~pl['inherited'][gi]]
                    g['ch3'] = _up(ch3, dev) \
                        if len(ch3) else None
                    g['n3'] = len(ch3)
            elif compare:
                g['keys'] = torch.empty(2 * total, dtype=torch.int64, device=dev)
            g['n1'], g['n2'] = len(ch1), len(ch2)
        if prev_sets is not None:
            need = np.zeros(len(prev_sets.K), dtype=bool)
            need[prev_idx[prev_idx >= 0]] = True
            if pr.part:
                done = np.zeros_like(need)
                hh = pl['h'][pl['inherited']]
                done[prev_idx[hh]] = True
                need &= ~done
            pr.unbucket_prev = np.flatnonzero(need & (prev_sets.K > 0))
        pr.rhat = torch.empty(n * 3, dtype=plan.torch_dx, device=dev)
        pr.meta = torch.empty(n, dtype=torch.int32, device=dev)
        pr.snap = snap
        pr.bulk_computed = bulk_cat is None and len(halos) > 0
        if pr.bulk_computed:
            pr.halo_list = torch.arange(len(halos), dtype=torch.int32, device=dev)
        if angles_in is not None and not compare:
            pr.angles_in = to_device(np.asarray(angles_in, dtype=np.float16).view(np.int16), dev)
        a = pr.args
        a.ids, a.coords, a.vels, a.n_cur = (snap['ids'].data_ptr(), snap['coordinates'].data_ptr(),
                                            snap['velocities'].data_ptr(), n)
        a.rhat_out, a.meta_out = pr.rhat.data_ptr(), pr.meta.data_ptr()
        a.angles_in = _ptr(pr.angles_in)
        a.halos, a.n_halos = pr.halos.data_ptr(), len(halos)
        a.items, a.n_items = pr.d_items.data_ptr(), len(items)
        a.items_single = items_single(items)
        g = pr.glob
        a.n_global_items = len(glob)
        if len(glob):
            a.n_gchunk1, a.n_gchunk2 = g['n1'], g['n2']
            a.gchunk1, a.gchunk2 = g['ch1'].data_ptr(), _ptr(g['ch2'])
            a.gtab, a.gtab_total = g['tab'].data_ptr(), g['total']
            a.gkeys, a.gvals = _ptr(g.get('keys')), _ptr(g.get('vals'))
            if pr.part:
                a.n_parts, a.part_kmax = g['n_parts'], g['kmax']
                a.part_e, a.part_slots = self.part_e, self.part_slots
                a.prow, a.gpart = g['prow'].data_ptr(), g['gpart'].data_ptr()
                a.pkey_cur, a.ppos_cur = g['pkey_cur'].data_ptr(), g['ppos_cur'].data_ptr()
                a.pmeta_cur, a.prh_cur = g['pmeta_cur'].data_ptr(), g['prh_cur'].data_ptr()
                a.pkey_prev, a.ppos_prev = g['pkey_prev'].data_ptr(), g['ppos_prev'].data_ptr()
                a.pmeta_prev, a.prh_prev = g['pmeta_prev'].data_ptr(), g['prh_prev'].data_ptr()
                inh = g.get('inherit')
                a.ikey, a.ipos = _ptr(inh and inh.key), _ptr(inh and inh.pos)
                a.imeta, a.irh, a.icnt = (_ptr(inh and inh.meta), _ptr(inh and inh.rh),
                                          _ptr(inh and inh.cnt))
                a.pcnt, a.n_pcnt = g['pcnt'].data_ptr(), int(g['pcnt'].numel())
                a.part_key4, a.part_hi = int(g['key4']), 0
                if 'n3' in g:
                    # a non-NULL pointer marks the list as given, even when empty
                    a.gchunk3 = g['ch3'].data_ptr() if g['ch3'] is not None else \
                        g['gpart'].data_ptr()
                    a.n_gchunk3 = g['n3']
        a.H, a.one_plus_z = float(H), float(1 + z)
        a.n_box_dims = len(plan.box)
        for d, L in enumerate(plan.box):
            a.box[d] = L
        a.coord_f64, a.vel_f64 = int(plan.coord == F64), int(plan.vel == F64)
        a.dx_f64, a.vb_f64, a.wrap_f64 = int(plan.dx == F64), int(plan.vb == F64), int(plan.wrap_f64)
        a.id_bytes = plan.ids.itemsize
        a.mode = N.MODE[self.mode]
        a.compare = int(bool(compare))
        a.lds_entries, a.lds_slots = lds_e, lds_s
        return pr

    def launch(self, pr, ws, prev=None, stream=None, step_events=None):
        """Device half of a step: enqueue bulk / step / compact on ``stream``
        (default: torch's current stream).  Never synchronises."""
        lib = self.lib
        st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        a = pr.args
        if pr.bulk_computed:
            m = pr.snap.get('masses') if pr.plan.mass is not None else None
            N.check(lib.oa_bulk_velocity(a.vels, int(pr.plan.vel == F64), _ptr(m),
                                         int(pr.plan.mass == F64), a.halos,
                                         pr.halo_list.data_ptr(), a.n_halos, st),
                    'oa_bulk_velocity')
        res = StepResult(n_slots=int(pr.has_prog.sum()), has_prog=pr.has_prog, halos=pr.halos)
        if pr.compare:
            p = prev if prev is not None else self.prev
            if pr.unbucket_prev is not None and len(pr.unbucket_prev):
                # progenitor blocks this step reads in position order (packed items, the
                # global tables) from the previous step's bucket set
                self.unbucket(p.buckets, pr.unbucket_prev, p.starts, p.rhat, p.meta, st)
            p_ids, p_rhat = p.ids, p.rhat
            if p.plan.dx != pr.plan.dx:                  # float32 -> float64 r̂: exact
                p_rhat = p.rhat.to(pr.plan.torch_dx)
            if p.plan.ids.itemsize != pr.plan.ids.itemsize:
                # 4-byte -> 8-byte IDs (unsigned ones zero-extended)
                p_ids = p.ids.to(torch.int64)
                if p.plan.ids.kind == 'u':
                    p_ids &= 0xFFFFFFFF
            res.extra['prev_widened'] = (p_ids, p_rhat)   # alive until the step is done
            a.ids_prev, a.rhat_prev, a.meta_prev = (p_ids.data_ptr(), p_rhat.data_ptr(),
                                                    p.meta.data_ptr())
            a.n_prev = pr.n_prev
            # packed items only: k_step writes the records, offsets and total itself
            direct = self.direct and pr.n_global == 0 and not a.onthefly
            if not direct:
                ws.reset(res.n_slots)
            ws.gen += 1
            res.ws, res.gen = ws, ws.gen
            a.scratch_ids, a.scratch_ang = ws.scratch_ids.data_ptr(), ws.scratch_ang.data_ptr()
            a.seg_count = ws.seg_count.data_ptr()
            a.halo_count, a.item_count, a.status = (ws.halo_count.data_ptr(),
                                                   ws.item_count.data_ptr(), ws.status.data_ptr())
            a.scratch_pos = _ptr(ws.scratch_pos)
            if pr.part:
                a.scratch_rk = ws.rk()
            a.direct = int(direct)
            if direct:
                a.lookback, a.lb_epoch = ws.lookback_words(len(pr.items))
                a.lb_spin_max = int(self.lb_spin_max)
                a.n_slots = res.n_slots
                a.offsets_out, a.out_ids = ws.offsets.data_ptr(), ws.out_ids.data_ptr()
                a.out_ang, a.out_pos = ws.out_ang.data_ptr(), _ptr(ws.out_pos)
                a.total_out = ws.total.data_ptr()
        if step_events is not None:
            step_events[0].record()
        N.check(lib.oa_step(a, st), 'oa_step')
        if step_events is not None:
            step_events[1].record()
        if not pr.compare:
            return res
        if a.direct:
            res.offsets = ws.offsets[:res.n_slots + 1]
            res.apsis_ids, res.apsis_ang, res.total = ws.out_ids, ws.out_ang, ws.total
            res.apsis_pos = ws.out_pos
            return res
        c = pr.cargs
        c.halos, c.n_halos = a.halos, a.n_halos
        c.items, c.n_items = a.items, a.n_items + a.n_global_items
        c.n_packed = a.n_items
        c.ids_prev, c.id_bytes = a.ids_prev, a.id_bytes
        c.scratch_ids, c.scratch_ang = a.scratch_ids, a.scratch_ang
        c.seg_count = a.seg_count
        c.halo_count, c.item_count, c.n_slots = a.halo_count, a.item_count, res.n_slots
        c.offsets_out, c.out_ids, c.out_ang = (ws.offsets.data_ptr(), ws.out_ids.data_ptr(),
                                               ws.out_ang.data_ptr())
        c.total_out = ws.total.data_ptr()
        c.scratch_pos, c.out_pos = _ptr(ws.scratch_pos), _ptr(ws.out_pos)
        # global items' records: one gather work-group per previous-block chunk
        c.gchunks, c.n_gchunks = (a.gchunk2, a.n_gchunk2) if a.n_global_items else (None, 0)
        # partitioned steps: the join's per-chunk record counters, ranked by scratch_rk
        c.chunk_count = (a.pcnt + 4 * pr.glob['rc0']) if pr.part else None
        c.scratch_rk = a.scratch_rk if pr.part else None
        N.check(lib.oa_compact(c, st), 'oa_compact')
        res.offsets = ws.offsets[:res.n_slots + 1]
        res.apsis_ids, res.apsis_ang, res.total = ws.out_ids, ws.out_ang, ws.total
        res.apsis_pos = ws.out_pos
        return res

    # ------------------------------------------------------------------ host views
    def fetch_async(self, res, ids_dtype):
        """Start the D2H of a compare step's records on the engine's copy stream and
        return a ``PendingFetch`` whose ``wait()`` gives (offsets, ids, angles) as
        ``fetch`` does.  The copies overlap whatever the compute stream runs next (the
        next snapshots' kernels write the other workspaces), so the records' transfer is
        off the per-snapshot critical path.  The workspaces rotate through ``N_WS``, so a
        result's workspace is reused ``N_WS`` steps later, and that launch waits on the
        GPU for this copy (``copy_done``)."""
        self.settle(res)
        res.check_fresh()
        dev = self.device
        if getattr(self, '_copy_stream', None) is None:
            # high priority: a normal-priority stream may share the compute stream's
            # hardware queue (GPU_MAX_HW_QUEUES) and hold the next snapshot's kernels
            # behind this copy (deployment note)
            self._copy_stream = torch.cuda.Stream(device=dev, priority=-1)
        cs = self._copy_stream
        n = res.n_slots + 1
        if res.done is None:                # a result of launch() itself, not of step()
            res.done = torch.cuda.Event()
            res.done.record(torch.cuda.current_stream(dev))
            total = int(res.total.item()) if res.n_slots else 0
        else:
            # the record count came back with the status word (settle waited for it)
            total = int(res.ws.h_total[0]) if res.n_slots else 0
        with torch.cuda.stream(cs):
            cs.wait_event(res.done)
            tev = None
            if self.copy_events is not None:
                tev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                tev[0].record(cs)
            h_off = _pinned(n, torch.int64)
            h_off.copy_(res.offsets[:n], non_blocking=True)
            h_ids = h_ang = None
            if total:
                h_ids = _pinned(total, res.apsis_ids.dtype)
                h_ang = _pinned(total, torch.int16)
                h_ids.copy_(res.apsis_ids[:total], non_blocking=True)
                h_ang.copy_(res.apsis_ang[:total], non_blocking=True)
            if tev is not None:
                tev[1].record(cs)
                self.copy_events.append(tev + (total,))
            done = torch.cuda.Event()
            done.record(cs)
        res.ws.copy_done = done             # the workspace's next launch waits for it
        return PendingFetch(done, h_off, h_ids, h_ang, np.dtype(ids_dtype))

    def fetch(self, res, ids_dtype):
        """Device results -> host arrays in the reference's dtypes.

        The apsis CSR (~10 B per record, ~65 MB per 1e8-particle snapshot) comes back
        through page-locked buffers from torch's caching host allocator: one DMA each
        at the link rate instead of the staged pageable copy (~8 GB/s).  The returned
        arrays own their buffers (a block is reused only once they are gone)."""
        self.settle(res)
        res.check_fresh()
        offsets = res.offsets.cpu().numpy()
        total = int(offsets[-1]) if len(offsets) else 0
        if not total:
            return offsets, np.zeros(0, dtype=ids_dtype), np.zeros(0, dtype=np.float16)
        ids_t = res.apsis_ids[:total]
        h_ids = _pinned(total, ids_t.dtype)
        h_ang = _pinned(total, torch.int16)
        h_ids.copy_(ids_t, non_blocking=True)
        h_ang.copy_(res.apsis_ang[:total], non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return offsets, ids_as(h_ids.numpy(), ids_dtype), h_ang.numpy().view(np.float16)

    def block_bulk(self, snapshot, halo_idx):
        """Bulk velocities (track_orbits.py:269-280) of the listed region blocks of a
        snapshot, computed on the device (oa_bulk_velocity) from those blocks only.
        Returns an (len(halo_idx), 3) array in the reference's result dtype."""
        halo_idx = np.asarray(halo_idx, dtype=np.int64)
        vel = snapshot['velocities']
        ids = snapshot['ids']
        n = int(ids.numel()) if isinstance(ids, torch.Tensor) else len(ids)
        starts = np.asarray(snapshot['region_offsets'], dtype=np.int64).reshape(-1)
        counts = np.append(starts[1:], n) - starts
        plan = plan_dtypes(snapshot, np.zeros(3), None, 0.0, 0.0)
        dev = self.device
        # the kernel reads each listed block in place (no row gather): the arrays move
        # to the device whole (a sharded run passes its stripe only)
        v = vel.reshape(-1, 3).to(dev).contiguous() if isinstance(vel, torch.Tensor) \
            else to_device(np.asarray(vel).reshape(-1, 3), dev)
        m = None
        if plan.mass is not None:
            ms = snapshot['masses']
            m = ms.to(dev).contiguous() if isinstance(ms, torch.Tensor) else to_device(ms, dev)
        # no rows at all: the kernel still needs real (unread) arrays
        if v.numel() == 0:
            v = torch.zeros((1, 3), dtype=v.dtype, device=dev)
        if m is not None and m.numel() == 0:
            m = torch.zeros(1, dtype=m.dtype, device=dev)
        halos = np.zeros(len(halo_idx), dtype=N.HALO_DTYPE)
        halos['cur_off'] = starts[halo_idx]
        halos['cur_cnt'] = counts[halo_idx]
        # pinned staging both ways: a pageable copy is synchronous and waits behind any
        # DMA in flight (a double-buffered snapshot H2D held the sharded on-the-fly
        # step's stripe bulk ~70 ms)
        d_h = _up(halos.view(np.uint8), dev)
        lst = torch.arange(len(halo_idx), dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        if len(halo_idx):
            N.check(self.lib.oa_bulk_velocity(v.data_ptr(), int(plan.vel == F64), _ptr(m),
                                              int(plan.mass == F64), d_h.data_ptr(),
                                              lst.data_ptr(), len(halo_idx), st),
                    'oa_bulk_velocity')
        h = _pinned(d_h.numel(), torch.uint8)
        h.copy_(d_h, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        out = h.numpy().view(N.HALO_DTYPE)['bulk']
        return out.astype(plan.bulk)

    def bulk_velocities(self, res, plan):
        self.settle(res)
        h = res.halos.cpu().numpy().view(N.HALO_DTYPE)
        return h['bulk'].astype(plan.bulk)

    def unbucket(self, bs, halos, starts, rhat, meta, stream=None):
        """Restore the position-order state (r̂, state word) of the listed halos of a
        step from its bucket set ``bs`` into that step's ``rhat`` / ``meta`` arrays (block
        starts ``starts``).  Idempotent; a halo is restored once."""
        halos = np.asarray(halos, dtype=np.int64)
        if bs.restored is None:
            bs.restored = np.zeros(len(bs.K), dtype=bool)
        halos = halos[(bs.K[halos] > 0) & ~bs.restored[halos]]
        if not len(halos):
            return
        dev = self.device
        st = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        rows = np.stack([bs.base[halos], bs.K[halos], bs.cbase[halos],
                         np.asarray(starts, np.int64)[halos]], axis=1).astype(np.int64)
        K = bs.K[halos]
        plist = np.stack([np.repeat(np.arange(len(halos)), K),
                          np.arange(int(K.sum())) - np.repeat(np.cumsum(K) - K, K)],
                         axis=1).astype(np.int32)
        d_rows = _upload(rows.view(np.uint8), dev)
        d_plist = _upload(plist.view(np.uint8), dev)
        u = N.UnbucketArgs()
        u.bpos, u.bmeta, u.brh, u.bcnt = (bs.pos.data_ptr(), bs.meta.data_ptr(),
                                          bs.rh.data_ptr(), bs.cnt.data_ptr())
        u.rows, u.plist, u.n_parts, u.cap = (d_rows.data_ptr(), d_plist.data_ptr(), len(plist),
                                             int(bs.cap))
        u.rhat_out, u.meta_out, u.td_f64 = rhat.data_ptr(), meta.data_ptr(), int(bs.td_f64)
        N.check(self.lib.oa_part_unbucket(u, st), 'oa_part_unbucket')
        bs.restored[halos] = True
        self._keep = (d_rows, d_plist)      # until the next call (stream-ordered use)

    def state_meta(self):
        """The current state words in position order (bucketed large halos restored)."""
        self.settle()
        p = self.prev
        if p.buckets is not None:
            self.unbucket(p.buckets, np.arange(len(p.buckets.K)), p.starts, p.rhat, p.meta)
        return p.meta

    def angles(self):
        """Current per-particle float16 angles (checkpoint payload, track_orbits.py:390-394)."""
        return meta_angles(self.state_meta())

    def checkpoint_layout(self):
        """Row layout of ``angles()``: None, the snapshot's own row order."""
        return None
