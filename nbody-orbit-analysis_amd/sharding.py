"""Multi-GPU orbit tagging: particles sharded by ID range across ranks.

One process per GPU, ``torch.distributed`` (RCCL on MI355X, gloo on CPU).  Every
rank runs the same ``track_orbits`` driver.  The reference's only parallel axis is
the halo pool of track_orbits.py:189-194; here the axis is the particle ID instead:
rank r owns the IDs of one contiguous range (``IdRangeOwner``, the default), so a
particle's current and previous rows -- including its copies in overlapping regions
-- sit on the same rank, and the join needs no exchange.

* **shard** (the reference's loader contract: every rank is handed the whole
  snapshot, track_orbits.py:118-122): the snapshot is cut into W block-aligned
  *stripes* of about N/W rows (``stripe_halos``).  Rank r moves only stripe r to its
  GPU -- 1/W of the snapshot over its own PCIe link -- computes the bulk velocities of
  the stripe's blocks there (whole blocks: the reference's sequential sums, bit for
  bit), sorts the stripe's rows by owner rank and routes them with one all-to-all
  over xGMI (``RowExchange``).  Received rows arrive in source-rank order, i.e. in
  global row order, so block order is preserved, and every row carries its global
  row (``sel``).  A *presharded* loader (``presharded=True``, e.g. a distributed
  reader) hands each rank its own rows directly; the global block is then the
  rank-ordered concatenation of the ranks' blocks.
* **step**: the rank's ``OrbitEngine`` on its shard; the kernel also emits each apsis
  record's previous-state row, which maps to its global previous-block position
  through the previous snapshot's gpos (a device gather).
* **records** stay on the device until the savefile needs them: ``fetch_async``
  has every rank store its own records at their final positions in one page-locked
  host buffer that all ranks map (``host_share.SharedRecordStage``), which is exactly
  the reference's order (previous-block order within each halo, halos in
  ``halo_exists`` order, track_orbits.py:199-227, 315-316); rank 0, the only writer,
  hands that buffer to the savefile.

Collectives per snapshot: the shard's all-to-all (not with presharded loaders), one
all-gather of the halo catalogue rows (centre, bulk velocity), an all-gather of the
computed bulk velocities when the catalogue gives none, and the output stage's count
all-gather and slot broadcast (with stripes, one all-reduce of a previous-row bitmap).
None of them exchanges per-particle data with every rank.

``ShardedEngine`` exposes the ``OrbitEngine`` interface the driver uses, so
``track_orbits(..., engine=ShardedEngine(EngineLocal(OrbitEngine())))`` is the
multi-GPU drop-in.
"""
import hashlib
import os
from dataclasses import dataclass
from typing import Optional

from contextlib import nullcontext as _nullcontext

import numpy as np
import torch

U64 = np.uint64
_HASH_C = np.int64(-7046029254386353131)        # 0x9E3779B97F4A7C15 as int64
_I64_MAX, _I64_MIN = np.iinfo(np.int64).max, np.iinfo(np.int64).min


# ------------------------------------------------------------------ ownership
class HashOwner:
    """rank = hash(ID) mod world (balanced for any ID distribution)."""

    def __call__(self, ids, world):
        h = np.asarray(ids).astype(np.int64, copy=False) * _HASH_C     # wrapping int64
        return ((h >> 33) & 0x7FFFFFFF) % world

    def fit(self, ids):
        pass

    def fit_group(self, ids_t, group):
        pass

    def reset(self):
        pass

    def ranks(self, ids_t, world):
        h = ids_t.to(torch.int64) * int(_HASH_C)
        return ((h >> 33) & 0x7FFFFFFF) % world

    def mask(self, ids_t, world, rank):
        return self.ranks(ids_t, world) == rank


class IdRangeOwner:
    """rank = floor((ID - lo) * world / (hi - lo)), clipped: contiguous ID ranges.
    Without bounds, [lo, hi) is fitted on the first snapshot the engine sees (the
    min / max over all ranks' rows); later IDs outside it go to the first / last rank.
    A fitted range is dropped by ``reset`` (a new run); given bounds are kept.
    IDs are taken as their int64 bit patterns (uint64 IDs >= 2^63 sort below the
    others, as device tensors hold them), and the ratio is evaluated in float64 (the
    same operations on the host and the device)."""

    def __init__(self, lo=None, hi=None):
        self.lo = None if lo is None else int(lo)
        self.hi = None if hi is None else int(hi)
        self.fixed = lo is not None

    def reset(self):
        if not self.fixed:
            self.lo = self.hi = None

    @staticmethod
    def _i64(ids):
        ids = np.asarray(ids)
        return ids.view(np.int64) if ids.dtype.itemsize == 8 else ids.astype(np.int64)

    def fit(self, ids):
        if self.lo is not None:
            return
        if isinstance(ids, torch.Tensor):
            t = ids.to(torch.int64)
            lo, hi = (int(t.min()), int(t.max()) + 1) if t.numel() else (0, 1)
        else:
            v = self._i64(ids)
            lo, hi = (int(v.min()), int(v.max()) + 1) if v.size else (0, 1)
        self.lo, self.hi = lo, hi

    def fit_group(self, ids_t, group):
        """Fit on the union of the ranks' rows (one 2-element all-reduce)."""
        import torch.distributed as dist
        if self.lo is not None:
            return
        if dist.get_world_size(group) == 1:
            return                              # one rank owns every ID: nothing to fit
        t = ids_t.to(torch.int64)
        if t.numel():
            mn, mx = (int(x) for x in torch.stack([t.min(), t.max()]).cpu())   # one D2H
        else:
            mn, mx = _I64_MAX, _I64_MIN + 1
        if dist.get_world_size(group) > 1:
            r = _h2d(np.asarray([mn, -mx], dtype=np.int64), _comm_device())
            dist.all_reduce(r, op=dist.ReduceOp.MIN, group=group)
            mn, mx = int(r[0]), -int(r[1])
        self.lo, self.hi = (mn, mx + 1) if mn <= mx else (0, 1)

    def __call__(self, ids, world):
        span = float(max(self.hi - self.lo, 1))
        v = self._i64(ids).astype(np.float64)
        r = np.floor((v - float(self.lo)) * world / span)
        return np.clip(r, 0, world - 1).astype(np.int64)

    def ranks(self, ids_t, world):
        span = float(max(self.hi - self.lo, 1))
        r = torch.floor((ids_t.to(torch.int64).to(torch.float64) - float(self.lo)) * world / span)
        return r.clamp_(0, world - 1).to(torch.int64)

    def mask(self, ids_t, world, rank):
        return self.ranks(ids_t, world) == rank


def block_layout(region_offsets, n):
    starts = np.asarray(region_offsets, dtype=np.int64).reshape(-1)
    counts = np.append(starts[1:], n) - starts
    return starts, counts


def shard_snapshot(snapshot, keep):
    """Host reference of the device shard (tests): rows of ``snapshot`` selected by
    boolean ``keep`` (block order preserved).  Returns (shard dict, global row index of
    every kept row, shard block starts, shard block counts)."""
    ids = np.asarray(snapshot['ids'])
    n = len(ids)
    starts, counts = block_layout(snapshot['region_offsets'], n)
    sel = np.flatnonzero(keep)
    block = np.repeat(np.arange(len(starts)), counts)
    cnt = np.bincount(block[sel], minlength=len(starts)).astype(np.int64)
    st = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.int64) if len(cnt) else cnt
    shard = dict(snapshot)
    shard['ids'] = ids[sel]
    shard['coordinates'] = np.asarray(snapshot['coordinates'])[sel]
    shard['velocities'] = np.asarray(snapshot['velocities'])[sel]
    if isinstance(snapshot['masses'], np.ndarray):
        shard['masses'] = snapshot['masses'][sel]
    shard['region_offsets'] = st
    return shard, sel, st, cnt


def stripe_halos(starts, n, world):
    """Block-aligned stripes of a snapshot: halo boundaries hb[0..world] such that rank
    r's stripe is the blocks [hb[r], hb[r+1]), i.e. rows [row(hb[r]), row(hb[r+1]))
    with row(j) = starts[j] (n past the last block), each about (n - starts[0]) / world
    rows.  Rows before the first block belong to no halo and to no stripe."""
    starts = np.asarray(starts, dtype=np.int64)
    nh = len(starts)
    hb = np.zeros(world + 1, dtype=np.int64)
    hb[world] = nh
    if nh and world > 1:
        lo = int(starts[0])
        targets = lo + (n - lo) * np.arange(1, world, dtype=np.float64) / world
        hb[1:world] = np.searchsorted(starts, targets, side='left')
    return hb


def stripe_rows(starts, n, hb, r):
    """Row range [lo, hi) of stripe r (``stripe_halos``)."""
    nh = len(starts)

    def row(j):
        return int(starts[j]) if j < nh else int(n)
    return row(int(hb[r])), row(int(hb[r + 1]))


def _h2d(a, device):
    """A small host array -> tensor on ``device`` through a page-locked staging block
    (``engine._up``: asynchronous on the current stream).  A pageable ``.to(device)`` is
    a synchronous copy that waits behind whatever DMA is in flight -- a double-buffered
    snapshot H2D on a copy stream held each sharded on-the-fly step's host ~70 ms
    (bench_onthefly --sharded, r04q)."""
    a = np.ascontiguousarray(a)
    if torch.device(device).type != 'cuda':
        return torch.from_numpy(a)
    from .engine import _up
    return _up(a, device)


# ------------------------------------------------------------------ collectives
def _comm_device():
    import torch.distributed as dist
    return torch.device('cuda', torch.cuda.current_device()) \
        if dist.get_backend() == 'nccl' else torch.device('cpu')


# gloo moves neither 16-bit integers nor bool: they travel widened
_WIDEN = {torch.int16: torch.int32, torch.bool: torch.uint8, torch.float16: torch.float32}
# the dtypes torch's NCCL backend maps to an RCCL type (ProcessGroupNCCL's ncclDataType
# table: no int16 / uint16 / uint32 / uint64); any other dtype travels as its bytes
NCCL_WIRE = frozenset({torch.uint8, torch.int8, torch.int32, torch.int64, torch.float16,
                       torch.bfloat16, torch.float32, torch.float64, torch.bool})


def to_wire(x, cpu_comm):
    """``x`` (rows along dim 0) in a dtype the backend moves: widened for gloo
    (``cpu_comm``), bit-viewed as (rows, bytes) uint8 for RCCL when torch's NCCL table
    has no type for it.  Returns (wire tensor, bit-viewed); ``from_wire`` undoes it."""
    dt = x.dtype
    if cpu_comm:
        return x.to(_WIDEN.get(dt, dt)), False
    if dt in NCCL_WIRE:
        return x, False
    return x.contiguous().reshape(x.shape[0], -1).view(torch.uint8), True


def from_wire(y, dt, tail, bitview):
    """The rows ``to_wire`` sent, from the received wire rows ``y`` (row shape ``tail``)."""
    if bitview:
        return y.view(dt).reshape((y.shape[0],) + tuple(tail))
    return y.to(dt)


class RowExchange:
    """Point-to-point row routing with known per-destination counts: one
    ``all_to_all_single`` per tensor, uneven splits, rows already sorted by destination
    rank.  The received rows are the senders' rows in rank order.  The counts are
    exchanged once (a W-element all-to-all), so several tensors with the same rows
    cost one small exchange plus one collective each.  World 1 moves nothing."""

    def __init__(self, send_counts, group=None):
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.send = [int(c) for c in send_counts]
        if self.world == 1:
            self.recv = list(self.send)
            return
        self.dev = _comm_device()
        s = _h2d(np.asarray(self.send, dtype=np.int64), self.dev)
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=group)
        self.recv = [int(x) for x in r.cpu()]

    @property
    def n_recv(self):
        return sum(self.recv)

    def move(self, t):
        import torch.distributed as dist
        if self.world == 1:
            return t
        home = t.device
        x = t.contiguous()
        dt, tail = x.dtype, tuple(x.shape[1:])
        x, bv = to_wire(x.to(self.dev), self.dev.type == 'cpu')
        out = torch.empty((self.n_recv,) + tuple(x.shape[1:]), dtype=x.dtype, device=self.dev)
        dist.all_to_all_single(out, x, self.recv, self.send, group=self.group)
        return from_wire(out, dt, tail, bv).to(home)


def _exchange_rows(t, group=None):
    """Equal-split all-to-all of a (world, ...) tensor: rank d receives row d of every
    rank, in rank order (on t's device)."""
    import torch.distributed as dist
    home = t.device
    dev = _comm_device()
    x = t.contiguous().to(dev)
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x, group=group)
    return out.to(home)


def gather_rows(group, root, *tensors):
    """Gather the rows of each tensor (same row count) to ``root``, rank-ordered; the
    other ranks get empty tensors.  One count exchange + one collective per tensor."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    n = int(tensors[0].shape[0])
    rx = RowExchange([n if q == root else 0 for q in range(world)], group)
    return [rx.move(t) for t in tensors]


def allgather_rows(a, group=None):
    """Variable-length all-gather of a 2-D int64 array (host); rank-ordered concatenation."""
    t = allgather_v(torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)), group)
    return t.cpu().numpy()


def allgather_v(t, group=None):
    """Variable-length all-gather of a tensor along dim 0 (device tensors over RCCL
    with the nccl backend, host tensors with gloo); rank-ordered concatenation, on
    the communication device."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = _comm_device()
    t = t.to(dev)
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    m = max(max(ns), 1)
    buf = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
    buf[:t.shape[0]] = t
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return torch.cat([o[:k] for o, k in zip(outs, ns)], dim=0)


def all_true(flag, group=None):
    """True on every rank iff ``flag`` is true on every rank (one 1-element all-reduce)."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return bool(flag)
    t = _h2d(np.asarray([1 if flag else 0], dtype=np.int32), _comm_device())
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def _f64_bits(x):
    return np.ascontiguousarray(x, dtype=np.float64).view(np.int64)


def _to_tensor(x, device):
    """A row range of a loader array -> tensor on ``device`` (uint dtypes bit-cast)."""
    if isinstance(x, torch.Tensor):
        return x.to(device)
    a = np.ascontiguousarray(x)
    if a.dtype.kind == 'u':
        a = a.view(a.dtype.str.replace('u', 'i'))
    return torch.from_numpy(a).to(device)


def gather_bulk(rows_local, h0, nh, group=None):
    """All-gather the bulk-velocity rows each rank computed for its halos [h0, h0+k):
    returns the (nh, 3) array in the computed dtype (float64 bits on the wire)."""
    b = np.asarray(rows_local).reshape(-1, 3) if rows_local is not None else np.zeros((0, 3))
    dt = b.dtype if len(b) else None
    rows = np.concatenate([(h0 + np.arange(len(b)))[:, None].astype(np.int64),
                           _f64_bits(b).reshape(-1, 3)], axis=1)
    allr = allgather_rows(rows, group)
    dts = allgather_rows(np.array([[0 if dt is None else np.dtype(dt).itemsize]]), group)[:, 0]
    size = int(dts.max()) if len(dts) else 8
    out = np.full((nh, 3), np.nan, dtype=np.float64)
    out[allr[:, 0]] = allr[:, 1:].copy().view(np.float64)
    return out.astype(np.float32 if size == 4 else np.float64)


# ------------------------------------------------------------------ stripes -> shards
@dataclass
class Shard:
    """This rank's rows of one snapshot (device tensors in block order)."""
    snap: dict                         # ids / coordinates / velocities (/ masses) + region_offsets
    sel: torch.Tensor                  # global snapshot row of every shard row (int64)
    gpos: Optional[torch.Tensor]       # position in its global block (presharded only)
    counts: np.ndarray                 # shard rows per halo
    bulk: Optional[np.ndarray] = None  # (nh, 3) bulk velocities of the whole blocks
    h2d_bytes: int = 0                 # loader bytes this rank moved to its device


def my_stripe(starts, n, group=None):
    """(lo, hi) rows of this rank's stripe of a snapshot of n rows with these block
    starts: what a reader that hands each rank its stripe (``STRIPE`` key) must load."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    return stripe_rows(np.asarray(starts, np.int64), n, stripe_halos(starts, n, world), rank)


STRIPE = 'stripe_rows'     # snapshot key: the arrays hold only rows [lo, hi) (my_stripe)


def stripe_shard(snapshot, starts, owner, group, device, bulk_fn=None, n=None):
    """The whole-snapshot loader contract on one rank (module docstring): upload stripe
    r only, compute its blocks' bulk velocities (``bulk_fn(stripe_snapshot, halos)``,
    when given), route its rows to their owners with one all-to-all per array, and lay
    the received rows out in block order.  A snapshot carrying ``STRIPE`` = (lo, hi)
    holds this rank's stripe only (a striped reader, e.g. one that double-buffers its
    stripe on a copy stream); ``n`` is then the global row count.  Returns a ``Shard``."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    ids = snapshot['ids']
    striped = snapshot.get(STRIPE)
    if n is None:
        if striped is not None:
            raise ValueError('a striped snapshot needs the global row count n')
        n = int(ids.numel()) if isinstance(ids, torch.Tensor) else len(ids)
    starts = np.asarray(starts, dtype=np.int64)
    nh = len(starts)
    hb = stripe_halos(starts, n, world)
    lo, hi = stripe_rows(starts, n, hb, rank)
    h0, h1 = int(hb[rank]), int(hb[rank + 1])
    masses = snapshot['masses']
    has_m = isinstance(masses, (np.ndarray, torch.Tensor))
    keys = ('ids', 'coordinates', 'velocities') + (('masses',) if has_m else ())
    if striped is not None:
        if tuple(int(x) for x in striped) != (lo, hi):
            raise ValueError('striped snapshot holds rows %s, this rank\'s stripe is %s'
                             % (tuple(striped), (lo, hi)))
        st = {k: _to_tensor(snapshot[k], device) for k in keys}
    else:
        st = {k: _to_tensor(snapshot[k][lo:hi], device) for k in keys}
    h2d = sum(int(v.numel()) * v.element_size() for k, v in st.items()
              if not (isinstance(snapshot[k], torch.Tensor) and snapshot[k].device.type ==
                      torch.device(device).type))
    for k in ('coordinates', 'velocities'):
        st[k] = st[k].reshape(-1, 3)
    bulk = None
    if bulk_fn is not None:
        stripe = dict(snapshot)
        stripe.update(st)
        stripe['region_offsets'] = starts[h0:h1] - lo
        rows = bulk_fn(stripe, np.arange(h1 - h0)) if h1 > h0 else None
        bulk = gather_bulk(rows, h0, nh, group) if world > 1 else \
            (np.asarray(rows) if rows is not None else np.zeros((0, 3)))
    owner.fit_group(st['ids'], group)
    nst = int(st['ids'].shape[0])
    sc = (np.append(starts[h0 + 1:h1], hi) - starts[h0:h1]) if h1 > h0 else np.zeros(0, np.int64)
    if world > 1:
        # every stripe row's block: the stripe holds blocks [h0, h1) (host layout)
        sblock = torch.repeat_interleave(torch.arange(h0, h1, device=device),
                                         _h2d(sc.astype(np.int64), device),
                                         output_size=nst) if nst else \
            torch.zeros(0, dtype=torch.int64, device=device)
        dest = owner.ranks(st['ids'], world)
        dest, perm = torch.sort(dest, stable=True)
        # rows per (destination, block): one D2H; the row counts of the exchange and,
        # after it, the shard's per-block counts follow from it and its exchange
        hist = torch.bincount(dest * max(nh, 1) + sblock[perm], minlength=world * max(nh, 1))
        hist = hist.view(world, max(nh, 1))
        rx = RowExchange(hist.sum(1).cpu().tolist(), group)
        sel = rx.move(perm + lo)
        sh = {k: rx.move(v[perm]) for k, v in st.items()}
        got = _exchange_rows(hist, group)       # row d of every sender: (world, nh)
        counts = got.sum(0).cpu().numpy().astype(np.int64)[:nh] if nh else np.zeros(0, np.int64)
    else:
        # one rank: the stripe is the snapshot, in its own row order
        sel = torch.arange(lo, hi, dtype=torch.int64, device=device)
        sh = st
        counts = np.zeros(nh, np.int64)
        counts[h0:h1] = sc
    shard = dict(snapshot)
    shard.update(sh)
    shard['region_offsets'] = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64) \
        if nh else counts
    # (a row's block position is its global row minus its block's start: the record
    # merges key on the global row itself, so it is not materialised)
    return Shard(snap=shard, sel=sel, gpos=None, counts=counts, bulk=bulk, h2d_bytes=h2d)


# ------------------------------------------------------------------ engine facade
@dataclass
class ShardedResult:
    n_slots: int
    has_prog: np.ndarray
    records: Optional[tuple] = None          # device (offsets, ids, f16 bits, prev-state row)
    prev_prep: object = None                 # the previous snapshot's ShardedPrep (its
                                             # shard rows' global block positions: gpos)
    bulk: Optional[np.ndarray] = None
    lp: object = None                        # the local step (deferred: settled later)


class ShardedFetch:
    """A sharded step's records on their way to rank 0 and its host (fetch_async)."""

    def __init__(self, done, n_slots, h_off, h_ids, h_ang, ids_dtype, root):
        self.done, self.n_slots, self.root = done, n_slots, root
        self.h_off, self.h_ids, self.h_ang, self.ids_dtype = h_off, h_ids, h_ang, ids_dtype

    def wait(self):
        from .engine import ids_as
        dt = np.dtype(self.ids_dtype)
        if not self.root:
            return np.zeros(self.n_slots + 1, np.int64), np.zeros(0, dt), np.zeros(0, np.float16)
        if self.done is not None:
            self.done.synchronize()
        return (self.h_off.numpy().astype(np.int64), ids_as(self.h_ids.numpy(), dt),
                self.h_ang.numpy().view(np.float16))


@dataclass
class ShardedPrep:
    """One snapshot's host half (ShardedEngine.prepare): the shard, its rows' global
    block positions and the local engine's prepared step.  With a presharded loader the
    global positions come from an all-gather of the ranks' block counts that runs when
    they are first needed (the records' gather, a checkpoint, a resume), not while the
    snapshot is planned: every rank reaches those points in the same order."""
    n: int
    exists: np.ndarray
    compare: bool
    gpos_: Optional[torch.Tensor]
    sel_: Optional[torch.Tensor]            # this rank's rows in the global snapshot
    n_global_: Optional[int]
    rows: Optional[np.ndarray]              # catalogue rows (centre, bulk) to exchange
    bulk_out: Optional[np.ndarray]
    plan: object
    lp: object = None
    layout_: Optional[str] = None           # checkpoint row layout (presharded runs)
    h2d_bytes: int = 0
    local_args: tuple = ()                  # the local engine's prepare arguments
    lazy: object = None                     # () -> (gpos, sel, n_global, layout)

    def _resolve(self):
        if self.lazy is not None:
            self.gpos_, self.sel_, self.n_global_, self.layout_ = self.lazy()
            self.lazy = None

    @property
    def gpos(self):
        self._resolve()
        return self.gpos_

    @property
    def sel(self):
        self._resolve()
        return self.sel_

    @property
    def n_global(self):
        self._resolve()
        return self.n_global_

    @property
    def layout(self):
        self._resolve()
        return self.layout_


class _Plan:
    def __init__(self, ids_dtype, bulk_dtype=None):
        self.ids = np.dtype(ids_dtype)
        self.bulk = bulk_dtype


def check_layout(want, have):
    """A checkpoint written in one row layout resumes only in the same one (ADVICE r02:
    a presharded checkpoint's rows depend on the world size and the reader's split)."""
    if (want or None) != (have or None):
        raise ValueError('checkpoint angles were written in row layout %r, this run reads '
                         'the snapshot in layout %r: resume with the same sharding'
                         % (want or 'global', have or 'global'))


class ShardedEngine:
    """``OrbitEngine`` interface over ID-sharded ranks (see module docstring).

    ``step`` = ``prepare`` (host: shard, plan, uploads) + ``launch`` (the catalogue
    all-gather and the device step).  The two halves are public so a benchmark can
    prepare a chain of snapshots and time ``launch`` alone, as bench.py does."""

    ROOT = 0                              # the rank that writes the savefile

    def __init__(self, local, group=None, owner=None, mode=None, presharded=False,
                 share_catalogue=True):
        import torch.distributed as dist
        self.local = local
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.owner = owner or IdRangeOwner()
        self.mode = mode or local.mode
        self.presharded = bool(presharded)
        self.share_catalogue = bool(share_catalogue)
        self.device = getattr(local, 'device', torch.device('cpu'))
        self.prev: Optional[ShardedPrep] = None
        self._pending: Optional[ShardedResult] = None   # a deferred step not yet settled
        self._side = None                               # stream of the records' gathers
        self._stage = None                              # shared host output (world > 1)
        self._xstream = None                            # catalogue all-gather (RCCL)
        # rank 0's record placement timed (synchronised) into fetch_stats (rehearsals)
        self.profile_fetch = False
        self.fetch_stats = None

    def reset(self):
        self.settle()
        self.prev = None
        self.owner.reset()
        self.local.reset()

    # ---------------------------------------------------------------- collectives
    def _exchange(self, rows, nh):
        """The one per-snapshot all-gather of catalogue rows: rank r contributes halos
        [r * nl, (r + 1) * nl) of its (nh, 6) float64 rows; every rank gets all nh.

        On the device (RCCL) the all-gather is issued from a side stream: it depends on
        nothing the previous step computes, so it runs while that step's kernels do,
        and only the next launch waits for it (the current stream waits on the side
        stream; the result is recorded as used there)."""
        import torch.distributed as dist
        nl = -(-nh // self.world)
        mine = np.zeros((nl, 6), dtype=np.float64)
        lo, hi = self.rank * nl, min((self.rank + 1) * nl, nh)
        if hi > lo:
            mine[:hi - lo] = rows[lo:hi]
        dev = _comm_device()
        if dev.type != 'cuda' or os.environ.get('ORBIT_XSTREAM', '1') == '0':
            out = torch.empty((nl * self.world, 6), dtype=torch.float64, device=dev)
            dist.all_gather_into_tensor(out, _h2d(mine, dev), group=self.group)
            return out[:nh]
        if self._xstream is None:
            self._xstream = torch.cuda.Stream(device=dev)
        cur = torch.cuda.current_stream(dev)
        with torch.cuda.stream(self._xstream):
            out = torch.empty((nl * self.world, 6), dtype=torch.float64, device=dev)
            dist.all_gather_into_tensor(out, _h2d(mine, dev), group=self.group)
        cur.wait_stream(self._xstream)
        out.record_stream(cur)
        return out[:nh]

    # ---------------------------------------------------------------- shard
    def _presharded_gpos(self, starts, counts):
        """Global block = the ranks' blocks concatenated in rank order: a shard row's
        position is the rows of lower ranks in its block + its own index.  Returns the
        block positions, the global snapshot rows, the global row count and the row
        layout tag of a checkpoint written in this layout.  One all-gather of the ranks'
        per-block counts (host arithmetic on them), then two device expansions with a
        known output size: no other host round trip."""
        import torch.distributed as dist
        nh = len(counts)
        dev = _comm_device()
        mine = _h2d(np.ascontiguousarray(counts, dtype=np.int64), dev)
        allc = torch.empty(self.world * nh, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(allc, mine, group=self.group)
        cnt_all = allc.cpu().numpy().reshape(self.world, nh)
        before = cnt_all[:self.rank].sum(0)
        tot = cnt_all.sum(0)
        gstart = np.cumsum(tot) - tot
        n = int(np.sum(counts))
        c = _h2d(np.ascontiguousarray(counts, dtype=np.int64), self.device)
        row = torch.arange(n, dtype=torch.int64, device=self.device)
        # gpos = before[block] + (row - starts[block]); sel = gstart[block] + gpos
        b0 = _h2d(before - starts, self.device)
        gpos = torch.repeat_interleave(b0, c, output_size=n) + row
        sel = torch.repeat_interleave(_h2d(gstart, self.device), c,
                                      output_size=n) + gpos
        digest = hashlib.sha256(np.ascontiguousarray(cnt_all, dtype='<i8').tobytes()).hexdigest()[:16]
        layout = 'rank-major/world=%d/blocks=%s' % (self.world, digest)
        return gpos, sel, int(tot.sum()), layout

    # ---------------------------------------------------------------- step
    def prepare(self, snapshot, centres, bulk_cat, H, z, exists, compare, angles_in=None,
                prev=None, angles_layout=None):
        """Host half of a step; ``prev`` (a ShardedPrep) defaults to the last step.
        ``angles_layout``: the row layout the resumed checkpoint was written in."""
        from .engine import check_angles_in
        exists = np.asarray(exists)
        ids = snapshot['ids']
        n = int(ids.numel()) if isinstance(ids, torch.Tensor) else len(ids)
        starts, counts = block_layout(snapshot['region_offsets'], n)
        nh = len(starts)
        bulk = bulk_cat
        layout, h2d = None, 0
        if self.presharded:
            if bulk_cat is None and nh:
                raise NotImplementedError('computed bulk velocities need whole blocks: give '
                                          'catalogue bulk velocities with presharded snapshots')
            # this rank's rows as they are; host arrays (a distributed reader) move to
            # the rank's device once
            shard = dict(snapshot)
            for k in ('ids', 'coordinates', 'velocities'):
                shard[k] = _to_tensor(snapshot[k], self.device)
            if isinstance(snapshot['masses'], (np.ndarray, torch.Tensor)):
                shard['masses'] = _to_tensor(snapshot['masses'], self.device)
            h2d = sum(int(np.asarray(snapshot[k]).nbytes) for k in ('ids', 'coordinates',
                                                                    'velocities')
                      if not isinstance(snapshot[k], torch.Tensor))
            lazy = (lambda st=starts, ct=counts: self._presharded_gpos(st, ct))
            gpos = sel = n_global = layout = None
            if angles_in is not None and not compare:      # a resume needs them now
                gpos, sel, n_global, layout = lazy()
                lazy = None
        else:
            sh = stripe_shard(snapshot, starts, self.owner, self.group, self.device,
                              bulk_fn=self.local.bulk if (bulk_cat is None and nh) else None)
            shard, sel, gpos, n_global, h2d = sh.snap, sh.sel, sh.gpos, n, sh.h2d_bytes
            if bulk_cat is None and nh:
                bulk = sh.bulk
        a_in = None
        if angles_in is not None and not compare:
            # a checkpoint holds the global snapshot's angles in this run's row layout
            check_layout(angles_layout, layout)
            check_angles_in(angles_in, n_global)
            a_in = np.asarray(angles_in)[sel.cpu().numpy()]
        rows = None
        if self.share_catalogue and nh:
            rows = np.zeros((nh, 6), dtype=np.float64)
            rows[:, :3] = np.asarray(centres, dtype=np.float64).reshape(nh, 3)
            if bulk_cat is not None:
                rows[:, 3:] = np.asarray(bulk_cat, dtype=np.float64).reshape(nh, 3)
        p = prev if prev is not None else self.prev
        ids_dt = np.asarray(ids[:0].cpu() if isinstance(ids, torch.Tensor) else ids[:0]).dtype
        sp = ShardedPrep(n=n, exists=exists, compare=bool(compare), gpos_=gpos, sel_=sel,
                         n_global_=n_global, lazy=lazy if self.presharded else None,
                         rows=rows, bulk_out=None if bulk_cat is not None else bulk,
                         plan=_Plan(ids_dt, None if bulk is None else np.asarray(bulk).dtype),
                         layout_=layout, h2d_bytes=h2d)
        sp.local_args = (shard, centres, bulk, H, z, exists, compare, a_in, bulk_cat is not None)
        sp.lp = self._local_prepare(sp, None if (prev is None or p is None) else p.lp)
        # the halos with a progenitor block, planned here (host work off the launch)
        sp.has_prog_for = (p, np.isin(exists, p.exists)) if compare and p is not None else None
        return sp

    def _local_prepare(self, sp, prev_lp):
        """The local engine's host half of a prepared step (no collective: a rank that
        re-ran its previous step plans again on its own)."""
        a = sp.local_args
        return self.local.prepare(*a[:8], prev_lp, share=a[8])

    def launch(self, sp, prev=None, step_events=None, check=True, defer=False):
        """Device half: the catalogue all-gather (written into the device halo table),
        then the local step.  Records stay on the device (``fetch`` gathers them).
        ``defer``: the local step's status is checked by ``settle`` (local engines that
        support it), so the host can plan the next snapshot meanwhile."""
        p = prev if prev is not None else self.prev
        nh = len(sp.exists)
        if sp.rows is not None:
            self.local.set_catalogue(sp.lp, self._exchange(sp.rows, nh))
        kw = {}
        if defer and getattr(self.local, 'deferrable', False):
            kw['defer'] = True
        out = self.local.launch(sp.lp, None if p is None else p.lp, step_events, check, **kw)
        res = ShardedResult(n_slots=0, has_prog=np.zeros(nh, dtype=bool), bulk=sp.bulk_out,
                            lp=sp.lp)
        if sp.compare:
            pre = getattr(sp, 'has_prog_for', None)
            has_prog = pre[1] if pre is not None and pre[0] is p else np.isin(sp.exists, p.exists)
            res.has_prog, res.n_slots = has_prog, int(has_prog.sum())
            res.records, res.prev_prep = out, p
        return res

    def step(self, snapshot, centres, bulk_cat, H, z, exists, compare, angles_in=None,
             angles_layout=None, defer=False):
        """One snapshot on every rank.  ``defer`` (track_orbits' pipelined driver): the
        host half of this snapshot (shard, plan) runs while the previous step's kernels
        run; that step is settled (re-run on an LDS overflow, locally) before this one
        launches, and this one returns without waiting for its kernels."""
        if compare and self.prev is None:
            raise RuntimeError('compare step without a previous snapshot')
        sp = self.prepare(snapshot, centres, bulk_cat, H, z, exists, compare, angles_in,
                          angles_layout=angles_layout)
        if self._pending is not None and self.settle(self._pending) and compare:
            # this rank's previous step was re-planned: plan this one again locally on
            # its new layout (the shard and the collectives stand)
            sp.lp = self._local_prepare(sp, self.prev.lp)
        res = self.launch(sp, defer=defer)
        if defer and compare and getattr(self.local, 'deferrable', False):
            self._pending = res
        self.prev = sp
        return res

    def settle(self, res=None):
        """Wait for a deferred step (default: the pending one) and re-run it locally if
        its kernels asked for a re-plan.  True when it was re-run."""
        res = self._pending if res is None else res
        if res is None or res.lp is None or not hasattr(res.lp, 'pending'):
            if res is not None and res is self._pending:
                self._pending = None
            return False
        if res is self._pending:
            self._pending = None
        out = self.local.settle(res.lp)
        if out is None:
            return False
        res.records = out
        return True

    def step_ready(self, res):
        f = getattr(self.local, 'ready', None)
        return True if f is None or res.lp is None else f(res.lp)

    # ---------------------------------------------------------------- outputs
    def fetch_async(self, res, ids_dtype):
        """Start moving a step's records to the host for rank 0 (the only writer);
        ``wait()`` returns (offsets, IDs, f16 angles) in the reference's order
        (track_orbits.py:199-227, 315-316) on rank 0 and zero offsets elsewhere.

        World > 1 (``host_share.SharedRecordStage``): every rank computes its own
        records' final positions from the all-gathered (rank, halo slot) counts --
        a count scan (presharded) or a bitmap rank over the global previous rows
        (stripes) -- and stores them into one page-locked host buffer that every rank
        maps, over its own PCIe link; rank 0 moves only its own records and waits for the
        others' epochs.  World 1: one D2H into reused page-locked blocks.  Both run on a
        side stream behind the step's own kernels only, so they overlap whatever the
        compute stream runs next (the next snapshot's step); the workspace holding the
        records is not reused before them."""
        self.settle(res)
        offs, a_ids, a_ang, a_pos = res.records
        lp = res.lp
        done = self.local.done_event(lp) if hasattr(self.local, 'done_event') else None
        dev = offs.device
        side = None
        if dev.type == 'cuda':
            if self._side is None:
                # high priority: its own hardware queue (engine.fetch_async)
                self._side = torch.cuda.Stream(device=dev, priority=-1)
            side = self._side
        ctx = torch.cuda.stream(side) if side is not None else _nullcontext()
        S = res.n_slots
        root = self.rank == self.ROOT
        prof = self.profile_fetch
        if self.world > 1:
            from .host_share import SharedRecordStage
            if self._stage is None:
                self._stage = SharedRecordStage(self.group, self.rank, self.world, self.ROOT)
            with ctx:
                if side is not None and done is not None:
                    side.wait_event(done)
                    done.synchronize()            # the record count's host copy (launch)
                total = self.local.total(lp) if hasattr(self.local, 'total') else int(offs[-1])
                cnt = (offs[1:S + 1] - offs[:S]).to(torch.int64)
                rows = n_rows = None
                if not self.presharded:
                    pp = res.prev_prep
                    rows = pp.sel[a_pos[:total].to(pp.sel.device).long()]
                    n_rows = int(pp.n_global)
                stats = {} if prof else None
                lib = getattr(getattr(self.local, 'engine', None), 'lib', None)
                f = self._stage.fetch(lib, side, done, offs, a_ids, a_ang, total, cnt, S,
                                      ids_dtype, rows=rows, n_rows=n_rows,
                                      comm_dev=_comm_device(), profile=stats)
                if prof:
                    stats['bytes_per_record'] = a_ids.element_size() + 2
                    self.fetch_stats = stats
                if side is not None:
                    ev = torch.cuda.Event()
                    ev.record(side)
                    if hasattr(self.local, 'records_consumed'):
                        self.local.records_consumed(lp, ev)
            return f
        # world 1: this rank's records are the whole output and already in the
        # reference's order (its shard is the snapshot): one D2H into reused page-locked
        # blocks, no placement
        with ctx:
            if side is not None and done is not None:
                side.wait_event(done)
                done.synchronize()                # the record count's host copy (launch)
            total = self.local.total(lp) if hasattr(self.local, 'total') else int(offs[-1])
            ev = None
            pin = offs.device.type == 'cuda'
            if pin:
                from .engine import _pinned
                h_off = _pinned(S + 1, torch.int64)
                h_ids = _pinned(total, a_ids.dtype)
                h_ang = _pinned(total, torch.int16)
            else:
                h_off = torch.empty(S + 1, dtype=torch.int64)
                h_ids = torch.empty(total, dtype=a_ids.dtype)
                h_ang = torch.empty(total, dtype=torch.int16)
            h_off.copy_(offs[:S + 1].to(torch.int64), non_blocking=pin)
            h_ids.copy_(a_ids[:total], non_blocking=pin)
            h_ang.copy_(a_ang[:total].view(torch.int16) if a_ang.dtype != torch.int16
                        else a_ang[:total], non_blocking=pin)
            if prof:
                self.fetch_stats = dict(records=total, own_records=total, place_ms=0.0,
                                        bytes_moved=total * (a_ids.element_size() + 2),
                                        bytes_per_record=a_ids.element_size() + 2,
                                        layout='presharded' if self.presharded else 'stripes')
            if side is not None:
                ev = torch.cuda.Event()
                ev.record(side)
                if hasattr(self.local, 'records_consumed'):
                    self.local.records_consumed(lp, ev)
        return ShardedFetch(ev, S, h_off, h_ids, h_ang, ids_dtype, root)

    def fetch(self, res, ids_dtype):
        """``fetch_async(...).wait()``: the records in the reference's order on rank 0."""
        return self.fetch_async(res, ids_dtype).wait()

    def bulk_velocities(self, res, plan):
        return res.bulk

    def angles(self):
        """Global float16 angle state in current-snapshot order (checkpoint payload) on
        rank 0, None on the other ranks.  World > 1: every rank stores its angles at
        their global rows in one shared page-locked buffer (``host_share``), so no rank's
        angles cross another rank's link."""
        self.settle()
        p = self.prev
        if self.world > 1:
            from .host_share import SharedRecordStage
            if self._stage is None:
                self._stage = SharedRecordStage(self.group, self.rank, self.world, self.ROOT)
            vals = self.local.angles_tensor()
            lib = getattr(getattr(self.local, 'engine', None), 'lib', None)
            return self._stage.place_rows(lib, vals, p.sel, p.n_global, _comm_device())
        loc = self.local.angles_tensor().to(torch.int64)
        rows = torch.stack([p.sel.to(loc.device), loc], dim=1) if loc.numel() else \
            torch.zeros((0, 2), dtype=torch.int64, device=loc.device)
        allr, = gather_rows(self.group, self.ROOT, rows)
        if self.rank != self.ROOT:
            return None
        allr = allr.cpu().numpy()
        out = np.zeros(p.n_global, dtype=np.uint16)
        out[allr[:, 0]] = allr[:, 1].astype(np.uint16)
        return out.view(np.float16)

    def checkpoint_layout(self):
        """Row layout of ``angles()`` (None: the global snapshot's own row order)."""
        return self.prev.layout if self.prev is not None else None


class EngineLocal:
    """Per-rank compute on this rank's GPU: the HIP ``OrbitEngine``."""

    def __init__(self, engine):
        self.engine = engine
        self.mode = engine.mode
        self.device = engine.device
        engine.emit_positions = True

    def reset(self):
        self.engine.reset()

    def prepare(self, shard, centres, bulk, H, z, exists, compare, angles_in, prev_lp, share):
        eng = self.engine
        layout = None
        if compare and prev_lp is not None:
            layout = (prev_lp.starts, prev_lp.counts, prev_lp.exists, prev_lp.plan, prev_lp.n,
                      prev_lp.buckets)
        lp = eng.prepare(shard, centres, bulk, H, z, exists, compare, angles_in=angles_in,
                         plan_src=shard, prev_layout=layout)
        lp.exists = np.asarray(exists)
        lp.src = (shard, centres, bulk, H, z, exists, compare, angles_in, layout)
        lp.share_bulk = bool(share)
        return lp

    def set_catalogue(self, lp, rows):
        """The exchanged catalogue rows into the device halo table (centre, and the
        bulk velocity when it comes from the catalogue)."""
        from . import _native as N
        hv = lp.halos.view(torch.float64).view(-1, N.HALO_DTYPE.itemsize // 8)
        hi = 10 if lp.share_bulk else 7
        hv[:, 4:hi] = rows[:, :hi - 4].to(hv.device, non_blocking=True)

    deferrable = True                  # launch(defer=True) + settle (ShardedEngine.step)

    def _prev_state(self, lp, prev_lp):
        from .engine import SnapshotState
        if not (lp.compare and prev_lp is not None):
            return None
        return SnapshotState.of(prev_lp, prev_lp.exists)

    def _set_prev(self, lp):
        from .engine import SnapshotState
        self.engine.prev = SnapshotState.of(lp, lp.exists)

    def _replan(self, lp, st):
        """The step re-planned after status ``st`` (smaller items / large halos on the
        global-table path), in place; the exchanged catalogue rows are kept."""
        from .engine import retry_plan
        eng = self.engine
        eng.note_status(st)
        entries, part = retry_plan(lp, st)
        shard, centres, bulk, H, z, exists, compare, angles_in, layout = lp.src
        from . import _native as N
        w = N.HALO_DTYPE.itemsize // 8
        cat = lp.halos.view(torch.float64).view(-1, w)[:, 4:10].clone()    # centre + bulk
        lp2 = eng.prepare(shard, centres, bulk, H, z, exists, compare, angles_in=angles_in,
                          plan_src=shard, prev_layout=layout, entries=entries, part=part)
        lp2.halos.view(torch.float64).view(-1, w)[:, 4:10] = cat
        lp2.exists, lp2.src, lp2.share_bulk = lp.exists, lp.src, lp.share_bulk
        lp2.ws_idx = getattr(lp, 'ws_idx', eng._wsi)
        lp.__dict__.update(lp2.__dict__)

    def launch(self, lp, prev_lp, step_events=None, check=True, defer=False):
        """The local step.  A compare step writes one of the engine's workspaces
        (alternating, so the previous step's records can still be on their way to rank
        0); ``defer``: return without reading the status word -- it is copied to host
        memory behind an event and ``settle`` checks it (and re-runs) before the next
        launch.  Returns (offsets, IDs, f16 bits, previous-state rows) on the device."""
        eng = self.engine
        if lp.compare and not hasattr(lp, 'ws_idx'):
            lp.ws_idx = eng._advance_ws()
        for _ in range(10):
            ws = eng.workspace(lp, lp.ws_idx) if lp.compare else None
            if ws is not None:
                if ws.copy_done is not None:
                    # the last records of this workspace may still be gathered / copied
                    torch.cuda.current_stream(eng.device).wait_event(ws.copy_done)
                    ws.copy_done = None
                ws.status.zero_()
            res = eng.launch(lp, ws, prev=self._prev_state(lp, prev_lp), step_events=step_events)
            lp.res = res
            if ws is not None:
                ws.post_status(eng.lib, torch.cuda.current_stream(eng.device))
                res.done = torch.cuda.Event()
                res.done.record(torch.cuda.current_stream(eng.device))
            if ws is None or not check:
                break
            if defer:
                lp.pending = prev_lp
                break
            res.done.synchronize()
            st = int(ws.h_status[0])
            if not st:
                break
            self._replan(lp, st)
        else:
            raise RuntimeError('LDS hash tables kept overflowing')
        self._set_prev(lp)
        if not lp.compare:
            return None
        return res.offsets, res.apsis_ids, res.apsis_ang, res.apsis_pos

    def settle(self, lp):
        """Wait for a deferred step; re-run it if its kernels asked for a re-plan.
        Returns the new device records when it was re-run, else None."""
        prev_lp = getattr(lp, 'pending', None)
        if prev_lp is None and not hasattr(lp, 'pending'):
            return None
        del lp.pending
        lp.res.done.synchronize()
        st = int(lp.res.ws.h_status[0])
        if not st:
            return None
        self._replan(lp, st)
        return self.launch(lp, prev_lp, check=True)

    def ready(self, lp):
        """Without waiting: None while a deferred step runs, else whether its records
        are final (False: it will be re-run)."""
        if not hasattr(lp, 'pending'):
            return True
        if not lp.res.done.query():
            return None
        return not int(lp.res.ws.h_status[0])

    def total(self, lp):
        """The step's record count (host copy behind its event; settle first)."""
        return int(lp.res.ws.h_total[0])

    def done_event(self, lp):
        return getattr(getattr(lp, 'res', None), 'done', None)

    def records_consumed(self, lp, event):
        """The records of ``lp``'s workspace are read once ``event`` completes."""
        ws = getattr(getattr(lp, 'res', None), 'ws', None)
        if ws is not None:
            ws.copy_done = event

    def angles_tensor(self):
        """float16 bits of the current angle state (low half of the meta words)."""
        return self.engine.state_meta() & 0xFFFF

    def bulk(self, snapshot, halo_idx):
        return self.engine.block_bulk(snapshot, halo_idx)
