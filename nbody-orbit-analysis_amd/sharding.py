"""Multi-GPU orbit tagging: particles sharded by ID across ranks.

One process per GPU, ``torch.distributed`` (RCCL on MI355X, gloo on CPU).  Every
rank runs the same ``track_orbits`` driver; the loader may return the whole
snapshot on every rank (the reference's callback contract, track_orbits.py:118-122)
and each rank keeps the rows whose ID it owns.  Because ownership is a function of
the ID, a particle's current and previous rows -- including its copies in
overlapping regions -- sit on the same rank, so the join needs no exchange: the
data path is collective-free and scales weakly.

Collectives per snapshot (small, all-gather only):

* bulk velocities computed from the particles (no catalogue value,
  track_orbits.py:269-280) are sequential sums over a WHOLE block, which no
  partial-sum exchange reproduces bit-for-bit; halo j's owner rank (j % world)
  computes them on the full block and the rows are all-gathered;
* apsis records (halo slot, position in the global previous block, ID, f16 angle)
  are all-gathered and merged by (slot, position): exactly the reference's output
  order (prev-block order within each halo, halos in ``halo_exists`` order,
  track_orbits.py:199-227, 315-316);
* checkpoint angles are all-gathered with their global row index.

``ShardedEngine`` exposes the ``OrbitEngine`` interface the driver uses, so
``track_orbits(..., engine=ShardedEngine(...))`` is the multi-GPU drop-in.  The
per-rank compute is a *local* object with ``step`` / ``angles`` / ``bulk``;
``EngineLocal`` wraps the HIP engine (the product path).
"""
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

U64 = np.uint64


# ------------------------------------------------------------------ ownership
class HashOwner:
    """rank = hash(ID) mod world (balanced for any ID distribution)."""

    def __call__(self, ids, world):
        h = np.asarray(ids).astype(np.int64, copy=False).view(U64) * U64(0x9E3779B97F4A7C15)
        return ((h >> U64(33)) % U64(world)).astype(np.int64)


class IdRangeOwner:
    """rank = floor((ID - lo) * world / (hi - lo)): contiguous ID ranges."""

    def __init__(self, lo, hi):
        self.lo, self.hi = int(lo), int(hi)

    def __call__(self, ids, world):
        ids = np.asarray(ids).astype(np.int64)
        span = max(self.hi - self.lo, 1)
        r = ((ids - self.lo).astype(np.float64) * world / span).astype(np.int64)
        return np.clip(r, 0, world - 1)


def block_layout(region_offsets, n):
    starts = np.asarray(region_offsets, dtype=np.int64).reshape(-1)
    counts = np.append(starts[1:], n) - starts
    return starts, counts


def shard_snapshot(snapshot, keep):
    """Rows of ``snapshot`` selected by boolean ``keep`` (block order preserved).

    Returns (shard dict, global row index of every kept row, shard block starts,
    shard block counts)."""
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


# ------------------------------------------------------------------ collectives
def _comm_device():
    import torch.distributed as dist
    return torch.device('cuda', torch.cuda.current_device()) \
        if dist.get_backend() == 'nccl' else torch.device('cpu')


def allgather_rows(a, group=None):
    """Variable-length all-gather of a 2-D int64 array; rank-ordered concatenation."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = _comm_device()
    a = np.ascontiguousarray(a, dtype=np.int64)
    if a.ndim != 2:
        raise ValueError('allgather_rows expects a 2-D array')
    width = a.shape[1]
    n = torch.tensor([a.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    m = max(max(ns), 1)
    buf = torch.zeros((m, width), dtype=torch.int64, device=dev)
    if a.shape[0]:
        buf[:a.shape[0]] = torch.from_numpy(a).to(dev)
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return np.concatenate([o[:k].cpu().numpy() for o, k in zip(outs, ns)], axis=0)


def _f64_bits(x):
    return np.ascontiguousarray(x, dtype=np.float64).view(np.int64)


# ------------------------------------------------------------------ engine facade
@dataclass
class ShardedResult:
    n_slots: int
    has_prog: np.ndarray
    offsets: Optional[np.ndarray] = None
    ids: Optional[np.ndarray] = None
    angles: Optional[np.ndarray] = None
    bulk: Optional[np.ndarray] = None


@dataclass
class _Prev:
    ids: np.ndarray            # shard IDs (loader dtype), shard order
    gpos: np.ndarray           # position of each shard row inside its global block
    starts: np.ndarray         # shard block starts / counts per halo
    counts: np.ndarray
    exists: np.ndarray
    plan: object = None
    sel: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    n_global: int = 0


class _Plan:
    def __init__(self, ids_dtype, bulk_dtype=None):
        self.ids = np.dtype(ids_dtype)
        self.bulk = bulk_dtype


class ShardedEngine:
    """``OrbitEngine`` interface over ID-sharded ranks (see module docstring)."""

    def __init__(self, local, group=None, owner=None, mode=None):
        import torch.distributed as dist
        self.local = local
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.owner = owner or HashOwner()
        self.mode = mode or local.mode
        self.prev: Optional[_Prev] = None

    def reset(self):
        self.prev = None
        self.local.reset()

    def _bulk(self, snapshot, nh):
        own = np.flatnonzero(np.arange(nh) % self.world == self.rank)
        b = np.asarray(self.local.bulk(snapshot, own)) if len(own) else np.zeros((0, 3))
        dt = b.dtype if len(own) else None
        rows = np.concatenate([own[:, None].astype(np.int64),
                               _f64_bits(b.reshape(-1, 3)).reshape(-1, 3)], axis=1)
        allr = allgather_rows(rows, self.group)
        dts = allgather_rows(np.array([[0 if dt is None else np.dtype(dt).itemsize]]),
                             self.group)[:, 0]
        size = int(dts.max())
        out = np.empty((nh, 3), dtype=np.float64)
        out[allr[:, 0]] = allr[:, 1:].copy().view(np.float64)
        return out.astype(np.float32 if size == 4 else np.float64)

    def step(self, snapshot, centres, bulk_cat, H, z, exists, compare, angles_in=None):
        exists = np.asarray(exists)
        ids = np.asarray(snapshot['ids'])
        n = len(ids)
        starts, counts = block_layout(snapshot['region_offsets'], n)
        nh = len(starts)
        bulk = bulk_cat
        if bulk_cat is None and nh:
            bulk = self._bulk(snapshot, nh)
        keep = self.owner(ids, self.world) == self.rank
        shard, sel, st, cnt = shard_snapshot(snapshot, keep)
        gpos = sel - np.repeat(starts, counts)[sel] if n else sel
        a_in = None if angles_in is None else np.asarray(angles_in)[sel]
        out = self.local.step(shard, centres, bulk, H, z, exists, compare, a_in)
        res = ShardedResult(n_slots=0, has_prog=np.zeros(nh, dtype=bool), bulk=(
            None if bulk_cat is not None else bulk))
        if compare:
            p = self.prev
            has_prog = np.isin(exists, p.exists)
            hinds = np.flatnonzero(has_prog)
            res.has_prog, res.n_slots = has_prog, len(hinds)
            offs, a_ids, a_ang = out
            recs = []
            for k, j in enumerate(hinds):
                lo, hi = int(offs[k]), int(offs[k + 1])
                if hi == lo:
                    continue
                q = int(np.searchsorted(p.exists, exists[j]))
                a, b = int(p.starts[q]), int(p.starts[q] + p.counts[q])
                blk = p.ids[a:b]
                sorter = np.argsort(blk, kind='stable')
                idx = sorter[np.searchsorted(blk, a_ids[lo:hi], sorter=sorter)]
                r = np.empty((hi - lo, 4), dtype=np.int64)
                r[:, 0] = k
                r[:, 1] = p.gpos[a:b][idx]
                r[:, 2] = np.asarray(a_ids[lo:hi]).astype(np.int64, copy=False)
                r[:, 3] = np.asarray(a_ang[lo:hi]).view(np.uint16)
                recs.append(r)
            mine = np.concatenate(recs) if recs else np.zeros((0, 4), dtype=np.int64)
            allr = allgather_rows(mine, self.group)
            order = np.lexsort((allr[:, 1], allr[:, 0]))
            allr = allr[order]
            res.offsets = np.concatenate([[0], np.cumsum(
                np.bincount(allr[:, 0], minlength=len(hinds)))]).astype(np.int64)
            res.ids = allr[:, 2].astype(ids.dtype)
            res.angles = allr[:, 3].astype(np.uint16).view(np.float16)
        self.prev = _Prev(ids=shard['ids'], gpos=gpos, starts=st, counts=cnt, exists=exists,
                          plan=_Plan(ids.dtype, None if bulk is None else
                                     np.asarray(bulk).dtype),
                          sel=sel, n_global=n)
        return res

    def fetch(self, res, ids_dtype):
        return res.offsets, res.ids.astype(ids_dtype, copy=False), res.angles

    def bulk_velocities(self, res, plan):
        return res.bulk

    def angles(self):
        """Global float16 angle state in current-snapshot order (checkpoint payload)."""
        p = self.prev
        loc = np.asarray(self.local.angles()).astype(np.float16).view(np.uint16)
        rows = np.stack([p.sel.astype(np.int64), loc.astype(np.int64)], axis=1) \
            if len(loc) else np.zeros((0, 2), dtype=np.int64)
        allr = allgather_rows(rows, self.group)
        out = np.zeros(p.n_global, dtype=np.uint16)
        out[allr[:, 0]] = allr[:, 1].astype(np.uint16)
        return out.view(np.float16)


class EngineLocal:
    """Per-rank compute on this rank's GPU: the HIP ``OrbitEngine``."""

    def __init__(self, engine):
        self.engine = engine
        self.mode = engine.mode

    def reset(self):
        self.engine.reset()

    def step(self, snapshot, centres, bulk, H, z, exists, compare, angles_in):
        res = self.engine.step(snapshot, centres, bulk, H, z, exists, compare,
                               angles_in=angles_in)
        if not compare:
            return None
        return self.engine.fetch(res, self.engine.prev.plan.ids)

    def angles(self):
        return self.engine.angles()

    def bulk(self, snapshot, halo_idx):
        return self.engine.block_bulk(snapshot, halo_idx)
