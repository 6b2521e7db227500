"""Multi-GPU orbit tagging: particles sharded by ID range across ranks.

One process per GPU, ``torch.distributed`` (RCCL on MI355X, gloo on CPU).  Every
rank runs the same ``track_orbits`` driver.  The reference's only parallel axis is
the halo pool of track_orbits.py:189-194; here the axis is the particle ID instead:
rank r owns the IDs of one contiguous range (``IdRangeOwner``, the default), so a
particle's current and previous rows -- including its copies in overlapping regions
-- sit on the same rank, and the join needs no exchange.  The data path is
collective-free and everything in it stays on the rank's device:

* **shard**: with a loader that returns the whole snapshot on every rank (the
  reference's callback contract, track_orbits.py:118-122), each rank moves it to its
  GPU once and keeps its rows with a device mask + compaction (the block order is
  preserved, and every kept row remembers its position in its global block, gpos).
  A *presharded* loader (``presharded=True``, e.g. a distributed reader) hands each
  rank its own rows directly; the global block is then the rank-ordered
  concatenation of the ranks' blocks.
* **step**: the rank's ``OrbitEngine`` on its shard; the kernel also emits each apsis
  record's previous-state row, which maps to its global previous-block position
  through the previous snapshot's gpos (a device gather).
* **records** stay on the device as (halo slot << 32 | gpos, ID, f16 angle).

Collectives per snapshot (all small):

* one all-gather of the halo catalogue rows (centre, bulk velocity): every rank then
  uses rank 0..N-1's identical rows (the north star's "all-gather of halo centres");
* bulk velocities computed from the particles (no catalogue value,
  track_orbits.py:269-280) are sequential sums over a WHOLE block, which no
  partial-sum exchange reproduces bit for bit: halo j's owner rank (j % world)
  computes them on the full block and the rows are all-gathered (not available with
  presharded snapshots);
* output: ``fetch`` (the savefile path, outside the per-snapshot tagging) all-gathers
  the records and sorts them by key -- exactly the reference's order (previous-block
  order within each halo, halos in ``halo_exists`` order, track_orbits.py:199-227,
  315-316).  Checkpoint angles are gathered with their global row index.

``ShardedEngine`` exposes the ``OrbitEngine`` interface the driver uses, so
``track_orbits(..., engine=ShardedEngine(EngineLocal(OrbitEngine())))`` is the
multi-GPU drop-in.
"""
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

U64 = np.uint64
_HASH_C = np.int64(-7046029254386353131)        # 0x9E3779B97F4A7C15 as int64


# ------------------------------------------------------------------ ownership
class HashOwner:
    """rank = hash(ID) mod world (balanced for any ID distribution)."""

    def __call__(self, ids, world):
        h = np.asarray(ids).astype(np.int64, copy=False) * _HASH_C     # wrapping int64
        return ((h >> 33) & 0x7FFFFFFF) % world

    def fit(self, ids):
        pass

    def mask(self, ids_t, world, rank):
        h = ids_t.to(torch.int64) * int(_HASH_C)
        return ((h >> 33) & 0x7FFFFFFF) % world == rank


class IdRangeOwner:
    """rank = floor((ID - lo) * world / (hi - lo)), clipped: contiguous ID ranges.
    Without bounds, [lo, hi) is taken from the first snapshot the engine sees (every
    rank sees the same one); later IDs outside it go to the first / last rank.
    IDs are taken as their int64 bit patterns (uint64 IDs >= 2^63 sort below the
    others, as device tensors hold them), and the ratio is evaluated in float64 (the
    same operations on the host and the device)."""

    def __init__(self, lo=None, hi=None):
        self.lo = None if lo is None else int(lo)
        self.hi = None if hi is None else int(hi)

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

    def __call__(self, ids, world):
        span = float(max(self.hi - self.lo, 1))
        v = self._i64(ids).astype(np.float64)
        r = np.floor((v - float(self.lo)) * world / span)
        return np.clip(r, 0, world - 1).astype(np.int64)

    def mask(self, ids_t, world, rank):
        span = float(max(self.hi - self.lo, 1))
        r = torch.floor((ids_t.to(torch.int64).to(torch.float64) - float(self.lo)) * world / span)
        return r.clamp_(0, world - 1) == rank


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


# ------------------------------------------------------------------ collectives
def _comm_device():
    import torch.distributed as dist
    return torch.device('cuda', torch.cuda.current_device()) \
        if dist.get_backend() == 'nccl' else torch.device('cpu')


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


def _f64_bits(x):
    return np.ascontiguousarray(x, dtype=np.float64).view(np.int64)


def _as_i64(t):
    """IDs of any 32/64-bit integer dtype as int64 values (bit pattern kept for 64-bit)."""
    return t if t.dtype == torch.int64 else t.to(torch.int64)


# ------------------------------------------------------------------ engine facade
@dataclass
class ShardedResult:
    n_slots: int
    has_prog: np.ndarray
    records: Optional[tuple] = None          # device (offsets, ids, f16 bits, prev-state row)
    gpos_prev: Optional[torch.Tensor] = None # previous shard row -> global block position
    bulk: Optional[np.ndarray] = None


@dataclass
class ShardedPrep:
    """One snapshot's host half (ShardedEngine.prepare): the shard, its rows' global
    block positions and the local engine's prepared step."""
    n: int
    exists: np.ndarray
    compare: bool
    gpos: torch.Tensor
    sel: torch.Tensor                       # this rank's rows in the global snapshot
    n_global: int
    rows: Optional[np.ndarray]              # catalogue rows (centre, bulk) to exchange
    bulk_out: Optional[np.ndarray]
    plan: object
    lp: object = None


class _Plan:
    def __init__(self, ids_dtype, bulk_dtype=None):
        self.ids = np.dtype(ids_dtype)
        self.bulk = bulk_dtype


class ShardedEngine:
    """``OrbitEngine`` interface over ID-sharded ranks (see module docstring).

    ``step`` = ``prepare`` (host: shard, plan, uploads) + ``launch`` (the catalogue
    all-gather and the device step).  The two halves are public so a benchmark can
    prepare a chain of snapshots and time ``launch`` alone, as bench.py does."""

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

    def reset(self):
        self.prev = None
        self.local.reset()

    # ---------------------------------------------------------------- collectives
    def _exchange(self, rows, nh):
        """The one per-snapshot all-gather of catalogue rows: rank r contributes halos
        [r * nl, (r + 1) * nl) of its (nh, 6) float64 rows; every rank gets all nh."""
        import torch.distributed as dist
        nl = -(-nh // self.world)
        mine = np.zeros((nl, 6), dtype=np.float64)
        lo, hi = self.rank * nl, min((self.rank + 1) * nl, nh)
        if hi > lo:
            mine[:hi - lo] = rows[lo:hi]
        dev = _comm_device()
        out = torch.empty((nl * self.world, 6), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(out, torch.from_numpy(mine).to(dev), group=self.group)
        return out[:nh]

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

    # ---------------------------------------------------------------- shard
    def _tensor(self, x):
        if isinstance(x, torch.Tensor):
            return x.to(self.device)
        a = np.ascontiguousarray(x)
        if a.dtype.kind == 'u':
            a = a.view(a.dtype.str.replace('u', 'i'))
        return torch.from_numpy(a).to(self.device)

    def _shard(self, snapshot, starts, counts):
        """Device shard of a whole snapshot: this rank's rows, block order kept."""
        nh = len(starts)
        ids_t = self._tensor(snapshot['ids'])
        self.owner.fit(ids_t)
        keep = self.owner.mask(ids_t, self.world, self.rank)
        sel = torch.nonzero(keep).squeeze(1)
        st_t = torch.from_numpy(starts).to(self.device)
        block = torch.searchsorted(st_t, sel, right=True) - 1 if nh else sel
        cnt = torch.bincount(block, minlength=nh) if nh else torch.zeros(0, dtype=torch.int64)
        gpos = sel - st_t[block] if nh else sel
        shard = dict(snapshot)
        shard['ids'] = ids_t[sel]
        for k in ('coordinates', 'velocities'):
            shard[k] = self._tensor(snapshot[k]).reshape(-1, 3)[sel]
        if isinstance(snapshot['masses'], (np.ndarray, torch.Tensor)):
            shard['masses'] = self._tensor(snapshot['masses'])[sel]
        cnt_h = cnt.cpu().numpy().astype(np.int64)
        shard['region_offsets'] = np.concatenate([[0], np.cumsum(cnt_h)[:-1]]).astype(np.int64) \
            if nh else cnt_h
        return shard, sel, gpos

    def _presharded_gpos(self, starts, counts):
        """Global block = the ranks' blocks concatenated in rank order: a shard row's
        position is the rows of lower ranks in its block + its own index.  Returns the
        block positions, the global snapshot rows and the global row count."""
        cnt_all = allgather_v(torch.from_numpy(counts.astype(np.int64))[None, :], self.group)
        before = cnt_all[:self.rank].sum(0).to(self.device) if self.rank else \
            torch.zeros(len(counts), dtype=torch.int64, device=self.device)
        tot = cnt_all.sum(0).to(self.device)
        gstart = torch.cumsum(tot, 0) - tot
        c = torch.from_numpy(counts).to(self.device)
        block = torch.repeat_interleave(torch.arange(len(counts), device=self.device), c)
        local = torch.arange(int(c.sum()), device=self.device) - \
            torch.from_numpy(starts).to(self.device)[block]
        gpos = before[block] + local
        return gpos, gstart[block] + gpos, int(tot.sum())

    # ---------------------------------------------------------------- step
    def prepare(self, snapshot, centres, bulk_cat, H, z, exists, compare, angles_in=None,
                prev=None):
        """Host half of a step; ``prev`` (a ShardedPrep) defaults to the last step."""
        exists = np.asarray(exists)
        ids = snapshot['ids']
        n = int(ids.numel()) if isinstance(ids, torch.Tensor) else len(ids)
        starts, counts = block_layout(snapshot['region_offsets'], n)
        nh = len(starts)
        bulk = bulk_cat
        if bulk_cat is None and nh:
            if self.presharded:
                raise NotImplementedError('computed bulk velocities need whole blocks: give '
                                          'catalogue bulk velocities with presharded snapshots')
            bulk = self._bulk(snapshot, nh)
        if self.presharded:
            # this rank's rows as they are; host arrays (a distributed reader) move to
            # the rank's device once
            shard, sel = dict(snapshot), None
            for k in ('ids', 'coordinates', 'velocities'):
                shard[k] = self._tensor(snapshot[k])
            if isinstance(snapshot['masses'], (np.ndarray, torch.Tensor)):
                shard['masses'] = self._tensor(snapshot['masses'])
            gpos, sel, n_global = self._presharded_gpos(starts, counts)
            # a checkpoint holds the global snapshot's angles (rank-major blocks)
            a_in = None if angles_in is None else np.asarray(angles_in)[sel.cpu().numpy()]
        else:
            shard, sel, gpos = self._shard(snapshot, starts, counts)
            n_global = n
            a_in = None if angles_in is None else np.asarray(angles_in)[sel.cpu().numpy()]
        rows = None
        if self.share_catalogue and nh:
            rows = np.zeros((nh, 6), dtype=np.float64)
            rows[:, :3] = np.asarray(centres, dtype=np.float64).reshape(nh, 3)
            if bulk_cat is not None:
                rows[:, 3:] = np.asarray(bulk_cat, dtype=np.float64).reshape(nh, 3)
        p = prev if prev is not None else self.prev
        ids_dt = np.asarray(ids[:0].cpu() if isinstance(ids, torch.Tensor) else ids[:0]).dtype
        sp = ShardedPrep(n=n, exists=exists, compare=bool(compare), gpos=gpos, sel=sel,
                         n_global=n_global,
                         rows=rows, bulk_out=None if bulk_cat is not None else bulk,
                         plan=_Plan(ids_dt, None if bulk is None else np.asarray(bulk).dtype))
        sp.lp = self.local.prepare(shard, centres, bulk, H, z, exists, compare, a_in,
                                   None if (prev is None or p is None) else p.lp,
                                   share=bulk_cat is not None)
        return sp

    def launch(self, sp, prev=None, step_events=None, check=True):
        """Device half: the catalogue all-gather (written into the device halo table),
        then the local step.  Records stay on the device (``fetch`` gathers them)."""
        p = prev if prev is not None else self.prev
        nh = len(sp.exists)
        if sp.rows is not None:
            self.local.set_catalogue(sp.lp, self._exchange(sp.rows, nh))
        out = self.local.launch(sp.lp, None if prev is None else prev.lp, step_events, check)
        res = ShardedResult(n_slots=0, has_prog=np.zeros(nh, dtype=bool), bulk=sp.bulk_out)
        if sp.compare:
            has_prog = np.isin(sp.exists, p.exists)
            res.has_prog, res.n_slots = has_prog, int(has_prog.sum())
            res.records, res.gpos_prev = out, p.gpos
        return res

    def step(self, snapshot, centres, bulk_cat, H, z, exists, compare, angles_in=None):
        if compare and self.prev is None:
            raise RuntimeError('compare step without a previous snapshot')
        sp = self.prepare(snapshot, centres, bulk_cat, H, z, exists, compare, angles_in)
        res = self.launch(sp)
        self.prev = sp
        return res

    # ---------------------------------------------------------------- outputs
    def fetch(self, res, ids_dtype):
        """Gather every rank's records and put them in the reference's order: key =
        halo slot << 32 | position in the global previous block."""
        offs, a_ids, a_ang, a_pos = res.records
        total = int(offs[-1])
        slot = torch.repeat_interleave(torch.arange(res.n_slots, device=offs.device),
                                       (offs[1:] - offs[:-1]).long())
        g = res.gpos_prev[a_pos[:total].to(res.gpos_prev.device).long()]
        key = allgather_v((slot.to(g.device) << 32) | g, self.group)
        ids = allgather_v(_as_i64(a_ids[:total]), self.group)
        ang = allgather_v(a_ang[:total].to(torch.int32), self.group)   # (gloo has no int16)
        order = torch.argsort(key)
        key, ids, ang = key[order], ids[order], ang[order]
        cnt = torch.bincount((key >> 32).long(), minlength=res.n_slots)[:res.n_slots] \
            if key.numel() else torch.zeros(res.n_slots, dtype=torch.int64)
        offsets = np.concatenate([[0], np.cumsum(cnt.cpu().numpy())]).astype(np.int64)
        dt = np.dtype(ids_dtype)
        ids_h = ids.cpu().numpy()
        ids_h = ids_h.view(np.uint64).astype(dt) if dt.kind == 'u' else ids_h.astype(dt)
        return offsets, ids_h, ang.cpu().numpy().astype(np.uint16).view(np.float16)

    def bulk_velocities(self, res, plan):
        return res.bulk

    def angles(self):
        """Global float16 angle state in current-snapshot order (checkpoint payload)."""
        p = self.prev
        loc = self.local.angles_tensor().to(torch.int64)
        rows = torch.stack([p.sel.to(loc.device), loc], dim=1) if loc.numel() else \
            torch.zeros((0, 2), dtype=torch.int64)
        allr = allgather_v(rows, self.group).cpu().numpy()
        out = np.zeros(p.n_global, dtype=np.uint16)
        out[allr[:, 0]] = allr[:, 1].astype(np.uint16)
        return out.view(np.float16)


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
        from .engine import SnapshotState  # noqa: F401
        eng = self.engine
        layout = None
        if compare and prev_lp is not None:
            layout = (prev_lp.starts, prev_lp.counts, prev_lp.exists, prev_lp.plan, prev_lp.n)
        lp = eng.prepare(shard, centres, bulk, H, z, exists, compare, angles_in=angles_in,
                         plan_src=shard, prev_layout=layout)
        lp.exists = np.asarray(exists)
        lp.src = (shard, centres, bulk, H, z, exists, compare, angles_in, layout)
        lp.share_bulk = bool(share)
        return lp

    def set_catalogue(self, lp, rows):
        """The exchanged catalogue rows into the device halo table (centre, and the
        bulk velocity when it comes from the catalogue)."""
        hv = lp.halos.view(torch.float64).view(-1, 12)
        hi = 10 if lp.share_bulk else 7
        hv[:, 4:hi] = rows[:, :hi - 4].to(hv.device, non_blocking=True)

    def launch(self, lp, prev_lp, step_events=None, check=True):
        from .engine import SnapshotState, retry_plan
        eng = self.engine
        for _ in range(10):
            ws = eng.workspace(lp) if lp.compare else None
            prev = None
            if lp.compare and prev_lp is not None:
                prev = SnapshotState(ids=prev_lp.snap['ids'], rhat=prev_lp.rhat, meta=prev_lp.meta,
                                     starts=prev_lp.starts, counts=prev_lp.counts,
                                     exists=prev_lp.exists, plan=prev_lp.plan)
            if check and ws is not None:
                ws.status.zero_()
            res = eng.launch(lp, ws, prev=prev, step_events=step_events)
            st = int(ws.status[0].item()) if (check and ws is not None) else 0
            if not st:
                break
            # re-plan: smaller items / large halos on the global-table path
            entries, part = retry_plan(lp, st)
            shard, centres, bulk, H, z, exists, compare, angles_in, layout = lp.src
            hv = lp.halos.view(torch.float64).view(-1, 12)[:, 4:10].clone()
            lp2 = eng.prepare(shard, centres, bulk, H, z, exists, compare, angles_in=angles_in,
                              plan_src=shard, prev_layout=layout, entries=entries, part=part)
            lp2.halos.view(torch.float64).view(-1, 12)[:, 4:10] = hv
            lp2.exists, lp2.src, lp2.share_bulk = lp.exists, lp.src, lp.share_bulk
            lp.__dict__.update(lp2.__dict__)
        else:
            raise RuntimeError('LDS hash tables kept overflowing')
        eng.prev = SnapshotState(ids=lp.snap['ids'], rhat=lp.rhat, meta=lp.meta, starts=lp.starts,
                                 counts=lp.counts, exists=lp.exists, plan=lp.plan)
        if not lp.compare:
            return None
        return res.offsets, res.apsis_ids, res.apsis_ang, res.apsis_pos

    def angles_tensor(self):
        """float16 bits of the current angle state (low half of the meta words)."""
        return self.engine.prev.meta & 0xFFFF

    def bulk(self, snapshot, halo_idx):
        return self.engine.block_bulk(snapshot, halo_idx)
