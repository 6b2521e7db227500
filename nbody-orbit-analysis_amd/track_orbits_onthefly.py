"""Drop-in on-the-fly driver: ``track_orbits`` of orbitanalysis/track_orbits_onthefly.py.

One call compares snapshot ``s`` with ``s - 1`` through ``progenitor_links`` (2, n)
(row 0: halos at s, row 1: their progenitors at s - 1, -1 = absent) and writes one
file per snapshot (``savefile.format('%0.3d' % s)``) with the reference's datasets
(track_orbits_onthefly.py:208-252):

    {peri|apo}center_offsets / _IDs  (key ``mode[:8] + 'er'``: apocentric ->
                                      'apocentrer', the reference's spelling)
    angles                           arccos(r̂_prev . r̂) of every matched particle
    entered_offsets / entered_IDs    setdiff1d(current, previous) per halo
    departed_offsets / departed_IDs  setdiff1d(previous, current) per halo
    progenitor_links, region_radii, region_positions, bulk_velocities, attr box_size

Both frames and the join run on the device (``OrbitEngine`` in on-the-fly mode:
r̂ in the coordinate dtype, no Hubble term, v_r in promote(velocity, coordinate);
track_orbits_onthefly.py:71-120).  The per-halo entered / departed lists are
compacted and sorted on the device from the kernel's match flags.
"""
import os
import time
from dataclasses import dataclass

import numpy as np
import torch

from . import _native as N
from .engine import OrbitEngine, SnapshotState, to_device, F64, np_dtype, is_array
from .sharding import _h2d

_TORCH = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64}


def repack(arr, length, inds):
    """track_orbits_onthefly.py:61-68: rows of absent halos filled with -1."""
    arr = np.asarray(arr)
    shape = list(np.shape(arr))
    shape[0] = length
    out = -np.ones(tuple(shape), dtype=arr.dtype)
    out[inds] = arr
    return out


def _block_starts(slices, n):
    """Repacked (start, end) rows (-1, -1 = absent) -> non-decreasing block starts that
    tile [0, n) (an absent halo gets an empty block)."""
    slices = np.asarray(slices, dtype=np.int64).reshape(-1, 2)
    present = slices[:, 0] >= 0
    if not present.any():
        return np.zeros(len(slices), dtype=np.int64)
    a, b = slices[:, 0], slices[:, 1]
    if np.any(present & (b < a)):
        return _block_starts_loop(slices)
    # an absent halo starts where the last present block before it ends (before the
    # first present one: where that one starts; rows before it are in no block), and
    # a present block may not start before that end: the running maximum of the present
    # blocks' ends (vectorised; 12,500 halos took 5.6 ms as a loop per call)
    first = int(a[present][0])
    run = np.maximum.accumulate(np.where(present, b, np.iinfo(np.int64).min))
    prev = np.empty_like(run)
    prev[0] = first
    prev[1:] = np.maximum(run[:-1], first)
    if np.any(present & (a < prev)):
        raise ValueError('region blocks must follow halo order')
    return np.where(present, a, prev)


def _block_starts_loop(slices):
    """_block_starts for rows with negative-size blocks (end < start): the running end
    then steps back, as the row-by-row rule does."""
    starts = np.empty(len(slices), dtype=np.int64)
    present = slices[:, 0] >= 0
    pos = int(slices[present, 0][0]) if present.any() else 0
    for j, (a, b) in enumerate(slices):
        if a >= 0:
            if a < pos:
                raise ValueError('region blocks must follow halo order')
            starts[j], pos = a, b
        else:
            starts[j] = pos
    return starts


def _sorted_unique_per_halo(lib, device, ids_t, counts, ids_dtype):
    """np.unique of each halo's rows (``ids_t``: device IDs grouped by halo, ``counts``
    rows per halo) on the device with the collation kernels (k_collate_new / _merge:
    per-halo LDS sort, run-length encoding, merge into an empty state).  Returns host
    (ids, offsets[nh + 1])."""
    from .postprocessing import _CollateState, _id_kind
    nh = len(counts)
    state = _CollateState(nh, device)
    n = int(ids_t.numel())
    signed = 1 if np.dtype(ids_dtype).kind == 'i' else 0
    if n:
        cnt = np.asarray(counts, dtype=np.int64)
        off = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.int64)
        zeros = torch.zeros(n, dtype=torch.int16, device=device)          # f16 0.0 angles
        keep = torch.ones(65536, dtype=torch.uint8, device=device)        # every row kept
        state.merge(lib, ids_t.contiguous(), _id_kind(ids_dtype, 'particle ID'), signed,
                    zeros, keep, off, cnt)
    ids, _ = state.export(lib, signed, np.dtype(ids_dtype))
    return ids, np.concatenate([[0], np.cumsum(state.lengths())]).astype(np.int64)


def _interleave_halos(take_a, a, a_off, b, b_off):
    """Per halo j: a[a_off[j]:a_off[j+1]] if take_a[j] else b[b_off[j]:b_off[j+1]],
    concatenated in halo order.  Returns (values, offsets)."""
    lens = np.where(take_a, np.diff(a_off), np.diff(b_off)).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    comb = np.concatenate([a, b]) if len(b) else a
    start = np.where(take_a, a_off[:-1], len(a) + b_off[:-1]).astype(np.int64)
    src = np.repeat(start - off[:-1], lens) + np.arange(off[-1], dtype=np.int64)
    return comb[src], off


class OnTheFly:
    """Pairwise (s, s-1) device pipeline on top of an ``OrbitEngine``."""

    def __init__(self, engine=None, mode='pericentric'):
        self.eng = engine if engine is not None else OrbitEngine(mode=mode)
        self.mode = self.eng.mode

    def _prepare(self, snap, slices, centres, compare, prev=None, entries=None, bulk=None):
        eng = self.eng
        n = len(snap['ids'])
        s = dict(snap)
        s['region_offsets'] = _block_starts(slices, n)
        dev = {k: to_device(snap[k], eng.device) for k in ('ids', 'coordinates', 'velocities')}
        dsnap = dict(s)
        dsnap.update(dev)
        if is_array(snap['masses']):
            dsnap['masses'] = to_device(snap['masses'], eng.device)
        nh = len(slices)
        layout = None
        if compare:
            layout = (prev.starts, prev.counts, prev.exists, prev.plan, prev.ids.numel())
        # bulk velocities computed from the blocks (:85-98), unless given (a shard's
        # rows do not hold whole blocks: ShardedOnTheFly passes the full-block ones)
        pr = eng.prepare(dsnap, centres, bulk, np.float64(0.0), 0.0, np.arange(nh), compare,
                         plan_src=s, prev_layout=layout, entries=entries, part=False)
        plan = pr.plan
        coord = np.dtype(plan.coord)
        # on-the-fly frame: r̂ stored in the coordinate dtype (:82-83, 112-113)
        pr.rhat = torch.empty(3 * n, dtype=_TORCH[coord], device=eng.device)
        a = pr.args
        a.rhat_out = pr.rhat.data_ptr()
        a.onthefly = 1
        a.vr_f64 = int(np.result_type(plan.vel, coord) == F64)
        return pr

    def compare(self, snaps, slices, centres, carried=None, bulks=None):
        """Device half of a call: frame the previous snapshot (unless ``carried``),
        frame + join the current one.  Returns the device outputs (``OTFDevice``) and
        leaves this call's current frame state in ``self.carry``.

        snaps / slices / centres: [current, previous].  ``bulks``: [current, previous]
        bulk-velocity rows to use instead of computing them from the blocks (a shard's
        rows do not hold whole blocks).  ``carried``: the (state, bulk velocities) a
        previous call left for its current snapshot (``self.carry``), when that
        snapshot is this call's previous one with the same regions; its frame is then
        not recomputed (``snaps[1]`` unused)."""
        eng = self.eng
        cur, prv = snaps
        if carried is None:
            if np_dtype(cur['coordinates']) != np_dtype(prv['coordinates']):
                raise NotImplementedError('coordinate dtype differs between the two snapshots')
            # previous snapshot: frame only
            pp = self._prepare(prv, slices[1], centres[1], False,
                               bulk=None if bulks is None else bulks[1])
            eng.launch(pp, None)
            prev = SnapshotState(ids=pp.snap['ids'], rhat=pp.rhat, meta=pp.meta,
                                 starts=pp.starts, counts=pp.counts,
                                 exists=np.arange(len(slices[1])), plan=pp.plan)
            bulk_p = None
        else:
            prev, bulk_p = carried
            if np_dtype(cur['coordinates']) != np.dtype(prev.plan.coord):
                raise NotImplementedError('coordinate dtype differs between the two snapshots')
        n_prev = prev.ids.numel()
        entries = None
        for _ in range(10):
            pc = self._prepare(cur, slices[0], centres[0], True, prev=prev, entries=entries,
                               bulk=None if bulks is None else bulks[0])
            coord = _TORCH[np.dtype(pc.plan.coord)]
            angle_out = torch.empty(max(n_prev, 1), dtype=coord, device=eng.device)
            matched_prev = torch.zeros(max(n_prev, 1), dtype=torch.uint8, device=eng.device)
            matched_cur = torch.zeros(max(pc.n, 1), dtype=torch.uint8, device=eng.device)
            a = pc.args
            a.angle_out, a.matched_prev, a.matched_cur = (angle_out.data_ptr(),
                                                          matched_prev.data_ptr(),
                                                          matched_cur.data_ptr())
            ws = eng.workspace(pc)
            ws.status.zero_()
            res = eng.launch(pc, ws, prev=prev)
            st = int(ws.status[0].item())
            if not st:
                break
            if st & N.STATUS_PLAN:
                raise RuntimeError('oa_step: an item exceeds the kernel limits (planner bug)')
            # stash full: smaller items, then every halo on the 64-bit global-table path
            entries = 0 if pc.entries <= 256 else max(256, pc.entries // 2)
        else:
            raise RuntimeError('LDS hash tables kept overflowing')
        nh = len(slices[0])
        bulk_c = pc.halos.cpu().numpy().view(N.HALO_DTYPE)['bulk'].astype(pc.plan.bulk)
        if bulk_p is None:
            bulk_p = pp.halos.cpu().numpy().view(N.HALO_DTYPE)['bulk'].astype(pp.plan.bulk)
        # this snapshot's frame state (r̂ in the coordinate dtype, sign bits) is exactly
        # what the next call needs for its previous snapshot
        self.carry = (SnapshotState(ids=pc.snap['ids'], rhat=pc.rhat, meta=pc.meta,
                                    starts=pc.starts, counts=pc.counts, exists=np.arange(nh),
                                    plan=pc.plan), bulk_c)
        return OTFDevice(pc=pc, prev=prev, res=res, angle_out=angle_out[:n_prev],
                         matched_prev=matched_prev[:n_prev].bool(),
                         matched_cur=matched_cur[:pc.n] != 0, bulk_c=bulk_c, bulk_p=bulk_p)

    def run(self, snaps, slices, centres, carried=None, bulks=None):
        """One call on this GPU (``compare``), outputs brought to the host in the
        reference's layout (track_orbits_onthefly.py:123-205)."""
        eng = self.eng
        d = self.compare(snaps, slices, centres, carried=carried, bulks=bulks)
        pc, prev, res = d.pc, d.prev, d.res
        nh = len(slices[0])
        ids_dtype = np_dtype(snaps[0]['ids'])
        # apsis records per halo, previous-block order (:154-166)
        offsets, apsis_ids, _ = eng.fetch(res, ids_dtype)
        # angle changes of every matched particle, previous-block order (:173-174):
        # N values, brought back through pinned memory
        mp = d.matched_prev
        sel = d.angle_out[mp]
        angles_h = torch.empty(sel.shape, dtype=sel.dtype, pin_memory=True)
        angles_h.copy_(sel)
        angles = angles_h.numpy()
        p_has = pc.halos.cpu().numpy().view(N.HALO_DTYPE)['prev_cnt'] > 0

        def halo_of(pos, starts):
            # block of each selected position (blocks tile [0, n) in halo order)
            st = _h2d(np.asarray(starts, dtype=np.int64), eng.device)
            return torch.searchsorted(st, pos, right=True) - 1
        # departed: setdiff1d(previous, current) per halo (:145), i.e. the sorted unique
        # IDs of the unmatched previous rows (which already sit in halo order)
        # rows before the first block are in no block (halo -1): the reference's slices
        # start at region_offsets[0] and never see them (as the sharded stripes)
        dsel = torch.nonzero(~mp).squeeze(1)
        dh = halo_of(dsel, prev.starts)
        dsel, dh = dsel[dh >= 0], dh[dh >= 0]
        departed, d_off = _sorted_unique_per_halo(
            eng.lib, eng.device, prev.ids[dsel],
            torch.bincount(dh, minlength=nh).cpu().numpy(), ids_dtype)
        # entered: setdiff1d(current, previous) per halo (:168); all of a halo's
        # particles, in loader order, when its progenitor block is empty (:178)
        esel = torch.nonzero(d.matched_cur == 0).squeeze(1)
        eh = halo_of(esel, pc.starts)
        esel, eh = esel[eh >= 0], eh[eh >= 0]
        e_ids = pc.snap['ids'][esel]
        sorted_h = _h2d(p_has, eng.device)[eh]
        srt, s_off = _sorted_unique_per_halo(
            eng.lib, eng.device, e_ids[sorted_h],
            torch.bincount(eh[sorted_h], minlength=nh).cpu().numpy(), ids_dtype)
        raw_t = e_ids[~sorted_h]
        raw = raw_t.cpu().numpy().view(ids_dtype) if raw_t.numel() else np.zeros(0, ids_dtype)
        r_off = np.concatenate([[0], np.cumsum(torch.bincount(eh[~sorted_h], minlength=nh)
                                                .cpu().numpy())]).astype(np.int64)
        entered, e_off = _interleave_halos(p_has, srt, s_off, raw, r_off)
        adt = _angles_dtype(pc.plan.coord, ids_dtype, p_has)
        return {'apsis_offsets': offsets, 'apsis_ids': apsis_ids,
                'angles': angles.astype(adt, copy=False),
                'entered_offsets': e_off, 'entered_ids': entered,
                'departed_offsets': d_off, 'departed_ids': departed,
                'bulk_velocities': [d.bulk_c, d.bulk_p]}


@dataclass
class OTFDevice:
    """Device outputs of one on-the-fly compare (OnTheFly.compare)."""
    pc: object                      # the current snapshot's PreparedStep
    prev: SnapshotState             # the previous snapshot's frame state
    res: object                     # StepResult: apsis CSR (+ previous-state rows)
    angle_out: torch.Tensor         # arccos(r̂_prev . r̂) per previous row (matched rows)
    matched_prev: torch.Tensor      # bool per previous row
    matched_cur: torch.Tensor       # bool per current row
    bulk_c: np.ndarray
    bulk_p: np.ndarray


def _angles_dtype(coord, ids_dtype, p_has):
    """Concatenation dtype of the reference's per-halo angle lists (:173-174, :183): a
    halo with a progenitor block contributes arccos in the coordinate dtype, one
    without an empty array of the IDs' dtype."""
    parts = [np.zeros(0, np.dtype(coord))] * int(np.sum(p_has)) + \
            [np.zeros(0, ids_dtype)] * int(np.sum(~np.asarray(p_has, bool)))
    return np.concatenate(parts).dtype if parts else np.dtype(np.float64)


# ------------------------------------------------------------------ multi-GPU
def id_order_key(ids64, ids_dtype):
    """int64 keys whose signed order is the IDs' numeric order (``ids64``: the IDs as
    int64 -- sign-extended 32-bit values, 64-bit bit patterns)."""
    dt = np.dtype(ids_dtype)
    if dt.kind == 'u' and dt.itemsize == 8:
        return ids64 ^ torch.tensor(np.iinfo(np.int64).min, dtype=torch.int64,
                                    device=ids64.device)
    if dt.kind == 'u':
        return ids64 & 0xFFFFFFFF
    return ids64


def ids_to_host(ids64, ids_dtype):
    """Device int64 IDs -> host array of the loader's dtype."""
    dt = np.dtype(ids_dtype)
    h = ids64.cpu().numpy()
    if dt.itemsize == 8:
        return h.view(dt)
    return h.astype(dt)


def _pinned_host(t):
    """Device tensor -> host numpy through a page-locked block (one DMA)."""
    if t.device.type == 'cpu':
        return t.numpy()
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h.numpy()


def _sort_pairs(h, key):
    """Order of the rows by (h, key): a stable sort by key, then a stable one by h."""
    o = torch.sort(key, stable=True)[1]
    o2 = torch.sort(h[o], stable=True)[1]
    return o[o2]


def _by_unique_key(v, g, n):
    """``v`` ordered by its distinct keys ``g`` in [0, n): as they are when every rank's
    rows arrive in order (world 1, or one contributing rank), else by a counting
    placement (one n-bit mark array and its prefix sum), not a comparison sort of
    the ~N matched rows."""
    if g.numel() < 2 or bool((g[1:] > g[:-1]).all()):
        return v
    # the bound covers every key (an index past the mark array would fault the device)
    n = max(int(n or 0), int(g.max()) + 1)
    mark = torch.zeros(int(n), dtype=torch.int32, device=g.device)
    mark[g] = 1
    dest = torch.cumsum(mark, 0, dtype=torch.int32)[g].long() - 1
    out = torch.empty_like(v)
    out[dest] = v
    return out


def _to_loader_width(ids64, ids_dtype):
    """int64 ID values -> a device tensor of the loader's width (bit patterns kept)."""
    return ids64 if np.dtype(ids_dtype).itemsize == 8 else ids64.to(torch.int32)


def _ids_to_host_pinned(ids64, ids_dtype):
    """ids_to_host through a page-locked block (one DMA, no pageable staging)."""
    dt = np.dtype(ids_dtype)
    h = _pinned_host(ids64)
    return h.view(dt) if dt.itemsize == 8 else h.astype(dt)


def merge_onthefly(parts, nh, prev_starts, p_has, ids_dtype, n_prev=None, ordered=False,
                   lib=None):
    """Merge the ranks' on-the-fly records of one snapshot pair on the root rank
    (ShardedOnTheFly), on whatever device the tensors are on.

    ``parts``: the rank-ordered concatenation of every rank's rows:
      * ``apsis`` (n, 2) int64: global previous row, ID;
      * ``angle_g`` (n,) int64 global previous row, ``angle_v`` (n,) the angle change;
      * ``departed`` (n, 2) int64: halo, ID;
      * ``entered`` (n, 3) int64: halo, ID, global current row.
    A halo's previous and current blocks tile their snapshots in halo order, so the
    global previous row orders apsis records and angle changes exactly as the reference
    emits them (previous-block order, halos in order, :154-174).  Departed and entered
    IDs are per-halo sorted unique (setdiff1d, :145, :168), except the entered IDs of a
    halo without a progenitor block, which keep loader order (:178), i.e. global
    current-row order.  ``n_prev``: the previous snapshot's row count (bounds the
    global previous rows).  ``ordered``: one rank contributed every row, in order
    (world 1): apsis records and angle changes need no sort (``angle_g`` may then be
    None), and departed / entered rows already come in halo order.  ``lib`` (device
    tensors): the per-halo sorted-unique IDs come from the collation kernels (per-halo
    LDS sort, as the single-GPU ``OnTheFly``) after at most one stable sort by halo, and
    the IDs come back through pinned memory; without it, two stable torch sorts per
    list (any device).  Returns host arrays (IDs in ``ids_dtype``)."""
    ap = parts['apsis']
    dev = ap.device
    out = {}
    if not ordered:
        ap = ap[torch.argsort(ap[:, 0])]
    st = _h2d(np.asarray(prev_starts, dtype=np.int64), dev)
    halo = torch.searchsorted(st, ap[:, 0].contiguous(), right=True) - 1 if len(st) else ap[:, 0]
    cnt = torch.bincount(halo, minlength=nh)[:nh] if ap.shape[0] else \
        torch.zeros(nh, dtype=torch.int64, device=dev)
    out['apsis_offsets'] = np.concatenate([[0], np.cumsum(cnt.cpu().numpy())]).astype(np.int64)
    kern = lib is not None and dev.type == 'cuda'
    out['apsis_ids'] = _ids_to_host_pinned(ap[:, 1].contiguous(), ids_dtype) if kern else \
        ids_to_host(ap[:, 1], ids_dtype)
    out['angles'] = _pinned_host(parts['angle_v'] if ordered or parts['angle_g'] is None else
                                 _by_unique_key(parts['angle_v'], parts['angle_g'], n_prev))

    def grouped(h, ids, second, uniq):
        o = _sort_pairs(h, second)
        h, ids, uniq = h[o], ids[o], uniq[o]
        if h.numel() > 1:                     # setdiff1d is unique: drop repeats in a halo
            dup = torch.zeros_like(h, dtype=torch.bool)
            dup[1:] = (h[1:] == h[:-1]) & (ids[1:] == ids[:-1]) & uniq[1:]
            h, ids = h[~dup], ids[~dup]
        c = torch.bincount(h, minlength=nh)[:nh] if h.numel() else \
            torch.zeros(nh, dtype=torch.int64, device=dev)
        return ids_to_host(ids, ids_dtype), \
            np.concatenate([[0], np.cumsum(c.cpu().numpy())]).astype(np.int64)

    if kern:
        _merge_lists_kernels(out, parts, nh, p_has, ids_dtype, ordered, lib, dev)
        return out
    dp = parts['departed']
    out['departed_ids'], out['departed_offsets'] = grouped(
        dp[:, 0], dp[:, 1], id_order_key(dp[:, 1], ids_dtype),
        torch.ones(dp.shape[0], dtype=torch.bool, device=dev))
    en = parts['entered']
    ph = _h2d(np.asarray(p_has, dtype=bool), dev)
    srt = ph[en[:, 0]] if en.shape[0] else torch.zeros(0, dtype=torch.bool, device=dev)
    second = torch.where(srt, id_order_key(en[:, 1], ids_dtype), en[:, 2])
    out['entered_ids'], out['entered_offsets'] = grouped(en[:, 0], en[:, 1], second, srt)
    return out


def _merge_lists_kernels(out, parts, nh, p_has, ids_dtype, ordered, lib, dev):
    """merge_onthefly's departed / entered lists with the collation kernels: rows put in
    halo order by one stable sort (none when ``ordered``), then each halo's sorted
    unique IDs (setdiff1d, :145, :168) by ``_sorted_unique_per_halo``; the entered IDs
    of a halo without a progenitor block keep global current-row order (:178)."""
    def by_halo(h, *cols):
        keep = h >= 0                          # rows before the first block: no halo
        h = h[keep]
        cols = [c[keep] for c in cols]
        if not ordered and h.numel() > 1:
            o = torch.sort(h, stable=True)[1]
            h = h[o]
            cols = [c[o] for c in cols]
        return h, cols

    def counts(h):
        return torch.bincount(h, minlength=nh)[:nh].cpu().numpy() if h.numel() else \
            np.zeros(nh, np.int64)
    dp = parts['departed']
    h, (ids,) = by_halo(dp[:, 0], dp[:, 1])
    out['departed_ids'], out['departed_offsets'] = _sorted_unique_per_halo(
        lib, dev, _to_loader_width(ids, ids_dtype), counts(h), ids_dtype)
    en = parts['entered']
    ph = _h2d(np.asarray(p_has, dtype=bool), dev)
    h, (ids, row) = by_halo(en[:, 0], en[:, 1], en[:, 2])
    srt = ph[h] if h.numel() else torch.zeros(0, dtype=torch.bool, device=dev)
    s_ids, s_off = _sorted_unique_per_halo(lib, dev, _to_loader_width(ids[srt], ids_dtype),
                                           counts(h[srt]), ids_dtype)
    hr, ir, rr = h[~srt], ids[~srt], row[~srt]
    if not ordered and hr.numel() > 1:         # loader order: the global current row
        o = _sort_pairs(hr, rr)
        hr, ir = hr[o], ir[o]
    raw = _ids_to_host_pinned(ir.contiguous(), ids_dtype) if ir.numel() else \
        np.zeros(0, np.dtype(ids_dtype))
    r_off = np.concatenate([[0], np.cumsum(counts(hr))]).astype(np.int64)
    out['entered_ids'], out['entered_offsets'] = _interleave_halos(
        np.asarray(p_has, dtype=bool), s_ids, s_off, raw, r_off)


class ShardedOnTheFly:
    """The on-the-fly driver over ID-range shards (BASELINE configs[4]):
    one process per GPU, ``torch.distributed`` (RCCL, or gloo in the tests).

    Each snapshot reaches the ranks as the reference's loader returns it (the whole
    snapshot, host or device arrays) and is sharded as ``ShardedEngine`` shards it
    (``sharding.stripe_shard``): rank r moves only its block-aligned stripe to its GPU,
    computes the bulk velocities of the stripe's blocks there (whole blocks, the
    reference's sums; the rows are all-gathered), and routes the stripe's rows to their
    owners with one all-to-all.  A particle's rows in the two snapshots are then on
    the same rank, so the join has no exchange.  A caller that already holds each
    rank's stripe on the device (``stripes``: a double-buffered reader, as
    ``tools/bench_onthefly.py --sharded``) skips the upload.

    Outputs, into exactly the single-process file on rank 0, the only writer: apsis IDs
    and angle changes (by global previous row) are stored by every rank straight into
    shared page-locked host buffers (``_stage_outputs``, ``host_share``; world > 1);
    departed (halo, ID) and entered (halo, ID, global current row) rows are gathered to
    rank 0 and merged there with device sorts (``merge_onthefly``).  Ranks other than 0
    return the per-halo tables with empty record arrays.

    ``track_orbits(..., engine=ShardedOnTheFly(OrbitEngine(mode=...)))``."""

    ROOT = 0

    def __init__(self, engine, group=None, owner=None):
        from .sharding import IdRangeOwner
        self.eng = engine
        self.mode = engine.mode
        self.group = group
        self.owner = owner if owner is not None else IdRangeOwner()
        # world > 1: apsis IDs and angle changes go into the shared host buffer
        # (host_share.SharedRecordStage); ORBIT_OTF_STAGE=0 gathers them to rank 0
        self.use_stage = os.environ.get('ORBIT_OTF_STAGE', '1') != '0'
        self._stage = None
        engine.emit_positions = True
        self.otf = OnTheFly(engine)
        self.carry = None
        self.h2d_bytes = 0
        # per-phase times of run() (ms lists by phase) when set to a dict: with
        # timing_sync each phase boundary synchronises the device (wall time per phase);
        # without, the host time between boundaries ('host:' phases) and the stream time
        # between events recorded at them ('gpu:' phases) are kept, unperturbed
        self.timings = None
        self.timing_sync = True
        self._t0 = 0.0
        self._evs = []

    def _mark(self, name):
        if self.timings is None:
            return
        if self.timing_sync:
            torch.cuda.synchronize(self.eng.device)
        t = time.perf_counter()
        self.timings.setdefault(('' if self.timing_sync else 'host:') + name, []).append(
            (t - self._t0) * 1e3)
        self._t0 = t
        if not self.timing_sync:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._evs.append((name, ev))

    def _close_marks(self):
        """Stream times between this call's events (the call's last D2H has completed)."""
        if self.timings is None or self.timing_sync or not self._evs:
            return
        self._evs[-1][1].synchronize()
        for (_, a), (name, b) in zip(self._evs[:-1], self._evs[1:]):
            self.timings.setdefault('gpu:' + name, []).append(a.elapsed_time(b))
        self._evs = []

    @property
    def rank(self):
        import torch.distributed as dist
        return dist.get_rank(self.group)

    @property
    def world(self):
        import torch.distributed as dist
        return dist.get_world_size(self.group)

    def agree(self, flag):
        """True on every rank iff ``flag`` is true on every rank (a carry is used only
        when all ranks hold one, so their collectives stay in step)."""
        from .sharding import all_true
        return all_true(flag, self.group)

    def shard(self, snap, sl):
        """This rank's shard of one snapshot (``sharding.stripe_shard``) and its local
        slices (absent halos (-1, -1)).  A snapshot with ``sharding.STRIPE`` holds only
        this rank's stripe, and then its ``n_rows`` the global row count."""
        from .sharding import stripe_shard, STRIPE
        sl = np.asarray(sl, dtype=np.int64).reshape(-1, 2)
        ids = snap['ids']
        n = int(snap['n_rows']) if STRIPE in snap else \
            (int(ids.numel()) if isinstance(ids, torch.Tensor) else len(ids))
        eng = self.eng
        # bulk velocities: of the stripe's whole blocks before the exchange splits them,
        # all-gathered (world > 1); at world 1 the shard is the snapshot and the step
        # computes them itself, as OnTheFly does (no host round trip)
        sh = stripe_shard(snap, _block_starts(sl, n), self.owner, self.group, eng.device,
                          bulk_fn=eng.block_bulk if self.world > 1 else None, n=n)
        st = np.concatenate([[0], np.cumsum(sh.counts)[:-1]]).astype(np.int64)
        lsl = np.where(sl[:, :1] >= 0, np.stack([st, st + sh.counts], axis=1), -1)
        self.h2d_bytes += sh.h2d_bytes
        return sh, lsl

    def run(self, snaps, slices, centres, carried=None):
        """``carried``: this object's ``carry`` from the previous call, whose current
        snapshot is this call's previous one (``snaps[1]`` is then None): the rank's
        shard of it, its device frame state and its bulk velocities are reused."""
        from .sharding import gather_rows
        eng = self.eng
        if self.timings is not None:
            if self.timing_sync:
                torch.cuda.synchronize(eng.device)
            self._t0 = time.perf_counter()
            self._evs = []
            self._mark('start')
        if carried is None:
            self.owner.reset()                # a fresh pair: fit the ID ranges on it
        shards, lslices, sels, bulks = [], [], [], []
        otf_carry = None
        if carried is not None:
            otf_carry, sel_prev = carried
        for snap, sl in zip(snaps, slices):
            if snap is None:                  # the carried previous snapshot
                shards.append(None)
                lslices.append(None)
                sels.append(sel_prev)
                bulks.append(None)
                continue
            sh, lsl = self.shard(snap, sl)
            shards.append(sh.snap)
            lslices.append(lsl)
            sels.append(sh.sel)
            bulks.append(sh.bulk)
        self._mark('shard')
        d = self.otf.compare(shards, lslices, centres, carried=otf_carry, bulks=bulks)
        self._mark('compare')
        self.carry = (self.otf.carry, sels[0])
        pc, prev, res = d.pc, d.prev, d.res
        nh = len(slices[0])
        ids_dtype = np.dtype(pc.plan.ids) if snaps[0] is None else np_dtype(snaps[0]['ids'])
        sel_c, sel_p = sels[0].to(eng.device), sels[1].to(eng.device)
        # this rank's records, each with its global row (device)
        total = int(res.offsets[-1]) if res.offsets is not None and res.offsets.numel() else 0
        a_ids = _i64(res.apsis_ids[:total])
        apsis = torch.stack([sel_p[res.apsis_pos[:total].long()], a_ids], dim=1)
        # angle changes: at world 1 the matched rows are already in global previous-row
        # order (the shard is the snapshot), so they need no row key
        angle_v = d.angle_out[d.matched_prev]
        angle_g = sel_p[torch.nonzero(d.matched_prev).squeeze(1)] if self.world > 1 else \
            torch.zeros(0, dtype=torch.int64, device=eng.device)
        drow = torch.nonzero(~d.matched_prev).squeeze(1)
        departed = torch.stack([_halo_of(drow, prev.starts, eng.device),
                                _i64(prev.ids[drow])], dim=1)
        erow = torch.nonzero(~d.matched_cur).squeeze(1)
        entered = torch.stack([_halo_of(erow, pc.starts, eng.device),
                               _i64(pc.snap['ids'][erow]), sel_c[erow]], dim=1)
        self._mark('records')
        sl1 = np.asarray(slices[1], dtype=np.int64).reshape(-1, 2)
        p_has = (sl1[:, 1] - sl1[:, 0]) > 0            # the reference's np.diff(sl_prev) > 0
        adt = _angles_dtype(pc.plan.coord, ids_dtype, p_has)
        n_prev = max(int(np.max(sl1[:, 1])) if len(sl1) else 0, 0)
        staged = None
        if self.world > 1 and self.use_stage:
            staged = self._stage_outputs(apsis, a_ids, angle_g, angle_v, nh,
                                         _block_starts(sl1, n_prev), n_prev, ids_dtype)
            apsis = apsis[:0]
            angle_g, angle_v = angle_g[:0], angle_v[:0]
        apsis, = gather_rows(self.group, self.ROOT, apsis)
        if self.world > 1:
            angle_g, angle_v = gather_rows(self.group, self.ROOT, angle_g, angle_v)
        departed, = gather_rows(self.group, self.ROOT, departed)
        entered, = gather_rows(self.group, self.ROOT, entered)
        self._mark('gather')
        if self.rank == self.ROOT:
            merged = merge_onthefly(dict(apsis=apsis, angle_g=angle_g if self.world > 1 else None,
                                         angle_v=angle_v, departed=departed, entered=entered),
                                    nh, _block_starts(sl1, n_prev), p_has, ids_dtype,
                                    n_prev=n_prev, ordered=self.world == 1,
                                    lib=eng.lib)
            if staged is not None:
                merged['apsis_offsets'], merged['apsis_ids'], merged['angles'] = staged
            merged['angles'] = merged['angles'].astype(adt, copy=False)
        else:
            z = np.zeros(nh + 1, np.int64)
            merged = {'apsis_offsets': z, 'apsis_ids': np.zeros(0, ids_dtype),
                      'angles': np.zeros(0, adt), 'entered_offsets': z,
                      'entered_ids': np.zeros(0, ids_dtype), 'departed_offsets': z,
                      'departed_ids': np.zeros(0, ids_dtype)}
        merged['bulk_velocities'] = [d.bulk_c, d.bulk_p]
        self._mark('merge+d2h')
        self._close_marks()
        return merged

    def _stage_outputs(self, apsis, a_ids, angle_g, angle_v, nh, prev_starts, n_prev, ids_dtype):
        """World > 1: this rank's apsis IDs and angle changes stored straight into one
        shared page-locked host buffer each (``host_share.SharedRecordStage``), at their
        positions among every rank's, ordered by global previous row as the reference emits
        them (previous-block order, halos in order, :154-174): the per-halo apsis counts
        are all-gathered, the positions come from one bitmap all-reduce per list.  Each rank
        moves its own outputs over its own link; nothing crosses to rank 0's GPU.  Returns
        (apsis offsets, apsis IDs, angle changes) on rank 0 (views of the buffers), None
        elsewhere."""
        import torch.distributed as dist
        from .host_share import SharedRecordStage
        from .sharding import _comm_device
        if self._stage is None:
            self._stage = SharedRecordStage(self.group, self.rank, self.world, self.ROOT)
        cdev = _comm_device()
        dev = apsis.device
        a_rows = apsis[:, 0]
        # a bound on every rank's global previous rows (rows after the last block included)
        hi = max(n_prev, int(a_rows.max()) + 1 if a_rows.numel() else 0,
                 int(angle_g.max()) + 1 if angle_g.numel() else 0)
        m = torch.tensor([hi], dtype=torch.int64).to(cdev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
        n_rows = int(m.item())
        st = _h2d(np.asarray(prev_starts, dtype=np.int64), dev)
        n = int(a_rows.numel())
        if n and len(st):
            halo = torch.searchsorted(st, a_rows.contiguous(), right=True) - 1
            cnt = torch.bincount(halo.clamp_(min=0), minlength=nh)[:nh]
        else:
            cnt = torch.zeros(nh, dtype=torch.int64, device=dev)
        lib = self.eng.lib
        f = self._stage.fetch(lib, None, None, None, _to_loader_width(a_ids, ids_dtype), None, n,
                              cnt, nh, ids_dtype, rows=a_rows, n_rows=n_rows, comm_dev=cdev)
        off, ids, _ = f.wait()
        ang = self._stage.place_ranked(lib, angle_v.contiguous(), angle_g, n_rows, cdev)
        if self.rank != self.ROOT:
            return None
        return off, ids, ang


def _i64(t):
    return t if t.dtype == torch.int64 else t.to(torch.int64)


def _halo_of(rows, starts, device):
    """Block of each row (blocks tile their snapshot in halo order)."""
    st = _h2d(np.asarray(starts, dtype=np.int64), device)
    if not len(st):
        return rows
    return torch.searchsorted(st, rows, right=True) - 1


# Frame state of the last call's current snapshot, keyed by the loader callable
# (SURVEY §8(f) f1): a stream of calls s, s+1, ... whose progenitor row and regions at
# s-1 equal the previous call's current ones loads and frames each snapshot once
# instead of twice.  ORBIT_OTF_CARRY=0 disables it; clear_carry() drops it.
_CARRY = {}


def _carry_enabled():
    return os.environ.get('ORBIT_OTF_CARRY', '1') != '0'


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b, equal_nan=True)


def clear_carry():
    """Release the device state kept between on-the-fly calls."""
    _CARRY.clear()


def track_orbits(snapshot_number, progenitor_links, regions, load_snapshot_data,
                 savefile, mode='pericentric', verbose=True, engine=None):
    """track_orbits_onthefly.py:8-58 (signature, callbacks and errors of the reference;
    ``engine`` optionally supplies a configured ``OrbitEngine``, or a
    ``ShardedOnTheFly`` for one rank of a multi-GPU run)."""
    if (mode != 'pericentric') and (mode != 'apocentric'):
        raise ValueError(
            "Orbit detection mode not recognized. Please specify either "
            "'pericentric' or 'apocentric'.")
    progenitor_links = np.asarray(progenitor_links)
    snaps, slices, positions, radii = [], [], [], []
    box_size = None
    key = load_snapshot_data              # bound methods compare by (instance, function)
    try:
        entry = _CARRY.get(key) if _carry_enabled() else None
    except TypeError:                     # an unhashable callable: no carry
        key, entry = None, None
    carried = None
    sharded = isinstance(engine, ShardedOnTheFly)
    if sharded:
        otf = engine                      # a carry is used only when every rank has one
    else:
        otf = OnTheFly(engine, mode)
    if otf.mode != mode:
        raise ValueError('engine mode %r != mode %r' % (otf.mode, mode))
    # device tensors of a carry belong to the engine (device, LDS configuration) that
    # made them: a call with another engine, or on another device, starts afresh
    if entry is not None and (entry['engine'] is not engine or entry['device'] != otf.eng.device):
        entry = None
    for s, halo_ids_ in zip([snapshot_number, snapshot_number - 1], progenitor_links):
        halo_exists = np.argwhere(halo_ids_ != -1).flatten()
        halo_ids = halo_ids_[halo_exists]
        region_pos, region_rad = regions(s, halo_ids)
        positions.append(repack(region_pos, len(halo_ids_), halo_exists))
        radii.append(repack(region_rad, len(halo_ids_), halo_exists))
        use = s == snapshot_number - 1 and entry is not None and entry['s'] == s and \
            np.array_equal(entry['row'], halo_ids_) and \
            _same(entry['pos'], region_pos) and _same(entry['rad'], region_rad)
        if sharded and s == snapshot_number - 1:
            use = otf.agree(use)
        if use:
            # the previous call's current snapshot, same regions: its device frame state
            # is reused and the snapshot is not loaded again
            snaps.append(None)
            slices.append(entry['slices'])
            box_size = entry['box_size']
            carried = entry['carry']
            continue
        snapshot = load_snapshot_data(s, region_pos, region_rad)
        snaps.append(snapshot)
        offsets = list(snapshot['region_offsets']) + [len(snapshot['ids'])]
        sl = np.array(list(zip(offsets[:-1], offsets[1:])))
        slices.append(repack(sl, len(halo_ids_), halo_exists))
        box_size = snapshot['box_size'] if 'box_size' in snapshot else None
        if s == snapshot_number:
            cur_meta = dict(s=s, row=halo_ids_.copy(), pos=np.array(region_pos, copy=True),
                            rad=np.array(region_rad, copy=True), slices=slices[-1],
                            box_size=box_size)
    if verbose:
        print('Identifying {}ers...'.format(mode[:8]))
        t0 = time.time()
    if key is not None:
        _CARRY.pop(key, None)             # a failing call leaves nothing stale behind
    out = otf.run(snaps, slices, positions, carried=carried)
    if key is not None and _carry_enabled():
        _CARRY.clear()                    # one carried snapshot at a time (device memory)
        _CARRY[key] = dict(cur_meta, carry=otf.carry,
                           engine=engine, device=otf.eng.device)
    if verbose:
        print('Identified {}ers in {} s\n'.format(mode[:8], time.time() - t0))
    tag = mode[:8] + 'er'
    data = {tag + '_offsets': out['apsis_offsets'], tag + '_IDs': out['apsis_ids'],
            'angles': out['angles'],
            'entered_offsets': out['entered_offsets'], 'entered_IDs': out['entered_ids'],
            'departed_offsets': out['departed_offsets'], 'departed_IDs': out['departed_ids'],
            'progenitor_links': progenitor_links, 'region_radii': np.array(radii),
            'region_positions': np.array(positions),
            'bulk_velocities': np.array(out['bulk_velocities'])}
    attrs = {} if box_size is None else {'box_size': box_size}
    if not sharded or otf.rank == 0:                  # one file per snapshot
        save_to_file(savefile, snapshot_number, data, attrs, verbose)
    return data


def save_to_file(savefile, snapshot_number, data, attrs, verbose):
    """track_orbits_onthefly.py:208-252: one file per snapshot."""
    if verbose:
        print('Saving to file...')
        t0 = time.time()
    if isinstance(savefile, str):
        import h5py
        with h5py.File(savefile.format('%0.3d' % snapshot_number), 'w') as hf:
            for k, v in data.items():
                hf.create_dataset(k, data=v)
            for k, v in attrs.items():
                hf.attrs[k] = v
    else:
        savefile.write_file(snapshot_number, data, attrs)
    if verbose:
        print('Saved to file in {} s\n'.format(time.time() - t0))
