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

import numpy as np
import torch

from . import _native as N
from .engine import OrbitEngine, SnapshotState, to_device, F64, np_dtype

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
    starts = np.empty(len(slices), dtype=np.int64)
    pos = 0
    for j, (a, b) in enumerate(np.asarray(slices, dtype=np.int64)):
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
        if isinstance(snap['masses'], np.ndarray):
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

    def run(self, snaps, slices, centres, carried=None, bulks=None, merge_parts=False):
        """snaps / slices / centres: [current, previous].  Returns host outputs.

        ``bulks``: [current, previous] bulk-velocity rows to use instead of computing
        them from the blocks.  ``merge_parts``: also return, under ``'parts'``, what a
        sharded run needs to merge ranks (the previous-state rows of the apsis records
        and of the angle changes, the per-halo entered lists before interleaving and
        the current rows of the loader-order ones).

        ``carried``: the (state, bulk velocities) a previous call left for its current
        snapshot (``self.carry``), when that snapshot is this call's previous one with
        the same regions; its frame is then not recomputed (``snaps[1]`` unused)."""
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
        ids_dtype = np_dtype(cur['ids'])
        unsigned = ids_dtype.kind == 'u'
        # apsis records per halo, previous-block order (:154-166)
        offsets, apsis_ids, _ = eng.fetch(res, ids_dtype)
        # angle changes of every matched particle, previous-block order (:173-174):
        # N values, brought back through pinned memory
        mp = matched_prev[:n_prev].bool()
        sel = angle_out[:n_prev][mp]
        angles_h = torch.empty(sel.shape, dtype=sel.dtype, pin_memory=True)
        angles_h.copy_(sel)
        angles = angles_h.numpy()
        p_has = pc.halos.cpu().numpy().view(N.HALO_DTYPE)['prev_cnt'] > 0

        def host_ids(t):
            return t.cpu().numpy().view(ids_dtype) if t.numel() else np.zeros(0, ids_dtype)

        def halo_of(pos, starts):
            # block of each selected position (blocks tile [0, n) in halo order)
            st = torch.from_numpy(np.asarray(starts, dtype=np.int64)).to(eng.device)
            return torch.searchsorted(st, pos, right=True) - 1
        # departed: setdiff1d(previous, current) per halo (:145), i.e. the sorted unique
        # IDs of the unmatched previous rows (which already sit in halo order)
        dsel = torch.nonzero(~mp).squeeze(1)
        dh = halo_of(dsel, prev.starts)
        departed, d_off = _sorted_unique_per_halo(
            eng.lib, eng.device, prev.ids[dsel],
            torch.bincount(dh, minlength=nh).cpu().numpy(), ids_dtype)
        # entered: setdiff1d(current, previous) per halo (:168); all of a halo's
        # particles, in loader order, when its progenitor block is empty (:178)
        esel = torch.nonzero(matched_cur[:pc.n] == 0).squeeze(1)
        e_ids = pc.snap['ids'][esel]
        eh = halo_of(esel, pc.starts)
        sorted_h = torch.from_numpy(p_has).to(eng.device)[eh]
        srt, s_off = _sorted_unique_per_halo(
            eng.lib, eng.device, e_ids[sorted_h],
            torch.bincount(eh[sorted_h], minlength=nh).cpu().numpy(), ids_dtype)
        raw = host_ids(e_ids[~sorted_h])
        r_off = np.concatenate([[0], np.cumsum(torch.bincount(eh[~sorted_h], minlength=nh)
                                                .cpu().numpy())]).astype(np.int64)
        entered, e_off = _interleave_halos(p_has, srt, s_off, raw, r_off)
        # concatenation dtype of the reference's per-halo lists (:183, :203): an empty
        # halo contributes np.array([], dtype=ids.dtype)
        parts = [np.zeros(0, np.dtype(pc.plan.coord))] * int(p_has.sum()) + \
                [np.zeros(0, ids_dtype)] * int((~p_has).sum())
        adt = np.concatenate(parts).dtype if parts else np.dtype(np.float64)

        bulk_c = pc.halos.cpu().numpy().view(N.HALO_DTYPE)['bulk'].astype(pc.plan.bulk)
        if bulk_p is None:
            bulk_p = pp.halos.cpu().numpy().view(N.HALO_DTYPE)['bulk'].astype(pp.plan.bulk)
        # this snapshot's frame state (r̂ in the coordinate dtype, sign bits) is exactly
        # what the next call needs for its previous snapshot
        self.carry = (SnapshotState(ids=pc.snap['ids'], rhat=pc.rhat, meta=pc.meta,
                                    starts=pc.starts, counts=pc.counts, exists=np.arange(nh),
                                    plan=pc.plan), bulk_c)
        extra = {}
        if merge_parts:
            total = int(offsets[-1]) if len(offsets) else 0
            extra['parts'] = dict(
                apsis_pos=res.apsis_pos[:total].cpu().numpy().astype(np.int64),
                angle_pos=torch.nonzero(mp).squeeze(1).cpu().numpy(),
                srt=srt, s_off=s_off, raw=raw, r_off=r_off,
                raw_pos=esel[~sorted_h].cpu().numpy(), p_has=p_has)
        return {**extra, 'apsis_offsets': offsets, 'apsis_ids': apsis_ids,
                'angles': angles.astype(adt, copy=False),
                'entered_offsets': e_off, 'entered_ids': entered,
                'departed_offsets': d_off, 'departed_ids': departed,
                'bulk_velocities': [bulk_c, bulk_p]}


def merge_onthefly(parts, nh):
    """Merge the ranks' on-the-fly outputs of one snapshot pair (ShardedOnTheFly).

    ``parts``: per rank, a dict with the rank's per-halo CSR outputs and each element's
    global row (``*_gpos``).  A halo's previous and current blocks tile their snapshots
    in halo order, so a global previous row orders apsis records and angle changes
    exactly as the reference emits them (previous-block order, halos in order,
    :154-174); entered / departed IDs are per-halo sorted unique (setdiff1d, :145,
    :168; the ranks' ID sets are disjoint), except the entered IDs of a halo without a
    progenitor block, which keep loader order (:178), i.e. global current-row order."""
    def cat(key, dt=None):
        xs = [np.asarray(q[key]) for q in parts]
        return np.concatenate(xs) if xs else np.zeros(0, dt)

    def halo_of(key):
        return np.concatenate([np.repeat(np.arange(nh), np.diff(q[key])) for q in parts]) \
            if parts else np.zeros(0, np.int64)

    def counts(key):
        return np.sum([np.diff(q[key]) for q in parts], axis=0) if parts else np.zeros(nh, np.int64)

    def offsets(c):
        return np.concatenate([[0], np.cumsum(c)]).astype(np.int64)

    out = {}
    order = np.argsort(cat('apsis_gpos'), kind='stable')
    out['apsis_ids'] = cat('apsis_ids')[order]
    out['apsis_offsets'] = offsets(counts('apsis_offsets'))
    out['angles'] = cat('angles')[np.argsort(cat('angle_gpos'), kind='stable')]
    dep, dh = cat('departed_ids'), halo_of('departed_offsets')
    out['departed_ids'] = dep[np.lexsort((dep, dh))]
    out['departed_offsets'] = offsets(counts('departed_offsets'))
    srt, sh = cat('srt'), halo_of('s_off')
    srt = srt[np.lexsort((srt, sh))]
    raw, rh = cat('raw'), halo_of('r_off')
    raw = raw[np.lexsort((cat('raw_gpos'), rh))]
    out['entered_ids'], out['entered_offsets'] = _interleave_halos(
        parts[0]['p_has'], srt, offsets(counts('s_off')), raw, offsets(counts('r_off')))
    return out


class ShardedOnTheFly:
    """The on-the-fly driver over ID-range shards (BASELINE configs[4]):
    one process per GPU, ``torch.distributed`` (RCCL, or gloo in the tests).

    Every rank receives both snapshots from the loader (the reference's contract),
    keeps the particles of its ID range (``IdRangeOwner``, fitted on the first
    snapshot it sees) and runs the on-the-fly pipeline on them; a particle's rows in
    the two snapshots are on the same rank, so the join has no exchange.  Bulk
    velocities are whole-block sums: halo j's is computed by rank j % world on the
    full block and the rows are all-gathered.  The outputs -- small next to the
    snapshots -- are all-gathered with their global rows and merged
    (``merge_onthefly``) into exactly the single-process file; rank 0 writes it.

    ``track_orbits(..., engine=ShardedOnTheFly(OrbitEngine(mode=...)))``."""

    def __init__(self, engine, group=None, owner=None):
        from .sharding import IdRangeOwner
        self.eng = engine
        self.mode = engine.mode
        self.group = group
        self.owner = owner if owner is not None else IdRangeOwner()
        engine.emit_positions = True
        self.otf = OnTheFly(engine)
        self.carry = None

    @property
    def rank(self):
        import torch.distributed as dist
        return dist.get_rank(self.group)

    def agree(self, flag):
        """True on every rank iff ``flag`` is true on every rank (a carry is used only
        when all ranks hold one, so their collectives stay in step)."""
        import torch.distributed as dist
        got = [None] * dist.get_world_size(self.group)
        dist.all_gather_object(got, bool(flag), group=self.group)
        return all(got)

    def run(self, snaps, slices, centres, carried=None):
        """``carried``: this object's ``carry`` from the previous call, whose current
        snapshot is this call's previous one (``snaps[1]`` is then None): the rank's
        shard of it, its device frame state and its bulk velocities are reused."""
        import torch.distributed as dist
        from .sharding import shard_snapshot
        world, rank = dist.get_world_size(self.group), dist.get_rank(self.group)
        eng = self.eng
        self.owner.fit(np.asarray(snaps[0]['ids']))
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
            sl = np.asarray(sl, dtype=np.int64).reshape(-1, 2)
            n = len(snap['ids'])
            nh = len(sl)
            full = dict(snap)
            full['region_offsets'] = _block_starts(sl, n)
            mine = np.arange(rank, nh, world)
            rows = eng.block_bulk(full, mine) if len(mine) else None
            got = [None] * world
            dist.all_gather_object(got, (mine, rows), group=self.group)
            bulk = None
            for idx, r in got:
                if r is not None:
                    if bulk is None:
                        bulk = np.zeros((nh, 3), dtype=r.dtype)
                    bulk[idx] = r
            keep = self.owner(np.asarray(snap['ids']), world) == rank
            sh, sel, st, cnt = shard_snapshot(full, keep)
            lsl = np.where(sl[:, :1] >= 0, np.stack([st, st + cnt], axis=1), -1)
            shards.append(sh)
            lslices.append(lsl)
            sels.append(sel)
            bulks.append(bulk if bulk is not None else np.zeros((0, 3)))
        out = self.otf.run(shards, lslices, centres, carried=otf_carry, bulks=bulks,
                           merge_parts=True)
        self.carry = (self.otf.carry, sels[0])
        q = out.pop('parts')
        mine = dict(apsis_offsets=out['apsis_offsets'], apsis_ids=out['apsis_ids'],
                    apsis_gpos=sels[1][q['apsis_pos']],
                    angles=out['angles'], angle_gpos=sels[1][q['angle_pos']],
                    departed_offsets=out['departed_offsets'], departed_ids=out['departed_ids'],
                    srt=q['srt'], s_off=q['s_off'], raw=q['raw'], r_off=q['r_off'],
                    raw_gpos=sels[0][q['raw_pos']], p_has=q['p_has'])
        allp = [None] * world
        dist.all_gather_object(allp, mine, group=self.group)
        merged = merge_onthefly(allp, len(slices[0]))
        out.update(merged)
        out['angles'] = out['angles'].astype(mine['angles'].dtype, copy=False)
        return out


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
