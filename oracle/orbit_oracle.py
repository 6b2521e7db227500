"""ORACLE — CPU restatement of the reference's per-snapshot orbit-tagging path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline — never as part of the product path.

Pinned: ``tests/test_oracle_golden.py`` checks every function here against golden
vectors produced by importing the reference itself in the build container
(``tools/gen_golden.py`` -> ``tests/golden/*.npz``), bit for bit.

Restated from ``/root/reference/orbitanalysis`` (numpy 2.2.6 semantics):

* ``dot3``                      einsum('...i,...i') rows; summation tree probed on the
                                reference host: f64 ``(p0+p2)+p1``, f32 ``(p0+p1)+p2``,
                                no FMA (SURVEY.md §7 "Bit-exact signs").  Written out
                                explicitly so the oracle does not depend on the SIMD
                                dispatch of whatever host runs it.
* ``recenter_coordinates``      utils.py:24-33
* ``hubble_parameter``          utils.py:36-39
* ``myin1d``                    utils.py:4-11 (precondition: unique values, b ⊆ a)
* ``region_frame``              track_orbits.py:247-290
* ``compare_radial_velocities`` track_orbits.py:293-327 (sort/searchsorted join;
                                identical result under the unique-ID precondition)
* ``calc_angles``               track_orbits.py:330-351
* ``track_orbits``              track_orbits.py:9-244 driver loop, writing to an
                                in-memory record instead of HDF5 (save_to_file :366-397)
* ``onthefly_*``                track_orbits_onthefly.py:8-205
"""
import numpy as np


# --------------------------------------------------------------------------- utils
def dot3(a, b):
    """Row-wise dot of (...,3) arrays in the reference host's einsum order."""
    dt = np.result_type(a, b)
    p = np.asarray(a, dtype=dt) * np.asarray(b, dtype=dt)
    if dt == np.float32:
        return (p[..., 0] + p[..., 1]) + p[..., 2]
    return (p[..., 0] + p[..., 2]) + p[..., 1]


def recenter_coordinates(position, boxsize):
    """Single periodic wrap per dimension (utils.py:24-33): strict ``> L/2`` then
    strict ``< -L/2`` on the already-shifted column.  A scalar box is broadcast to 3
    dims as float64; an array box wraps only its first ``len(box)`` dims."""
    if isinstance(boxsize, (float, np.floating, int, np.integer)):
        boxsize = np.full(3, np.float64(boxsize))
    for d, L in enumerate(boxsize):
        col = position[:, d]
        position[:, d] = np.where(col > L / 2, col - L, col)
        col = position[:, d]
        position[:, d] = np.where(col < -L / 2, col + L, col)
    return position


def hubble_parameter(z, H0, Omega_m, Omega_L, Omega_k=0):
    """H(z) = H0 sqrt(Om (1+z)^3 + Ok (1+z)^2 + OL)  (utils.py:36-39); np.float64."""
    return H0 * np.sqrt(Omega_m * (1 + z) ** 3 + Omega_k * (1 + z) ** 2 + Omega_L)


def myin1d(a, b):
    """Indices of ``a`` whose values are in ``b``, in ``b``'s order (utils.py:4-11)."""
    a = np.asarray(a)
    b = np.asarray(b)
    order = np.argsort(a, kind='stable')
    pos = np.searchsorted(a[order], b)
    return order[pos]


def seq_sum_rows(x):
    """numpy ``sum(axis=0)`` of a C-contiguous (n,k) array: first row, then rows
    added one at a time (probed: sequential, not pairwise)."""
    acc = x[0].copy()
    for i in range(1, len(x)):
        acc = acc + x[i]
    return acc


def pairwise_sum(a):
    """numpy 1-D ``sum``: 0 + pairwise(chunk) over 8192-element buffer chunks,
    pairwise = numpy's 8-accumulator blocked recursion (leaves <= 128)."""
    t = a.dtype.type

    def pw(x):
        n = len(x)
        if n < 8:
            r = t(0)
            for v in x:
                r = t(r + v)
            return r
        if n <= 128:
            acc = [x[j] for j in range(8)]
            i = 8
            while i < n - (n % 8):
                for j in range(8):
                    acc[j] = t(acc[j] + x[i + j])
                i += 8
            r = t(t(t(acc[0] + acc[1]) + t(acc[2] + acc[3])) +
                  t(t(acc[4] + acc[5]) + t(acc[6] + acc[7])))
            while i < n:
                r = t(r + x[i])
                i += 1
            return r
        h = n // 2
        h -= h % 8
        return t(pw(x[:h]) + pw(x[h:]))

    total = t(0)
    for s in range(0, len(a), 8192):
        total = t(total + pw(a[s:s + 8192]))
    return total


# --------------------------------------------------------------- batch hot path
def bulk_velocity(velocities, masses, region_bulk_vel=None):
    """Catalogue value if given, else mass-weighted (masses ndarray) or plain mean
    (track_orbits.py:262-284)."""
    if region_bulk_vel is not None:
        return region_bulk_vel
    if isinstance(masses, np.ndarray):
        return np.sum(masses[:, None] * velocities, axis=0) / np.sum(masses)
    return np.mean(velocities, axis=0)


def region_frame(snapshot, region_slice, region_position, region_bulk_vel, H):
    """Unit radial vectors, radial velocities and bulk velocity of one region
    block (track_orbits.py:247-290)."""
    lo, hi = int(region_slice[0]), int(region_slice[1])
    x = snapshot['coordinates'][lo:hi]
    v = snapshot['velocities'][lo:hi]
    dx = x - region_position
    if 'box_size' in snapshot:
        dx = recenter_coordinates(dx, snapshot['box_size'])
    m = snapshot['masses']
    bulk = bulk_velocity(v, m[lo:hi] if isinstance(m, np.ndarray) else m, region_bulk_vel)
    w = (v - bulk) + (H * dx) / (1 + snapshot['redshift'])
    with np.errstate(divide='ignore', invalid='ignore'):
        r = np.sqrt(dot3(dx, dx))
        rhat = dx / r[:, None]
        vr = dot3(w, rhat)
    return rhat, vr, bulk


def _join(ids, ids_prev):
    """For each previous-block ID: found flag and its index in the current block."""
    order = np.argsort(ids, kind='stable')
    sid = ids[order]
    if sid.size == 0:
        return np.zeros(ids_prev.size, dtype=bool), np.zeros(ids_prev.size, dtype=np.int64)
    pos = np.minimum(np.searchsorted(sid, ids_prev), sid.size - 1)
    found = sid[pos] == ids_prev
    return found, order[pos]


def compare_radial_velocities(ids, ids_prev, radial_vels, radial_vels_prev,
                              rhat, rhat_prev, mode):
    """Sign-flip detection between a block and its progenitor block
    (track_orbits.py:293-327).  Output order follows the previous block."""
    found, where = _join(ids, ids_prev)
    inds_departed = np.flatnonzero(~found)
    keep = found
    ids_prev_ = ids_prev[keep]
    inds_match = where[keep]
    vr_prev_ = radial_vels_prev[keep]
    vr_match = radial_vels[inds_match]
    if mode == 'pericentric':
        cond = (vr_prev_ < 0) & (vr_match > 0)
    else:
        cond = (vr_prev_ > 0) & (vr_match < 0)
    apsis_inds = np.flatnonzero(cond)
    with np.errstate(invalid='ignore'):
        changes = np.arccos(dot3(rhat_prev[keep], rhat[inds_match]))
    return {'apsis_inds': apsis_inds, 'apsis_ids': ids_prev_[apsis_inds],
            'ids_match': ids[inds_match], 'inds_match': inds_match,
            'inds_departed': inds_departed, 'angle_changes': changes}


def calc_angles(npart, angles_prev, apsis_dict):
    """Swept angle since the last apsis; reset at apsis (track_orbits.py:330-351)."""
    acc = np.delete(angles_prev, apsis_dict['inds_departed']) + apsis_dict['angle_changes']
    at_apsis = acc[apsis_dict['apsis_inds']].copy()
    acc[apsis_dict['apsis_inds']] = 0.0
    out = np.zeros(npart)
    out[apsis_dict['inds_match']] = acc
    return out.astype(np.float16), at_apsis.astype(np.float16)


class MemoryRecord:
    """In-memory stand-in for the HDF5 savefile layout (track_orbits.py:354-397)."""

    def __init__(self):
        self.attrs = {}
        self.groups = {}
        self.checkpoint = None

    def last_snapshot(self):
        return int(sorted(self.groups)[-1].split('_')[1])


def track_orbits(snapshot_numbers, main_branches, regions, load_snapshot_data,
                 record, mode='pericentric', checkpoint=False, resume=False):
    """Batch driver loop (track_orbits.py:73-240) writing into ``record``."""
    if len(main_branches) != len(snapshot_numbers):
        raise ValueError('len(main_branches) != len(snapshot_numbers)')
    if mode not in ('pericentric', 'apocentric'):
        raise ValueError('bad mode')
    mb = np.asarray(main_branches)
    if mb.ndim == 1:
        mb = mb[:, None]
    sn = np.asarray(snapshot_numbers)
    o = np.argsort(sn)
    sn, mb = sn[o], mb[o]
    if resume:
        k = int(np.flatnonzero(sn == record.last_snapshot())[0])
        sn, mb = sn[k:], mb[k:]
    istart, started = 0, False
    prev = None
    for i, (halo_ids, snap_no) in enumerate(zip(mb, sn)):
        exists = np.flatnonzero(halo_ids != -1)
        if exists.size == 0:
            if not started:
                istart = i + 1
            continue
        hids = halo_ids[exists]
        pos, radii, bulks = regions(snap_no, hids)
        snap = load_snapshot_data(snap_no, pos, radii)
        if len(snap['coordinates']) == 0:
            if not started:
                istart = i + 1
            continue
        started = True
        offs = list(snap['region_offsets']) + [len(snap['ids'])]
        slices = np.array(list(zip(offs[:-1], offs[1:])))
        H = hubble_parameter(snap['redshift'], snap['H0'], snap['Omega_m'],
                             snap['Omega_L'], snap.get('Omega_k', 0))
        if i == 0 and not resume:
            record.attrs['mode'] = mode
            if 'box_size' in snap:
                record.attrs['box_size'] = snap['box_size']
        rh_l, vr_l, bulk_l, ang_l, aps_ids, aps_angs = [], [], [], [], [], []
        for j, hind in enumerate(exists):
            rh, vr, bulk = region_frame(snap, slices[j], pos[j],
                                        None if bulks is None else bulks[j], H)
            n = int(slices[j][1] - slices[j][0])
            angs = np.zeros(n, dtype=np.float16)
            if i > istart and hind in prev['exists']:
                p = int(np.flatnonzero(prev['exists'] == hind)[0])
                a, b = prev['slices'][p]
                d = compare_radial_velocities(snap['ids'][slices[j][0]:slices[j][1]],
                                              prev['ids'][a:b], vr, prev['vr'][a:b],
                                              rh, prev['rhat'][a:b], mode)
                angs, aang = calc_angles(n, prev['angles'][a:b], d)
                aps_ids.append(d['apsis_ids'])
                aps_angs.append(aang)
            rh_l.append(rh)
            vr_l.append(vr)
            bulk_l.append(bulk)
            ang_l.append(angs)
        angles = np.concatenate(ang_l)
        if i > istart:
            hinds = np.flatnonzero(np.isin(exists, prev['exists']))
            g = {
                'region_offsets': np.cumsum([0] + [len(x) for x in aps_ids]),
                '{}er_IDs'.format(mode[:-3]): np.concatenate(aps_ids),
                'angles': np.concatenate(aps_angs),
                'halo_IDs': hids[hinds],
                'region_radii': radii[hinds],
                'region_positions': pos[hinds],
                'bulk_velocities': np.array(bulk_l)[hinds],
            }
            if snap_no != sn[-1]:
                g['final_descendant_IDs'] = mb[-1][prev['exists']]
            record.groups['snapshot_%03d' % snap_no] = g
            if checkpoint:
                record.checkpoint = angles
        elif resume:
            angles = record.checkpoint
        prev = {'rhat': np.concatenate(rh_l), 'vr': np.concatenate(vr_l),
                'ids': snap['ids'], 'angles': angles, 'slices': slices,
                'exists': exists}
    return record


# ------------------------------------------------------------ on-the-fly pair
def onthefly_region_frame(snapshot, region_slices, region_positions):
    """All-halo frame without Hubble term or catalogue bulk; r̂/vr buffers take the
    input coordinate/velocity dtypes (track_orbits_onthefly.py:71-120)."""
    x, v = snapshot['coordinates'], snapshot['velocities']
    dx = np.empty(x.shape, dtype=x.dtype)
    w = np.empty(v.shape, dtype=v.dtype)
    bulks = []
    m = snapshot['masses']
    for (lo, hi), c in zip(region_slices, region_positions):
        lo, hi = int(lo), int(hi)
        d = x[lo:hi] - c
        if 'box_size' in snapshot:
            d = recenter_coordinates(d, snapshot['box_size'])
        dx[lo:hi] = d
    for lo, hi in region_slices:
        lo, hi = int(lo), int(hi)
        with np.errstate(invalid='ignore', divide='ignore'):
            b = bulk_velocity(v[lo:hi], m[lo:hi] if isinstance(m, np.ndarray) else m)
        w[lo:hi] = v[lo:hi] - b
        bulks.append(b)
    with np.errstate(divide='ignore', invalid='ignore'):
        r = np.sqrt(dot3(dx, dx))
        rhat = dx / r[:, None]
        vr = dot3(w, rhat)
    return rhat, vr, np.array(bulks)


def onthefly_compare(ids, ids_prev, vr, vr_prev, rhat, rhat_prev, slices, slices_prev, mode):
    """Per-halo CSR outputs of track_orbits_onthefly.py:123-205 (keys use
    ``mode[:8] + 'er'``, so apocentric -> 'apocentrer')."""
    tag = mode[:8] + 'er'
    orb_ids, orb_inds, ent, dep, mat, ang = [], [], [], [], [], []
    for (pa, pb), (ca, cb) in zip(slices_prev, slices):
        pa, pb, ca, cb = int(pa), int(pb), int(ca), int(cb)
        cur = ids[ca:cb]
        if pb - pa > 0:
            pid = ids_prev[pa:pb]
            d = compare_radial_velocities(cur, pid, vr[ca:cb], vr_prev[pa:pb],
                                          rhat[ca:cb], rhat_prev[pa:pb], mode)
            orb_inds.append(d['apsis_inds'])
            orb_ids.append(d['apsis_ids'])
            ent.append(np.setdiff1d(cur, pid))
            dep.append(np.setdiff1d(pid, cur))
            mat.append(d['ids_match'])
            ang.append(d['angle_changes'])
        else:
            e = np.array([], dtype=ids.dtype)
            ent.append(cur)
            orb_inds.append(e)
            orb_ids.append(e)
            dep.append(e)
            mat.append(e)
            ang.append(e)

    def csr(lst):
        return np.concatenate(lst), np.cumsum([0] + [len(x) for x in lst])

    out = {}
    out[tag + '_ids'], out[tag + '_offsets'] = csr(orb_ids)
    out[tag + '_inds'] = np.concatenate(orb_inds)
    out['entered_ids'], out['entered_offsets'] = csr(ent)
    out['departed_ids'], out['departed_offsets'] = csr(dep)
    out['matched_ids'], out['matched_offsets'] = csr(mat)
    out['angle_changes'] = np.concatenate(ang)
    return out


def onthefly_repack(arr, length, inds):
    arr = np.asarray(arr)
    shape = list(np.shape(arr))
    shape[0] = length
    out = -np.ones(tuple(shape), dtype=arr.dtype)
    out[inds] = arr
    return out


def onthefly_track_orbits(snapshot_number, progenitor_links, regions, load_snapshot_data,
                          mode='pericentric'):
    """Pairwise (s, s-1) driver (track_orbits_onthefly.py:8-58); returns the dict
    that save_to_file would write (:229-249)."""
    if mode not in ('pericentric', 'apocentric'):
        raise ValueError('bad mode')
    ids, rh, vr, rpos, rrad, bulks, sls = [], [], [], [], [], [], []
    box = None
    for s, row in zip([snapshot_number, snapshot_number - 1], progenitor_links):
        row = np.asarray(row)
        ex = np.flatnonzero(row != -1)
        p, r = regions(s, row[ex])
        p_, r_ = onthefly_repack(p, len(row), ex), onthefly_repack(r, len(row), ex)
        rpos.append(p_)
        rrad.append(r_)
        snap = load_snapshot_data(s, p, r)
        ids.append(snap['ids'])
        offs = list(snap['region_offsets']) + [len(snap['ids'])]
        sl = onthefly_repack(np.array(list(zip(offs[:-1], offs[1:]))), len(row), ex)
        sls.append(sl)
        a, b, c = onthefly_region_frame(snap, sl, p_)
        rh.append(a)
        vr.append(b)
        bulks.append(c)
        box = snap.get('box_size', None)
    d = onthefly_compare(ids[0], ids[1], vr[0], vr[1], rh[0], rh[1], sls[0], sls[1], mode)
    tag = mode[:8] + 'er'
    out = {tag + '_offsets': d[tag + '_offsets'], tag + '_IDs': d[tag + '_ids'],
           'angles': d['angle_changes'],
           'entered_offsets': d['entered_offsets'], 'entered_IDs': d['entered_ids'],
           'departed_offsets': d['departed_offsets'], 'departed_IDs': d['departed_ids'],
           'progenitor_links': np.asarray(progenitor_links),
           'region_radii': rrad, 'region_positions': rpos, 'bulk_velocities': bulks}
    if box is not None:
        out['attr_box_size'] = box
    return out
