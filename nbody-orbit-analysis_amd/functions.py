"""The module-level functions of ``orbitanalysis.track_orbits`` on the device.

The reference exposes its per-halo building blocks as importable functions
(track_orbits.py:247-351) and users call them directly; these are the same
functions -- same names, arguments, return values and dtypes -- computed by the
HIP library:

* ``region_frame``               a frame-only ``oa_step`` launch over the one block,
                                 with the exact float64 radial velocities written out
* ``compare_radial_velocities``  ``oa_match_ids`` (the in1d / myin1d join) and
                                 ``oa_compare_pairs`` (sign flips, arccos)
* ``calc_angles``                ``oa_angle_add`` (float16 + change, rounded to f16)

Inputs and outputs are host NumPy arrays, as in the reference; the index
bookkeeping around the device results (boolean selections) stays on the host.
"""
import numpy as np
import torch

from . import _native as N
from .engine import OrbitEngine, to_device, _TORCH_FROM_NP

_ENGINES = {}


def _engine(mode='pericentric'):
    dev = torch.cuda.current_device() if torch.cuda.is_available() else None
    key = (dev, mode)
    if key not in _ENGINES:
        _ENGINES[key] = OrbitEngine(mode=mode)
    return _ENGINES[key]


def _stream():
    return torch.cuda.current_stream().cuda_stream


def region_frame(snapshot, region_slice, region_position, region_bulk_vel, H):
    """Unit radial vectors, radial velocities and bulk velocity of one region block
    (track_orbits.py:247-290)."""
    eng = _engine()
    lo, hi = int(region_slice[0]), int(region_slice[1])
    n = max(hi - lo, 0)
    m = snapshot['masses']
    sub = {'ids': np.arange(n, dtype=np.int64),
           'coordinates': np.asarray(snapshot['coordinates'])[lo:hi],
           'velocities': np.asarray(snapshot['velocities'])[lo:hi],
           'masses': m[lo:hi] if isinstance(m, np.ndarray) else m,
           'region_offsets': np.zeros(1, dtype=np.int64),
           'redshift': snapshot['redshift']}
    if 'box_size' in snapshot:
        sub['box_size'] = snapshot['box_size']
    dsub = dict(sub)
    for k in ('ids', 'coordinates', 'velocities'):
        dsub[k] = to_device(sub[k], eng.device)
    if isinstance(m, np.ndarray):
        dsub['masses'] = to_device(sub['masses'], eng.device)
    centres = np.asarray([region_position])
    bulk_cat = None if region_bulk_vel is None else np.asarray([region_bulk_vel])
    pr = eng.prepare(dsub, centres, bulk_cat, H, snapshot['redshift'], np.zeros(1, np.int64),
                     False, plan_src=sub)
    vr = torch.empty(max(n, 1), dtype=torch.float64, device=eng.device)
    pr.args.vr_out = vr.data_ptr()
    eng.launch(pr, None)
    rhat = pr.rhat[:3 * n].view(n, 3).cpu().numpy()
    if region_bulk_vel is None:
        bulk = pr.halos.cpu().numpy().view(N.HALO_DTYPE)['bulk'][0].astype(pr.plan.bulk)
    else:
        bulk = region_bulk_vel
    return rhat, vr[:n].cpu().numpy(), bulk


def compare_radial_velocities(ids, ids_prev, radial_vels, radial_vels_prev, rhat, rhat_prev,
                              mode):
    """Sign flips of v_r between a block and its progenitor block
    (track_orbits.py:293-327); outputs in previous-block order."""
    if mode not in N.MODE:
        raise ValueError("Orbit detection mode not recognized. Please specify either "
                         "'pericentric' or 'apocentric'.")
    lib = N.load(require_device=True)
    dev = torch.device('cuda', torch.cuda.current_device())
    ids, ids_prev = np.asarray(ids), np.asarray(ids_prev)
    if ids.dtype.itemsize != ids_prev.dtype.itemsize or ids.dtype.kind not in 'iu':
        raise NotImplementedError('ids and ids_prev must be integers of one width')
    n, n_prev = len(ids), len(ids_prev)
    td = np.result_type(np.asarray(rhat).dtype, np.asarray(rhat_prev).dtype)
    if td not in (np.float32, np.float64):
        raise NotImplementedError('r-hat dtype %s' % td)
    st = _stream()
    d_ids = to_device(ids, dev)
    d_idp = to_device(ids_prev, dev)
    ws = torch.empty(int(lib.oa_match_workspace_bytes(n)), dtype=torch.uint8, device=dev)
    match = torch.empty(max(n_prev, 1), dtype=torch.int64, device=dev)
    N.check(lib.oa_match_ids(d_ids.data_ptr() if n else None, n, d_idp.data_ptr(), n_prev,
                             ids.dtype.itemsize, ws.data_ptr(), match.data_ptr(), st),
            'oa_match_ids')
    vr = to_device(np.asarray(radial_vels, dtype=np.float64), dev)
    vrp = to_device(np.asarray(radial_vels_prev, dtype=np.float64), dev)
    rh = to_device(np.asarray(rhat, dtype=td).reshape(-1, 3), dev)
    rhp = to_device(np.asarray(rhat_prev, dtype=td).reshape(-1, 3), dev)
    flag = torch.empty(max(n_prev, 1), dtype=torch.uint8, device=dev)
    change = torch.empty(max(n_prev, 1), dtype=_TORCH_FROM_NP[np.dtype(td)], device=dev)
    N.check(lib.oa_compare_pairs(match.data_ptr(), n_prev, vr.data_ptr() if n else None,
                                 vrp.data_ptr(), rh.data_ptr() if n else None, rhp.data_ptr(),
                                 int(td == np.float64), N.MODE[mode], flag.data_ptr(),
                                 change.data_ptr(), st), 'oa_compare_pairs')
    m = match[:n_prev].cpu().numpy()
    keep = m >= 0
    inds_match = m[keep]
    apsis_inds = np.flatnonzero(flag[:n_prev].cpu().numpy()[keep])
    ids_prev_ = ids_prev[keep]
    return {'apsis_inds': apsis_inds, 'apsis_ids': ids_prev_[apsis_inds],
            'ids_match': ids[inds_match], 'inds_match': inds_match,
            'inds_departed': np.flatnonzero(~keep),
            'angle_changes': change[:n_prev].cpu().numpy()[keep]}


def calc_angles(npart, angles_prev, apsis_dict):
    """Swept angles since the last apsis, reset at apsis (track_orbits.py:330-351)."""
    lib = N.load(require_device=True)
    dev = torch.device('cuda', torch.cuda.current_device())
    angles_prev = np.asarray(angles_prev)
    if angles_prev.dtype != np.float16:
        raise NotImplementedError('angles_prev must be float16 (the reference state dtype)')
    kept = np.delete(angles_prev, apsis_dict['inds_departed'])
    ch = np.asarray(apsis_dict['angle_changes'])
    if ch.dtype not in (np.float32, np.float64):
        raise NotImplementedError('angle_changes dtype %s' % ch.dtype)
    k = len(kept)
    if len(ch) != k:
        raise ValueError('operands could not be broadcast together with shapes (%d,) (%d,)'
                         % (k, len(ch)))
    out = torch.empty(max(k, 1), dtype=torch.int16, device=dev)
    if k:
        d_prev = to_device(kept.view(np.uint16), dev)
        d_ch = to_device(ch, dev)
        N.check(lib.oa_angle_add(d_prev.data_ptr(), d_ch.data_ptr(), k, int(ch.dtype == np.float64),
                                 out.data_ptr(), _stream()), 'oa_angle_add')
    acc = out[:k].cpu().numpy().view(np.float16).copy()
    ai = apsis_dict['apsis_inds']
    apsis_angles = acc[ai].copy()
    acc[ai] = 0
    angles = np.zeros(npart, dtype=np.float16)
    angles[apsis_dict['inds_match']] = acc
    return angles, apsis_angles
