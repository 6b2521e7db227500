"""CPU baseline leg of ``bench.py`` — BENCH INFRASTRUCTURE ONLY.

Times the CPU restatement of the reference's per-halo path (``orbit_oracle``) on a
bounded sample of the bench workload, on the host cores of the GPU box, in a process
that never touches the GPU (``bench.py`` starts it as a child and reads one JSON
line).  Two algorithms are timed, both restating the reference's dataflow of
``track(j)`` for a compared snapshot (track_orbits.py:147-185):

* ``ref``   the reference's own join: ``setdiff1d`` + ``in1d`` + ``delete`` + ``myin1d``
            (three argsorts; utils.py:4-11, track_orbits.py:300-306), then the strict
            sign test, ``arccos`` and ``calc_angles`` (:311-351).  This is what the
            reference runs.
* ``port``  the oracle's ``compare_radial_velocities``: one argsort + ``searchsorted``
            join (identical output under the unique-ID precondition, faster).

Each is timed on 1 core, and ``ref`` also with the halos split over P processes
(the reference's own parallel axis, the halo pool of track_orbits.py:189-194):
contiguous halo ranges, every worker loads the sample (memory-mapped) and frames its
previous blocks untimed, then all start together at a barrier; the rate is the sample's
particles / (last end - first start).
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import orbit_oracle as O  # noqa: E402


def ref_compare(ids, ids_prev, vr, vr_prev, rhat, rhat_prev, mode):
    """compare_radial_velocities with the reference's own join (track_orbits.py:300-327)."""
    gone = np.setdiff1d(ids_prev, ids)
    inds_departed = np.where(np.isin(ids_prev, gone))[0]
    keep_ids = np.delete(ids_prev, inds_departed)
    keep_vr = np.delete(vr_prev, inds_departed)
    keep_rh = np.delete(rhat_prev, inds_departed, axis=0)
    # myin1d (utils.py:4-11): indices of ids in keep_ids, in keep_ids' order
    loc = np.isin(ids, keep_ids)
    order = ids[loc].argsort()[keep_ids.argsort().argsort()]
    inds_match = np.where(loc)[0][order]
    vm = vr[inds_match]
    cond = (keep_vr < 0) & (vm > 0) if mode == 'pericentric' else (keep_vr > 0) & (vm < 0)
    apsis_inds = np.flatnonzero(cond)
    with np.errstate(invalid='ignore'):
        changes = np.arccos(O.dot3(keep_rh, rhat[inds_match]))
    return {'apsis_inds': apsis_inds, 'apsis_ids': keep_ids[apsis_inds],
            'inds_match': inds_match, 'inds_departed': inds_departed,
            'angle_changes': changes}


def _load(path):
    d = np.load(path, mmap_mode='r')
    return {k: d[k] for k in d.files}


def _snap(d, pre):
    return {'ids': d[pre + 'ids'], 'coordinates': d[pre + 'x'], 'velocities': d[pre + 'v'],
            'masses': float(d['mass']), 'box_size': float(d['box']), 'redshift': float(d['z'])}


def _work(path, lo, hi, algo):
    """Untimed set-up of halos [lo, hi): their previous frames.  Returns a closure
    running the timed per-halo path and returning (particles, apsis IDs)."""
    d = _load(path)
    cur, prv = _snap(d, 'c_'), _snap(d, 'p_')
    cb, pb = d['c_off'], d['p_off']
    H, mode = float(d['H']), str(d['mode'])
    prev = []
    for j in range(lo, hi):
        rh, vr, _ = O.region_frame(prv, (pb[j], pb[j + 1]), d['p_centre'][j], d['p_bulk'][j], H)
        prev.append((rh, vr))
    ang = d['angles_prev']
    cmp = ref_compare if algo == 'ref' else O.compare_radial_velocities

    def timed():
        out = []
        for k, j in enumerate(range(lo, hi)):
            sl = (cb[j], cb[j + 1])
            rh, vr, _ = O.region_frame(cur, sl, d['c_centre'][j], d['c_bulk'][j], H)
            r = cmp(np.asarray(cur['ids'][sl[0]:sl[1]]), np.asarray(prv['ids'][pb[j]:pb[j + 1]]),
                    vr, prev[k][1], rh, prev[k][0], mode)
            O.calc_angles(sl[1] - sl[0], np.asarray(ang[pb[j]:pb[j + 1]]), r)
            out.append(r['apsis_ids'])
        return int(cb[hi] - cb[lo]), (np.concatenate(out) if out else np.zeros(0, np.int64))
    return timed


def _proc(path, lo, hi, algo, barrier, q):
    os.environ.setdefault('OMP_NUM_THREADS', '1')
    timed = _work(path, lo, hi, algo)
    barrier.wait()
    t0 = time.perf_counter()
    units, _ = timed()
    t1 = time.perf_counter()
    q.put((t0, t1, units))


def run_parallel(path, n_halos, workers, algo='ref'):
    """Rate over ``workers`` processes (halo ranges), timed from a common barrier."""
    ctx = mp.get_context('fork')            # this process never initialised a GPU
    bounds = np.linspace(0, n_halos, workers + 1).astype(int)
    barrier, q = ctx.Barrier(workers), ctx.Queue()
    ps = [ctx.Process(target=_proc, args=(path, int(bounds[i]), int(bounds[i + 1]), algo,
                                          barrier, q)) for i in range(workers)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    t0, t1 = min(r[0] for r in res), max(r[1] for r in res)
    units = sum(r[2] for r in res)
    return units / (t1 - t0), t1 - t0, units


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('sample')
    ap.add_argument('--workers', type=int, default=16)
    ap.add_argument('--ids-out', default=None)
    a = ap.parse_args()
    d = _load(a.sample)
    nh = len(d['c_off']) - 1
    out = {'halos': nh, 'particles': int(d['c_off'][-1])}
    for algo in ('port', 'ref'):
        timed = _work(a.sample, 0, nh, algo)
        t0 = time.perf_counter()
        units, ids = timed()
        dt = time.perf_counter() - t0
        out[algo + '_1core'] = {'rate': units / dt, 'seconds': dt}
        if a.ids_out and algo == 'ref':
            np.save(a.ids_out, ids)
    rate, dt, units = run_parallel(a.sample, nh, a.workers, 'ref')
    out['ref_pcore'] = {'rate': rate, 'seconds': dt, 'workers': a.workers}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
