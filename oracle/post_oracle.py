"""ORACLE — CPU restatement of the reference's consumers/producers of the orbit path
(SURVEY.md §8(f) rows f3 and f4).

TEST INFRASTRUCTURE ONLY.  Only ``tests/`` and the ``cpu_baseline`` leg of the
benchmarks may import this module, as the checker / the timed CPU baseline — never as
part of the product path (``orbitanalysis_amd.postprocessing`` / ``.progenitors`` run
on the device and raise without it).

Pinned: ``tests/test_oracle_golden.py`` checks every function here against vectors
produced by importing the reference itself in the build container
(``tools/gen_golden.py`` -> ``tests/golden/g9_collate.npz``,
``tests/golden/g10_progenitors.npz``).

Restated from ``/root/reference/orbitanalysis`` (numpy 2.2.6 semantics):

* ``collate_apsides``          postprocessing.py:30-174 on an in-memory store
                               ({group: {dataset: array}}, attrs)
* ``save_final_apsis_counts``  postprocessing.py:176-240
* ``get_central_particle_ids`` progenitors.py:5-56 (ties in radius broken by block
                               position; numpy's introsort leaves their order
                               unspecified, so tied radii are "parity unpinned")
* ``find_main_progenitors``    progenitors.py:59-117
"""
import numpy as np

from oracle.orbit_oracle import dot3, recenter_coordinates, myin1d


def _tag(mode):
    return '{}er'.format(mode[:-3])


def collate_apsides(groups, attrs, halo_ids=None, snapshot_number=None,
                    angle_cut=np.pi / 4, data_type=None):
    """Cumulative per-halo unique orbiting IDs + passage counts per snapshot
    (postprocessing.py:30-174).  Returns {group name: {dataset: array}} of the
    collated file, in the reference's dataset creation order (:148-162)."""
    skeys = sorted(groups)
    snaps = np.array([int(k.split('_')[1]) for k in skeys])
    final = groups[skeys[-1]]['halo_IDs']
    tag = _tag(str(attrs['mode']))
    if halo_ids is None:
        halo_ids = final
    elif len(np.intersect1d(final, halo_ids)) < len(halo_ids):            # :70-78
        raise ValueError('halo IDs not processed: %s' % np.setdiff1d(halo_ids, final))
    last = len(snaps) - 1
    sind = last if snapshot_number is None else np.argwhere(snaps == snapshot_number).flatten()[0]
    out = {}
    acc = None                 # per collated halo: list of appended ID arrays
    for s in snaps[:sind + 1]:
        g = groups['snapshot_%03d' % s]
        cur = g['halo_IDs']
        fin = g['final_descendant_IDs'] if s != snaps[-1] else cur      # :98-101
        common = np.intersect1d(fin, halo_ids)
        h1 = myin1d(fin, common)
        h2 = myin1d(halo_ids, common)
        ids = g[tag + '_IDs']
        if len(ids) == 0:                                              # :106, :130-131
            continue
        if acc is None:
            dt = ids.dtype if data_type is None else data_type
            acc = [[np.array([], dtype=dt)] for _ in halo_ids]
        off = g['region_offsets']
        ang = g['angles']
        for a, b in zip(h1, h2):
            sl = slice(off[a], off[a + 1])
            acc[b].append(ids[sl][ang[sl] > angle_cut])               # :123-128
        uniq, cnt, lens = [], [], []
        present = set(int(b) for b in h2)
        for i, parts in enumerate(acc):
            u, c = np.unique(np.concatenate(parts), return_counts=True)
            uniq.append(u)
            cnt.append(c)
            if i in present:                                            # :138-139
                lens.append(len(u))
        d = {'particle_IDs': np.concatenate(uniq),
             tag + '_counts': np.concatenate(cnt),
             'halo_offsets': np.cumsum([0] + lens)[:-1]}
        if s != snaps[-1]:
            d['final_descendant_IDs'] = fin[h1]
        d['halo_IDs'] = cur[h1]
        d['halo_positions'] = g['region_positions'][h1]
        d['halo_velocities'] = g['bulk_velocities'][h1]
        d['region_radii'] = g['region_radii'][h1]
        out['snapshot_%03d' % s] = d
    return out


def save_final_apsis_counts(cgroups, mode, snapshot_numbers=None):
    """Per collated snapshot, the count each listed particle has at the final
    snapshot (postprocessing.py:176-240).  Returns {group: counts_final (float64)}.
    Entries no halo slice covers stay 0 here (np.empty in the reference)."""
    tag = _tag(mode)
    skeys = np.array(sorted(cgroups))
    lastg = cgroups[skeys[-1]]
    ids_f = lastg['particle_IDs']
    cnt_f = lastg[tag + '_counts']
    halos_f = lastg['halo_IDs']
    off_f = list(lastg['halo_offsets']) + [len(ids_f)]
    if snapshot_numbers is None:
        sel = skeys[:-1]
    else:
        nums = np.array([int(k.split('_')[-1]) for k in skeys])
        sel = skeys[np.where(np.isin(nums, snapshot_numbers))[0]]
    out = {}
    for k in sel:
        g = cgroups[k]
        ids = g['particle_IDs']
        desc = g['final_descendant_IDs']
        off = list(g['halo_offsets']) + [len(ids)]
        hinds = myin1d(halos_f, desc)
        retro = np.zeros(len(ids))
        for h2, h1 in enumerate(hinds):
            fs = slice(off_f[h1], off_f[h1 + 1])
            cs = slice(off[h2], off[h2 + 1])
            fid = ids_f[fs]
            q = ids[cs]
            order = np.argsort(fid, kind='stable')
            pos = np.searchsorted(fid[order], q)
            ok = (pos < len(fid)) & (fid[order][np.minimum(pos, len(fid) - 1)] == q) \
                if len(fid) else np.zeros(len(q), bool)
            if not np.all(ok):
                raise ValueError('%s: particle IDs absent from the final snapshot' % k)
            retro[cs] = cnt_f[fs][order[pos]]
        out[k] = retro
    return out


def get_central_particle_ids(snapshot, halo_positions, n=100):
    """IDs of the n particles nearest each halo centre (progenitors.py:5-56)."""
    ids = snapshot['ids']
    x = snapshot['coordinates']
    offs = list(snapshot['region_offsets']) + [len(ids)]
    rc = np.empty(np.shape(x))
    for k, pos in enumerate(halo_positions):
        if k + 1 >= len(offs):
            break
        a, b = offs[k], offs[k + 1]
        d = x[a:b] - pos
        if 'box_size' in snapshot:
            d = recenter_coordinates(d, snapshot['box_size'])
        rc[a:b] = d
    r = np.sqrt(dot3(rc, rc))
    blocks = [ids[a + np.argsort(r[a:b], kind='stable')[:n]] for a, b in zip(offs[:-1], offs[1:])]
    return np.hstack(blocks), np.cumsum([0] + [len(c) for c in blocks])[:-1]


def find_main_progenitors(halo_pids, halo_offsets, tracked_pids, tracked_offsets):
    """Halo (block number) holding the plurality of each tracked block's IDs, ties to
    the lowest number, -1 if none (progenitors.py:59-117)."""
    tp = np.asarray(tracked_pids)
    _, first = np.unique(tp, return_index=True)
    t = -np.ones(len(tp), dtype=int)
    t[first] = tp[first]                                                # :82-84
    hp = np.asarray(halo_pids)
    ho = np.asarray(halo_offsets)
    hnum = np.searchsorted(ho, np.arange(len(hp)), side='right') - 1    # :92-93
    order = np.argsort(hp, kind='stable')
    srt = hp[order]
    pos = np.searchsorted(srt, t)
    pc = np.minimum(pos, max(len(hp) - 1, 0))
    found = (pos < len(hp)) & (srt[pc] == t) if len(hp) else np.zeros(len(t), bool)
    prog = np.where(found, hnum[order[pc]] if len(hp) else -1, -1)
    toff = list(tracked_offsets) + [len(tp)]
    out = []
    for a, b in zip(toff[:-1], toff[1:]):
        v = prog[a:b]
        v = v[v != -1]
        if len(v) == 0:
            out.append(-1)
        else:
            u, c = np.unique(v, return_counts=True)
            out.append(u[np.argmax(c)])
    return out
