"""Drop-in batch driver: ``track_orbits`` with the reference's signature, callbacks,
errors, verbose messages and savefile layout (orbitanalysis/track_orbits.py:9-244).

What changes is underneath: the per-halo Python loop and the pathos process pool
(track_orbits.py:147-194) are replaced by one fused HIP kernel launch per snapshot
over all halos (``engine.OrbitEngine``); the previous snapshot's state stays in
HBM.  ``npool`` is accepted for signature compatibility and ignored (halo
parallelism is the GPU grid).
"""
import inspect
import time

import numpy as np

from .engine import OrbitEngine
from .functions import region_frame, compare_radial_velocities, calc_angles  # noqa: F401
from .savefile import RankSink, open_savefile, group_datasets
from .utils import hubble_parameter


def track_orbits(snapshot_numbers, main_branches, regions, load_snapshot_data,
                 savefile, mode='pericentric', checkpoint=False, resume=False,
                 npool=1, verbose=True, engine=None):
    """
    Track the orbits of particles in gravitating systems (reference docstring:
    track_orbits.py:13-71).

    Parameters are those of the reference.  ``savefile`` may be a path (HDF5 via
    h5py) or a savefile object (``savefile.MemorySavefile``).  ``engine`` optionally
    supplies a configured ``OrbitEngine`` (device, LDS table sizes).
    """
    if len(main_branches) != len(snapshot_numbers):
        raise ValueError(
            "Number of halo main branch nodes does not equal the number of "
            "snapshot numbers supplied. Must have len(main_branches) == "
            "len(snapshot_numbers).")
    if (mode != 'pericentric') and (mode != 'apocentric'):
        raise ValueError(
            "Orbit detection mode not recognized. Please specify either "
            "'pericentric' or 'apocentric'.")

    tstart = time.time()
    out = open_savefile(savefile)

    main_branches = np.asarray(main_branches)
    if main_branches.ndim == 1:
        main_branches = main_branches[:, np.newaxis]
    snapshot_numbers = np.asarray(snapshot_numbers)
    order = np.argsort(snapshot_numbers)
    snapshot_numbers = snapshot_numbers[order]
    main_branches = main_branches[order]

    if resume:
        print('Resuming from file...\n')
        last = out.last_snapshot_number()
        sind = np.argwhere(snapshot_numbers == last).flatten()[0]
        snapshot_numbers = snapshot_numbers[sind:]
        main_branches = main_branches[sind:]

    eng = engine if engine is not None else OrbitEngine(mode=mode)
    if eng.mode != mode:
        raise ValueError('engine mode %r != mode %r' % (eng.mode, mode))
    if getattr(eng, 'rank', 0) != 0:
        # sharded run (sharding.ShardedEngine): every rank computes, rank 0 writes
        out = RankSink(out)
        verbose = False
    eng.reset()

    istart, started = 0, False
    progen_exists = None
    # A compare step's records come back while the next snapshot is loaded, planned
    # and run (engine.fetch_async), and are written one or two iterations later (or
    # after the loop).  With ``defer`` the engine does not even wait for a step's
    # kernels: the next snapshot's host planning overlaps them, and the step's status
    # is checked (and a re-plan run) before the next launch (OrbitEngine.step).
    # Engines without fetch_async (sharded: a collective gather) fetch inline.
    pipelined = hasattr(eng, 'fetch_async')
    defer = pipelined and not verbose and 'defer' in inspect.signature(eng.step).parameters
    groups = []                     # [res, ids dtype, fetched or None, save args, kw]
    # the pipelined run keeps the copy engine busy with records D2H: the engines pull
    # their per-step tables with a kernel instead (engine._upload), restored on exit
    pulls = [e for e in (eng, getattr(getattr(eng, 'local', None), 'engine', None))
             if pipelined and e is not None and hasattr(e, 'table_pull')]
    saved_pull = [e.table_pull for e in pulls]
    for e in pulls:
        e.table_pull = True

    def flush(keep=0):
        """Write the groups oldest first, leaving the newest ``keep`` in flight."""
        while len(groups) > keep:
            g = groups[0]
            if g[2] is None:
                g[2] = eng.fetch_async(g[0], g[1])
            offsets, ids, angles = g[2].wait()
            groups.pop(0)
            save_to_file(out, ids, offsets, angles, *g[3], **g[4])

    try:
        for i, (halo_ids, snapshot_number) in enumerate(zip(main_branches, snapshot_numbers)):

            if verbose:
                print('-' * 30, '\n')
                print('Snapshot {}\n'.format('%03d' % snapshot_number))

            halo_exists = np.argwhere(halo_ids != -1).flatten()
            if len(halo_exists) == 0:
                if started is False:
                    istart = i + 1
                continue
            halo_ids_ = halo_ids[halo_exists]

            region_positions, region_radii, region_bulk_vels = regions(snapshot_number, halo_ids_)
            snapshot = load_snapshot_data(snapshot_number, region_positions, region_radii)
            if len(snapshot['coordinates']) == 0:
                if started is False:
                    istart = i + 1
                continue
            started = True

            if 'Omega_k' not in snapshot:
                snapshot['Omega_k'] = 0
            H = hubble_parameter(snapshot['redshift'], snapshot['H0'], snapshot['Omega_m'],
                                 snapshot['Omega_L'], snapshot['Omega_k'])

            if i == 0 and not resume:
                box_size = snapshot['box_size'] if 'box_size' in snapshot else None
                out.initialize(mode, box_size)
                if verbose:
                    print('Savefile initialized\n')

            compare = i > istart
            angles_in, step_kw = None, {}
            if resume and not compare:
                # the reference opens savefile + '.checkpoint' here (track_orbits.py:229-232)
                angles_in = out.read_checkpoint()
                if angles_in is None:
                    raise FileNotFoundError('resume: no checkpoint angles in the savefile '
                                            '(run with checkpoint=True first)')
                layout = read_checkpoint_layout(out)
                if layout is not None:
                    step_kw['angles_layout'] = layout
            if defer:
                step_kw['defer'] = True
            # apsis IDs are the previous snapshot's IDs (ids_prev_[apsis_inds], :315-316):
            # they keep that snapshot's dtype
            ids_dtype_prev = eng.prev.plan.ids if compare else None

            if verbose:
                t0 = time.time()
            res = eng.step(snapshot, region_positions, region_bulk_vels, H, snapshot['redshift'],
                           halo_exists, compare, angles_in=angles_in, **step_kw)
            if defer:
                # the previous step, settled now, starts its D2H (queued on the copy
                # stream behind the older group's, so the copy engine does not idle while
                # the host writes), which runs during this step's kernels; then the group
                # before it is written (its records crossed PCIe during the previous
                # step's kernels; its host blocks are then free for reuse)
                if groups and groups[-1][2] is None:
                    groups[-1][2] = eng.fetch_async(groups[-1][0], groups[-1][1])
                flush(keep=1)
            else:
                flush()
            if compare and res.n_slots == 0:
                # the reference concatenates an empty list here (track_orbits.py:216)
                raise ValueError('need at least one array to concatenate')
            fetched = None
            if compare and not defer:
                fetched = eng.fetch_async(res, ids_dtype_prev) if pipelined else \
                    _Fetched(eng.fetch(res, ids_dtype_prev))
            if verbose:
                if pipelined and compare:
                    fetched.wait()
                print('Finished pericenter detection for snapshot {} in {} s\n'.format(
                    '%03d' % snapshot_number, time.time() - t0))

            if compare:
                hinds = np.where(res.has_prog)[0]
                if region_bulk_vels is None:
                    bulk = eng.bulk_velocities(res, eng.prev.plan)
                else:
                    # the reference's per-halo bulk_vels rows stacked (track_orbits.py:155,
                    # :199-203): one slice copy for an array (7 ms of Python per 1e4
                    # halos as a loop), the loop for any other sequence
                    nb = len(halo_exists)
                    bulk = np.array(region_bulk_vels[:nb]) if isinstance(
                        region_bulk_vels, np.ndarray) else \
                        np.array([region_bulk_vels[j] for j in range(nb)])
                halo_ids_final = main_branches[-1][progen_exists] if \
                    snapshot_number != snapshot_numbers[-1] else None
                # checkpoint angles now: the next step replaces the engine's state
                groups.append([res, ids_dtype_prev, fetched,
                               (region_positions[hinds], region_radii[hinds], bulk[hinds],
                                halo_ids_[hinds], halo_ids_final, snapshot_number, mode,
                                checkpoint, eng.angles() if checkpoint else None, verbose),
                               dict(layout=checkpoint_layout(eng) if checkpoint else None)])
                if not pipelined:
                    flush()

            progen_exists = halo_exists
    except BaseException as e:
        # the reference had written every group before the failing snapshot: write
        # those whose records are available without re-running anything (a step that
        # asks for a re-plan, a device that does not answer within a few seconds, or a
        # failing query ends this).  No new record fetch is started when fetching is a
        # collective (a sharded engine: the other ranks may already be in the next
        # step's collectives, and an unmatched gather would hang them) or after a
        # KeyboardInterrupt / SystemExit (only fetches already complete are written).
        collective = getattr(eng, 'world', 1) > 1
        interrupted = not isinstance(e, Exception)
        _salvage(groups, eng, out, new_fetches=not (collective or interrupted),
                 timeout=0.0 if interrupted else 10.0)
        raise
    finally:
        for e, v in zip(pulls, saved_pull):
            e.table_pull = v
    flush()

    if verbose:
        print('Finished pericenter detection for all snapshots in {} s\n'.format(
            time.time() - tstart))


def _poll(ready, t_end):
    while not ready():
        if time.time() > t_end:
            return False
        time.sleep(0.002)
    return True


def _salvage(groups, eng, out, timeout=10.0, new_fetches=True):
    """Error path of track_orbits: write pending groups oldest first while each one's
    records can be had without a re-run or an unbounded wait (``new_fetches`` False:
    only groups whose fetch was already issued)."""
    t_end = time.time() + timeout
    try:
        while groups:
            g = groups[0]
            if g[2] is None:
                if not new_fetches:
                    return
                ready = getattr(eng, 'step_ready', None)
                if ready is None or not _poll(lambda: ready(g[0]) is not None, t_end) or \
                        not ready(g[0]):
                    return
                g[2] = eng.fetch_async(g[0], g[1])
            done = getattr(g[2], 'done', None)
            if done is not None and not _poll(done.query, t_end):
                return
            offsets, ids, angles = g[2].wait()
            groups.pop(0)
            save_to_file(out, ids, offsets, angles, *g[3], **g[4])
    except Exception as e:          # the original error propagates; this one is reported
        import warnings
        warnings.warn('track_orbits: pending groups not written after an error (%s: %s)'
                      % (type(e).__name__, e), RuntimeWarning)


class _Fetched:
    """An inline fetch's arrays behind the PendingFetch interface."""

    def __init__(self, arrays):
        self.arrays = arrays

    def wait(self):
        return self.arrays


def checkpoint_layout(eng):
    """Row layout of the engine's checkpoint angles (None: the snapshot's own rows)."""
    f = getattr(eng, 'checkpoint_layout', None)
    return f() if f is not None else None


def read_checkpoint_layout(out):
    f = getattr(out, 'read_checkpoint_layout', None)
    return f() if f is not None else None


def save_to_file(savefile, apsis_ids, apsis_offsets, apsis_angles, region_positions,
                 region_radii, bulk_velocities, halo_ids, halo_ids_final, snapshot_number,
                 mode, checkpoint, angles, verbose, layout=None):
    """Write one snapshot group (+ checkpoint) in the reference layout (:366-397)."""
    out = open_savefile(savefile)
    if verbose:
        print('Saving to file...')
        t0 = time.time()
    out.write_group('snapshot_{}'.format('%0.3d' % snapshot_number),
                    group_datasets(mode, apsis_ids, apsis_offsets, apsis_angles,
                                   region_positions, region_radii, bulk_velocities,
                                   halo_ids, halo_ids_final))
    if checkpoint:
        # a checkpoint in a non-global row layout (presharded ranks) records it, so a
        # resume in another layout is refused instead of mis-assigning angles
        if layout is None:
            out.write_checkpoint(angles)
        else:
            out.write_checkpoint(angles, layout=layout)
    if verbose:
        print('Saved to file ({} s)\n'.format(time.time() - t0))


def initialize_savefile(savefile, mode, box_size, verbose):
    """Create the savefile with its attributes (:354-363)."""
    open_savefile(savefile).initialize(mode, box_size)
    if verbose:
        print('Savefile initialized\n')
