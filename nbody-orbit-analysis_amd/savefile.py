"""Output writers with the reference's savefile layout (track_orbits.py:354-397).

* ``HDF5Savefile``  — h5py, byte-for-byte the reference layout: file attrs ``mode``
  (+ ``box_size``), one group ``snapshot_%03d`` per compared snapshot holding
  ``region_offsets``, ``{peri|apo}center_IDs``, ``angles`` (f16), ``halo_IDs``,
  ``final_descendant_IDs`` (not at the last snapshot), ``region_radii``,
  ``region_positions``, ``bulk_velocities``; checkpoint file ``<savefile>.checkpoint``
  with ``angles``.
* ``MemorySavefile`` — the same layout in memory (tests; h5py is not installed in
  this image).

``open_savefile`` accepts a path (HDF5; raises ImportError without h5py, as the
reference does at import time) or any object with this interface.
"""
import numpy as np


class MemorySavefile:
    def __init__(self):
        self.attrs = {}
        self.groups = {}
        self.checkpoint = None
        self.checkpoint_layout = None

    def initialize(self, mode, box_size):
        self.attrs = {'mode': mode}
        if box_size is not None:
            self.attrs['box_size'] = box_size
        self.groups = {}

    def write_group(self, name, datasets):
        if name in self.groups:
            raise ValueError('group %s exists' % name)
        self.groups[name] = {k: np.asarray(v) for k, v in datasets.items()}

    def write_checkpoint(self, angles, layout=None):
        self.checkpoint = np.asarray(angles)
        self.checkpoint_layout = layout

    def last_snapshot_number(self):
        return int(sorted(self.groups)[-1].split('_')[1])

    def read_checkpoint(self):
        return self.checkpoint

    def read_checkpoint_layout(self):
        return self.checkpoint_layout

    def write_file(self, snapshot_number, datasets, attrs):
        """On-the-fly driver: one 'file' per snapshot (track_orbits_onthefly.py:229)."""
        self.files = getattr(self, 'files', {})
        self.files[int(snapshot_number)] = ({k: np.asarray(v) for k, v in datasets.items()},
                                            dict(attrs))


class HDF5Savefile:
    def __init__(self, path):
        import h5py  # noqa: F401  (ImportError like the reference's module import)
        self.path = path

    def initialize(self, mode, box_size):
        import h5py
        with h5py.File(self.path, 'w') as hf:
            hf.attrs['mode'] = mode
            if box_size is not None:
                hf.attrs['box_size'] = box_size

    def write_group(self, name, datasets):
        import h5py
        with h5py.File(self.path, 'r+') as hf:
            g = hf.create_group(name)
            for k, v in datasets.items():
                g.create_dataset(k, data=v)

    def write_checkpoint(self, angles, layout=None):
        import h5py
        with h5py.File(self.path + '.checkpoint', 'w') as hf:
            hf.create_dataset('angles', data=angles)
            if layout is not None:            # only sharded runs with presharded loaders
                hf.attrs['row_layout'] = layout

    def last_snapshot_number(self):
        import h5py
        with h5py.File(self.path, 'r') as hf:
            return int(list(hf.keys())[-1].split('_')[1])

    def read_checkpoint(self):
        """The checkpoint angles (:229-232); the row layout attribute is read in the
        same open, as the reference opens the checkpoint once."""
        import h5py
        with h5py.File(self.path + '.checkpoint', 'r') as hf:
            v = hf.attrs.get('row_layout')
            self._layout = None if v is None else (v.decode() if isinstance(v, bytes) else str(v))
            return hf['angles'][:]

    def read_checkpoint_layout(self):
        if not hasattr(self, '_layout'):
            self.read_checkpoint()
        return self._layout


class RankSink:
    """Savefile stand-in for ranks other than 0 in a sharded run: writes are dropped
    (rank 0 writes the file); resume reads go to the real savefile."""

    def __init__(self, source=None):
        self.source = source

    def initialize(self, mode, box_size):
        pass

    def write_group(self, name, datasets):
        pass

    def write_checkpoint(self, angles, layout=None):
        pass

    def last_snapshot_number(self):
        return self.source.last_snapshot_number()

    def read_checkpoint(self):
        return self.source.read_checkpoint()

    def read_checkpoint_layout(self):
        f = getattr(self.source, 'read_checkpoint_layout', None)
        return f() if f is not None else None


def open_savefile(savefile):
    if isinstance(savefile, (str, bytes)) or hasattr(savefile, '__fspath__'):
        return HDF5Savefile(str(savefile))
    for m in ('initialize', 'write_group', 'write_checkpoint', 'last_snapshot_number',
              'read_checkpoint'):
        if not hasattr(savefile, m):
            raise TypeError('savefile must be a path or a savefile object (missing %s)' % m)
    return savefile


def group_datasets(mode, apsis_ids, apsis_offsets, apsis_angles, region_positions,
                   region_radii, bulk_velocities, halo_ids, halo_ids_final):
    """Dataset dict of one snapshot group, in the reference's creation order (:379-388)."""
    d = {'region_offsets': apsis_offsets,
         '{}er_IDs'.format(mode[:-3]): apsis_ids,
         'angles': apsis_angles,
         'halo_IDs': halo_ids}
    if halo_ids_final is not None:
        d['final_descendant_IDs'] = halo_ids_final
    d['region_radii'] = region_radii
    d['region_positions'] = region_positions
    d['bulk_velocities'] = bulk_velocities
    return d
