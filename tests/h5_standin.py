"""In-memory, recording stand-in for the part of h5py the reference and this package
use (test infrastructure; h5py is not installed in this image and cannot be).

It models the h5py semantics the savefile contract depends on:
* ``File(name, mode='r')`` with h5py's modes: ``'r'`` / ``'r+'`` need an existing
  file (``FileNotFoundError``), ``'w'`` truncates, ``'w-'`` / ``'x'`` refuse an existing
  file, ``'a'`` opens or creates.  Writes through a ``'r'`` handle raise.
* groups and datasets: ``create_group`` / ``create_dataset`` refuse an existing name
  (``ValueError``, as h5py), ``keys()`` in HDF5's default name order (lexicographic),
  ``hf['g']['d'][:]`` / ``hf['g/d']``, ``len``, ``dtype``, ``shape``;
* attributes: ``attrs[k] = v`` stores NumPy's array of ``v`` (a ``str`` stays a
  ``str``, as h5py reads variable-length strings back), ``in``, ``get``.
Every file keeps its nodes' creation order, and the module logs each open
``(path, mode)``: ``tree()`` / ``opens()`` are what the f2 fixtures record.

Use: ``sys.modules['h5py'] = h5_standin`` (``install()``), ``reset()`` between cases.
"""
import sys
import types

import numpy as np

FILES = {}        # path -> _Node (the file's root group)
OPENS = []        # (path, mode) of every File() call, in order


class _Attrs:
    def __init__(self, node):
        self._node = node
        self._d = {}

    def __setitem__(self, k, v):
        self._node._check_writable()
        self._d[k] = v if isinstance(v, str) else np.asarray(v)

    def __getitem__(self, k):
        return self._d[k]

    def __contains__(self, k):
        return k in self._d

    def __iter__(self):
        return iter(sorted(self._d))

    def __len__(self):
        return len(self._d)

    def get(self, k, default=None):
        return self._d.get(k, default)

    def keys(self):
        return sorted(self._d)

    def items(self):
        return [(k, self._d[k]) for k in sorted(self._d)]


class _Dataset:
    def __init__(self, data):
        self._a = np.array(data)          # a copy, as a write to the file is
        if self._a.dtype == object:
            raise TypeError('Object dtype dtype(\'O\') has no native HDF5 equivalent')

    @property
    def dtype(self):
        return self._a.dtype

    @property
    def shape(self):
        return self._a.shape

    def __len__(self):
        return len(self._a)

    def __getitem__(self, k):
        return np.array(self._a[k])

    def __array__(self, dtype=None, copy=None):
        return self._a if dtype is None else self._a.astype(dtype)


class _Node:
    """A group (the root group is the file)."""

    def __init__(self, root=None):
        self._root = root if root is not None else self
        self._children = {}
        self._order = []                  # creation order
        self.attrs = _Attrs(self)
        self._writable = True             # root only: set per open handle

    def _check_writable(self):
        if not self._root._writable:
            raise ValueError('Unable to create (no write intent on file)')

    def _new(self, name, obj):
        self._check_writable()
        if '/' in name:
            head, rest = name.split('/', 1)
            return self[head]._new(rest, obj)
        if name in self._children:
            raise ValueError('Unable to create %r (name already exists)' % name)
        self._children[name] = obj
        self._order.append(name)
        return obj

    def create_group(self, name):
        return self._new(name, _Node(self._root))

    def create_dataset(self, name, shape=None, dtype=None, data=None):
        if data is None:
            data = np.zeros(shape, dtype=dtype)
        elif dtype is not None:
            data = np.asarray(data, dtype=dtype)
        return self._new(name, _Dataset(data))

    def __getitem__(self, name):
        node = self
        for part in name.strip('/').split('/'):
            if part not in node._children:
                raise KeyError("Unable to open object (object '%s' doesn't exist)" % part)
            node = node._children[part]
        return node

    def __contains__(self, name):
        try:
            self[name]
        except KeyError:
            return False
        return True

    def keys(self):
        return sorted(self._children)

    def __iter__(self):
        return iter(self.keys())

    def __len__(self):
        return len(self._children)

    def items(self):
        return [(k, self._children[k]) for k in self.keys()]


class File:
    """``h5py.File``: a handle on the in-memory file ``name``."""

    def __init__(self, name, mode='r'):
        name = str(name)
        OPENS.append((name, mode))
        exists = name in FILES
        if mode in ('r', 'r+'):
            if not exists:
                raise FileNotFoundError(
                    "[Errno 2] Unable to synchronously open file (unable to open file: "
                    "name = '%s')" % name)
        elif mode == 'w':
            FILES[name] = _Node()
        elif mode in ('w-', 'x'):
            if exists:
                raise FileExistsError('Unable to synchronously create file (file exists)')
            FILES[name] = _Node()
        elif mode == 'a':
            if not exists:
                FILES[name] = _Node()
        else:
            raise ValueError('Invalid mode; must be one of r, r+, w, w-, x, a')
        self._node = FILES[name]
        self.filename = name
        self.mode = 'r' if mode == 'r' else 'r+'
        self._node._writable = mode != 'r'
        self.attrs = self._node.attrs

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def close(self):
        self._node._writable = True

    def create_group(self, name):
        return self._node.create_group(name)

    def create_dataset(self, name, shape=None, dtype=None, data=None):
        return self._node.create_dataset(name, shape=shape, dtype=dtype, data=data)

    def __getitem__(self, name):
        return self._node[name]

    def __contains__(self, name):
        return name in self._node

    def keys(self):
        return self._node.keys()

    def __iter__(self):
        return iter(self._node.keys())

    def __len__(self):
        return len(self._node)

    def items(self):
        return self._node.items()


def reset():
    FILES.clear()
    OPENS.clear()


def install():
    """Make ``import h5py`` resolve to this module; returns the previous entry."""
    prev = sys.modules.get('h5py')
    mod = types.ModuleType('h5py')
    mod.File = File
    mod.__doc__ = __doc__
    mod._standin = sys.modules[__name__]
    sys.modules['h5py'] = mod
    return prev


def uninstall(prev):
    if prev is None:
        sys.modules.pop('h5py', None)
    else:
        sys.modules['h5py'] = prev


def opens(prefix=''):
    """The logged opens of files under ``prefix``, paths relative to it."""
    return [(p[len(prefix):], m) for p, m in OPENS if p.startswith(prefix)]


def _walk(node, path, order, arrays):
    for name in node._order:
        child = node._children[name]
        p = path + name
        if isinstance(child, _Node):
            order.append(('group', p))
            _walk(child, p + '/', order, arrays)
        else:
            order.append(('dataset', p))
            arrays[p] = np.array(child._a)


def tree(path):
    """One file as data: {'attrs': {name: value}, 'order': [(kind, path)] in creation
    order, 'arrays': {dataset path: array}}."""
    node = FILES[path]
    order, arrays = [], {}
    _walk(node, '', order, arrays)
    return {'attrs': {k: node.attrs[k] for k in node.attrs.keys()}, 'order': order,
            'arrays': arrays}


def files(prefix=''):
    """Names (relative to ``prefix``) of the in-memory files under it, sorted."""
    return sorted(p[len(prefix):] for p in FILES if p.startswith(prefix))
