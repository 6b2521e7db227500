"""Host helpers with the reference's names and semantics (orbitanalysis/utils.py).

These are user-side utilities (region cuts in loaders, halo bookkeeping); the
per-particle hot path never calls them — it runs in the HIP kernels.
"""
import numpy as np


def myin1d(a, b, kind=None):
    """Indices of ``a`` whose values are also in ``b``, in ``b``'s order
    (utils.py:4-11; precondition as in the reference: unique values, b ⊆ a)."""
    a = np.asarray(a)
    b = np.asarray(b)
    order = np.argsort(a, kind='stable')
    return order[np.searchsorted(a[order], b)]


def vector_norm(vectors, return_norm=True, return_unit_vectors=False):
    """Row norms and/or unit vectors (utils.py:14-21)."""
    v = np.asarray(vectors)
    mags = np.sqrt(np.einsum('...i,...i', v, v))
    if return_norm and return_unit_vectors:
        return mags, v / mags[:, np.newaxis]
    if return_norm:
        return mags
    if return_unit_vectors:
        return v / mags[:, np.newaxis]
    return None


def recenter_coordinates(position, boxsize):
    """Wrap relative coordinates into [-L/2, L/2] in place, once per dimension
    (utils.py:24-33; a scalar box applies to all three dims)."""
    if isinstance(boxsize, (float, np.floating, int, np.integer)):
        boxsize = boxsize * np.ones(3)
    for d, L in enumerate(boxsize):
        hi = position[:, d] > L / 2
        position[hi, d] -= L
        lo = position[:, d] < -L / 2
        position[lo, d] += L
    return position


def hubble_parameter(z, H0, Omega_m, Omega_L, Omega_k=0):
    """H(z) for a Lambda-CDM background (utils.py:36-39)."""
    return H0 * np.sqrt(Omega_m * (1 + z) ** 3 + Omega_k * (1 + z) ** 2 + Omega_L)
