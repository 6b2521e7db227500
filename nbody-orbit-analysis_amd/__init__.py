"""orbitanalysis_amd — MI355X-native drop-in for the per-snapshot orbit-tagging hot
path of ``orbitanalysis`` (s-balu/nbody-orbit-analysis).

Public API (same names, signatures, callbacks, errors and output layout as the
reference):

* ``orbitanalysis_amd.track_orbits.track_orbits``            (track_orbits.py:9-244)
* ``orbitanalysis_amd.track_orbits_onthefly.track_orbits``   (track_orbits_onthefly.py:8-58)
* helpers ``region_frame``, ``compare_radial_velocities``, ``calc_angles`` and
  ``utils.myin1d / recenter_coordinates / hubble_parameter``.

Compute runs in hand-written HIP kernels for gfx950 (``csrc/orbit_hip.hip``)
behind a C-ABI shared library (``liborbit_hip.so``, header ``include/orbit_hip.h``)
loaded with ctypes.  There is no CPU fallback: device entry points raise if the
library or a HIP device is missing.
"""
__version__ = '0.1'
