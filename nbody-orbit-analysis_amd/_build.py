"""Build liborbit_hip.so (hipcc, gfx950) in-tree.  Used by __graft_entry__.build()."""
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRC = os.path.join(PKG, 'csrc', 'orbit_hip.hip')
HDR = os.path.join(ROOT, 'include', 'orbit_hip.h')
LIB = os.path.join(PKG, 'liborbit_hip.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-shared',
         # the reference's NumPy arithmetic rounds every product and sum: no FMA
         '-ffp-contract=off', '-fno-fast-math',
         # the work-counter atomics are issued a loop trip before their results are
         # used: the atomic optimizer's wave-reduction rewrite would wait on them at once
         '-mllvm', '-amdgpu-atomic-optimizer-strategy=None',
         '-I' + os.path.join(ROOT, 'include')]


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in (SRC, HDR, __file__))


def build(force=False, verbose=True):
    if not force and not stale():
        return LIB
    cmd = [HIPCC] + FLAGS + ['-o', LIB + '.tmp', SRC]
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + '.tmp', LIB)
    return LIB


if __name__ == '__main__':
    build(force=True)
