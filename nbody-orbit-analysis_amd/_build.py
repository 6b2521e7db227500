"""Build liborbit_hip.so (hipcc, gfx950) in-tree.  Used by __graft_entry__.build().

Two translation units: ``orbit_hip.hip`` (the per-snapshot path) and
``orbit_post.hip``; each is compiled to an object only
when it (or a header) changed, then both are linked into one shared library."""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRCS = [os.path.join(PKG, 'csrc', f) for f in ('orbit_hip.hip', 'orbit_post.hip')]
HDRS = [os.path.join(ROOT, 'include', f) for f in ('orbit_hip.h', 'orbit_post.h')]
LIB = os.path.join(PKG, 'liborbit_hip.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC',
         # the reference's NumPy arithmetic rounds every product and sum: no FMA
         '-ffp-contract=off', '-fno-fast-math',
         # the work-counter atomics are issued a loop trip before their results are
         # used: the atomic optimizer's wave-reduction rewrite would wait on them at once
         '-mllvm', '-amdgpu-atomic-optimizer-strategy=None',
         '-I' + os.path.join(ROOT, 'include')]


def _obj(src):
    return os.path.join(PKG, 'csrc', os.path.basename(src) + '.o')


def _newer(path, deps):
    if not os.path.exists(path):
        return True
    t = os.path.getmtime(path)
    return any(os.path.getmtime(p) > t for p in deps)


def stale():
    return _newer(LIB, SRCS + HDRS + [__file__])


def build(force=False, verbose=True):
    if not force and not stale():
        return LIB

    def compile_one(src):
        obj = _obj(src)
        hdrs = HDRS if src.endswith('orbit_post.hip') else HDRS[:1]
        if force or _newer(obj, [src] + hdrs + [__file__]):
            cmd = [HIPCC] + FLAGS + ['-c', '-o', obj + '.tmp', src]
            if verbose:
                print(' '.join(cmd), flush=True)
            subprocess.run(cmd, check=True)
            os.replace(obj + '.tmp', obj)
        return _obj(src)

    with ThreadPoolExecutor(len(SRCS)) as ex:
        objs = list(ex.map(compile_one, SRCS))
    cmd = [HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', LIB + '.tmp'] + objs
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + '.tmp', LIB)
    return LIB


if __name__ == '__main__':
    build(force=True)
