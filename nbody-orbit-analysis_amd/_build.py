"""Build liborbit_hip.so (hipcc, gfx950) in-tree.  Used by __graft_entry__.build().

Two source files: ``orbit_hip.hip`` (the per-snapshot path) and ``orbit_post.hip``
(SURVEY §8(f) rows f3/f4).  ``orbit_hip.hip`` is compiled as four units in parallel
(OA_TU = -1: the C ABI and the helper kernels; 1, 2, 3: the step kernels of one dtype
plan each -- their template instantiations are most of the device compile time).  Each
object is rebuilt only when its source (or a header) changed, then all are linked into
one shared library."""
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
UNITS = (-1, 1, 2, 3)           # OA_TU units of orbit_hip.hip


def _obj(src, tu=None):
    tag = '' if tu is None else '.tu%s' % str(tu).replace('-', 'm')
    return os.path.join(PKG, 'csrc', os.path.basename(src) + tag + '.o')


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

    def compile_one(job):
        src, tu = job
        obj = _obj(src, tu)
        hdrs = HDRS if src.endswith('orbit_post.hip') else HDRS[:1]
        if force or _newer(obj, [src] + hdrs + [__file__]):
            extra = [] if tu is None else ['-DOA_TU=%d' % tu]
            cmd = [HIPCC] + FLAGS + extra + ['-c', '-o', obj + '.tmp', src]
            if verbose:
                print(' '.join(cmd), flush=True)
            subprocess.run(cmd, check=True)
            os.replace(obj + '.tmp', obj)
        return obj

    jobs = [(SRCS[0], tu) for tu in UNITS] + [(SRCS[1], None)]
    with ThreadPoolExecutor(len(jobs)) as ex:
        objs = list(ex.map(compile_one, jobs))
    cmd = [HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', LIB + '.tmp'] + objs
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + '.tmp', LIB)
    return LIB


if __name__ == '__main__':
    build(force=True)
