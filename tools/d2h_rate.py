"""D2H rate of device -> page-locked host copies on this box (why the batch driver's
record fetch runs at ~20-26 GB/s): torch's pinned tensors
(hipHostMalloc default flags: coherent) against hipHostMalloc(..., NonCoherent), one
copy alone and back to back, for the sizes one snapshot's apsis records take.

  python tools/d2h_rate.py
"""
import ctypes
import json
import time

import torch

HIP_NONCOHERENT = 0x80000000
HIP_D2H = 2


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    hip = ctypes.CDLL('libamdhip64.so')
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    out = []
    for mb in (4, 16, 64, 100, 256):
        n = mb << 20
        src = torch.empty(n, dtype=torch.uint8, device=dev).fill_(7)
        res = {'MiB': mb}
        pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        for rep in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            pin.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
        res['torch_pinned_GBs'] = n / dt / 1e9
        p = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(p), n, HIP_NONCOHERENT) == 0
        st = torch.cuda.current_stream().cuda_stream
        for rep in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            assert hip.hipMemcpyAsync(p, src.data_ptr(), n, HIP_D2H, st) == 0
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
        res['noncoherent_GBs'] = n / dt / 1e9
        # two halves on two streams at once (two DMA engines?)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for rep in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            with torch.cuda.stream(s1):
                pin[:n // 2].copy_(src[:n // 2], non_blocking=True)
            with torch.cuda.stream(s2):
                pin[n // 2:].copy_(src[n // 2:], non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
        res['torch_pinned_2streams_GBs'] = n / dt / 1e9
        # H2D for comparison
        for rep in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            src.copy_(pin, non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
        res['h2d_pinned_GBs'] = n / dt / 1e9
        hip.hipHostFree(p)
        out.append(res)
        print(json.dumps(res), flush=True)


if __name__ == '__main__' and len(__import__('sys').argv) == 1:
    main()


def alloc_pattern():
    """The batch driver's fetch pattern: per snapshot a pinned block of a slightly
    different size (engine._pinned rounds to 4 MiB), filled by one D2H, freed a
    snapshot later.  Times the allocation and the copy separately."""
    import numpy as np
    from orbitanalysis_amd.engine import _pinned
    dev = torch.device('cuda', 0)
    src = torch.empty(12_000_000, dtype=torch.int64, device=dev).fill_(3)
    rng = np.random.default_rng(0)
    keep = None
    for it in range(8):
        n = int(10_000_000 + rng.integers(-200_000, 200_000))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h = _pinned(n, torch.int64)
        t1 = time.perf_counter()
        h.copy_(src[:n], non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({'pattern_iter': it, 'n': n, 'alloc_ms': (t1 - t0) * 1e3,
                          'copy_ms': (t2 - t1) * 1e3, 'GBs': n * 8 / (t2 - t1) / 1e9}), flush=True)
        keep = h                     # freed at the next iteration, as the driver's
    del keep


if __name__ == '__main__' and 'pattern' in __import__('sys').argv:
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import orbitanalysis_amd  # noqa: F401
    alloc_pattern()


def issue_cost():
    """Host time to ISSUE one ~100 MB D2H (as fetch_async does: on a side stream after an
    event) against the time until it completes: if the issue itself takes the copy's
    duration, the copy blocks the host and cannot overlap the next snapshot."""
    import numpy as np
    from orbitanalysis_amd.engine import _pinned
    dev = torch.device('cuda', 0)
    hip = ctypes.CDLL('libamdhip64.so')
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    hip.hipMemcpyDtoHAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_void_p]
    n = 10_000_000
    src = torch.empty(n, dtype=torch.int64, device=dev).fill_(3)
    busy = torch.empty(1 << 26, dtype=torch.float32, device=dev)
    cs = torch.cuda.Stream(device=dev)
    h = _pinned(n, torch.int64)
    for mode in ('torch_side', 'torch_side_busy', 'hip_side', 'hip_side_busy', 'torch_cur'):
        for rep in range(4):
            torch.cuda.synchronize()
            if mode.endswith('busy'):
                for _ in range(20):
                    busy.mul_(1.0001)          # ~ms of compute queued on the current stream
            t0 = time.perf_counter()
            if mode.startswith('torch_side'):
                with torch.cuda.stream(cs):
                    h.copy_(src, non_blocking=True)
            elif mode.startswith('hip_side'):
                assert hip.hipMemcpyAsync(h.data_ptr(), src.data_ptr(), n * 8, HIP_D2H,
                                          cs.cuda_stream) == 0
            else:
                h.copy_(src, non_blocking=True)
            t1 = time.perf_counter()
            cs.synchronize()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        print(json.dumps({'mode': mode, 'issue_ms': (t1 - t0) * 1e3, 'done_ms': (t2 - t0) * 1e3}),
              flush=True)


if __name__ == '__main__' and 'issue' in __import__('sys').argv:
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import orbitanalysis_amd  # noqa: F401
    issue_cost()
