"""The multi-GPU output stage's device pieces on one GPU (host_share.py): a shared-memory
segment page-locked for device stores, ``oa_place_records`` storing records at their
positions through the mapping's device address (positions outside the buffer dropped
and counted), and ``oa_stream_set_flag`` publishing an epoch once the stream's work is
done.  The collective protocol around them is covered at world 2 / 3 on CPU
(tests/test_sharding.py) and through ``track_orbits`` at world 2 on this GPU
(tests/test_gpu_multi_configs.py)."""
import ctypes
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('ib,with_ang', [(8, True), (4, True), (8, False), (4, False)])
def test_place_records_into_shared_host_buffer(ib, with_ang, tmp_path):
    import torch
    from orbitanalysis_amd import _native as N
    from orbitanalysis_amd.host_share import _Slot
    lib = N.load(require_device=True)
    dev = torch.device('cuda', 0)
    rng = np.random.default_rng(ib)
    cap, n = 1 << 16, 40000
    import os
    from orbitanalysis_amd.host_share import _shm_dir
    slot = _Slot(os.path.join(_shm_dir(), 'oa_test_%d_%d_%d' % (os.getpid(), ib, with_ang)), 2,
                 cap, ib, create=True)
    base = slot.register(lib)
    try:
        idt = np.int64 if ib == 8 else np.int32
        ids = rng.integers(-2 ** 30, 2 ** 30, n).astype(idt)
        ang = rng.integers(-2 ** 15, 2 ** 15, n).astype(np.int16)
        dst = rng.permutation(cap)[:n].astype(np.int64)
        bad = rng.choice(n, 37, replace=False)
        dst[bad[:20]] = cap + rng.integers(0, 100, 20)      # past the buffer
        dst[bad[20:]] = -1 - rng.integers(0, 100, 17)       # before it
        slot.ids[:] = 0
        slot.ang[:] = 0
        t_ids, t_ang, t_dst = (torch.from_numpy(x).to(dev) for x in (ids, ang, dst))
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        # without angles: the 4- / 8-byte values alone (the on-the-fly driver's lists)
        N.check(lib.oa_place_records(ctypes.c_void_p(t_ids.data_ptr()),
                                     ctypes.c_void_p(t_ang.data_ptr()) if with_ang else None,
                                     ctypes.c_void_p(t_dst.data_ptr()), n, ib,
                                     ctypes.c_void_p(base + slot.ids_off),
                                     ctypes.c_void_p(base + slot.ang_off) if with_ang else None, cap,
                                     ctypes.c_void_p(status.data_ptr()), st),
                'oa_place_records')
        flag = slot.flag(1)
        flag[0] = 0
        N.check(lib.oa_stream_set_flag(st, ctypes.c_void_p(flag.ctypes.data), 12345),
                'oa_stream_set_flag')
        t_end = time.time() + 30
        while int(flag[0]) != 12345:                   # the host callback, not a sync
            assert time.time() < t_end, 'the stream flag was never set'
            time.sleep(1e-4)
        torch.cuda.synchronize()
        assert int(status.item()) > 0                  # out-of-range records counted
        good = np.ones(n, bool)
        good[bad] = False
        assert np.array_equal(slot.ids[dst[good]], ids[good])
        if with_ang:
            assert np.array_equal(slot.ang[dst[good]], ang[good])
        else:
            assert not slot.ang.any()
        untouched = np.ones(cap, bool)
        untouched[dst[good]] = False
        assert not slot.ids[untouched].any() and not slot.ang[untouched].any()
    finally:
        slot.release(lib)


@pytest.mark.parametrize('pull', [True, False])
@pytest.mark.parametrize('n', [0, 1, 15, 16, 4097, (1 << 20) + 3, (3 << 20) + 16])
def test_table_upload_by_kernel_pull(n, pull, monkeypatch):
    """engine._upload: with table pulls (the pipelined batch driver) a host table
    reaches the device through a page-locked staging block pulled by oa_copy_bytes
    (16-byte lanes, tail bytes by block 0), blocks reused only after their pull has run,
    so back-to-back uploads keep their own bytes; without, by a DMA."""
    import torch
    from orbitanalysis_amd import engine as E
    from orbitanalysis_amd.engine import _upload
    monkeypatch.setattr(E, '_TABLE_PULL', [pull])
    dev = torch.device('cuda', 0)
    rng = np.random.default_rng(n)
    a = rng.integers(0, 256, n).astype(np.uint8)
    b = rng.integers(0, 256, n).astype(np.uint8)
    want_a = a.copy()
    ta, tb = _upload(a, dev), _upload(b, dev)          # the second may not reuse a's block
    a[:] = 0                                           # the staging block holds its own copy
    torch.cuda.synchronize()
    assert ta.dtype == torch.uint8 and ta.numel() == n
    assert np.array_equal(ta.cpu().numpy(), want_a)
    assert np.array_equal(tb.cpu().numpy(), b)
