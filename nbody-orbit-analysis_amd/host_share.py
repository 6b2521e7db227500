"""Multi-GPU output stage: every rank stores its own apsis records straight into one
page-locked host buffer that all ranks map (the reference's single
writer is track_orbits.py:189-227 with save_to_file :366-397).

Before this stage, each rank's records were gathered to rank 0's GPU and crossed PCIe
over rank 0's link alone: at configs[3] on 8 GPUs, ~65 MB per snapshot through one
link (~1.2 ms) against ~0.2 ms of kernel per rank.  Here:

1. the (world, halo slot) record-count matrix is all-gathered (8 B per slot per rank);
2. every rank computes its own records' final positions: with a presharded reader a
   halo's records from rank r follow those of ranks < r (a count scan); with stripes,
   the ranks' records of a halo interleave by global previous row, so each rank marks
   its rows in a bitmap of the previous snapshot, one all-reduce (disjoint bits, so a
   byte sum is an OR) gives every rank every row's rank among the records;
3. each rank's placement kernel (``oa_place_records``) stores its records at those
   positions through the device address of the shared mapping (zero-copy, over its own
   PCIe link), and a host callback on the rank's stream publishes the fetch's epoch in
   the buffer's header when the stores are done (``oa_stream_set_flag``);
4. rank 0 waits for every rank's epoch and hands the buffer to the savefile writer.

Buffers are POSIX shared-memory files (``/dev/shm``) in a small pool of slots chosen by
rank 0 (a slot stays busy while the arrays it handed out are alive; a new or larger one
is created when none fits) and announced with one broadcast per fetch.  Each slot is
unlinked once every rank has mapped it.  CPU ranks (gloo tests) run the same protocol
with numpy stores.
"""
import atexit
import mmap
import os
import secrets
import time
import weakref

import numpy as np
import torch

HDR = 64                          # header bytes per rank (one cache line each)
_POP8 = np.array([bin(i).count('1') for i in range(256)], dtype=np.int64)


def _shm_dir():
    return '/dev/shm' if os.path.isdir('/dev/shm') else os.environ.get('TMPDIR', '/tmp')


def _pow2(n, lo=1 << 20):
    n = max(int(n), lo)
    return 1 << (n - 1).bit_length()


class _Slot:
    """One shared-memory segment: [world x HDR header][cap IDs][cap f16 angles]."""

    def __init__(self, path, world, cap, ib, create):
        self.path, self.cap, self.ib = path, int(cap), int(ib)
        self.hdr_bytes = -(-world * HDR // 4096) * 4096
        ids_bytes = -(-self.cap * self.ib // 4096) * 4096
        self.nbytes = self.hdr_bytes + ids_bytes + -(-self.cap * 2 // 4096) * 4096
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(path, flags, 0o600)
        try:
            if create:
                os.ftruncate(fd, self.nbytes)
            self.mm = mmap.mmap(fd, self.nbytes, mmap.MAP_SHARED,
                                mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self.linked = create              # rank 0 unlinks it once every rank mapped it
        buf = np.frombuffer(self.mm, dtype=np.uint8)
        self.base = buf.ctypes.data
        self.hdr = buf[:self.hdr_bytes].view(np.int64)
        o = self.hdr_bytes
        # ib = 0: a slot of 16-bit values alone (checkpoint angles)
        self.ids = buf[o:o + self.cap * self.ib].view(np.int64 if self.ib == 8 else np.int32)
        self.ang_off = o + ids_bytes
        self.ang = buf[self.ang_off:self.ang_off + 2 * self.cap].view(np.int16)
        self.ids_off = o
        self.dev = None                   # device address of the mapping (registered)
        self.busy = 0                     # rank 0: arrays handed out and still alive

    def flag(self, rank):
        return self.hdr[rank * (HDR // 8):rank * (HDR // 8) + 1]

    def register(self, lib):
        if self.dev is None:
            import ctypes
            from . import _native as N
            p = ctypes.c_void_p()
            N.check(lib.oa_host_register(ctypes.c_void_p(self.base), self.nbytes,
                                         ctypes.byref(p)), 'oa_host_register')
            self.dev = p.value
        return self.dev

    def release(self, lib):
        if self.dev is not None and lib is not None:
            import ctypes
            lib.oa_host_unregister(ctypes.c_void_p(self.base))
            self.dev = None
        if self.linked:
            try:
                os.unlink(self.path)
            except OSError:
                pass
            self.linked = False


class StageFetch:
    """One fetch's records on their way into the shared buffer (``ShardedEngine``'s
    fetch_async result).  ``done.query()`` (the error path's poll) is true once this
    rank's stores are done and, on rank 0, every rank's epoch is in the header."""

    def __init__(self, stage, slot, epoch, event, off, total, ids_dtype, root, moved):
        self.stage, self.slot, self.epoch, self.event = stage, slot, epoch, event
        self.off, self.total, self.ids_dtype, self.root = off, total, ids_dtype, root
        self.moved = moved                # bytes this rank stored into the buffer
        self.done = self

    def _mine(self):
        return self.event is None or self.event.query()

    def query(self):
        if not self._mine():
            return False
        if not self.root:
            return True
        return all(int(self.slot.flag(r)[0]) == self.epoch for r in range(self.stage.world))

    def wait(self):
        from .engine import ids_as
        dt = np.dtype(self.ids_dtype)
        if self.event is not None:
            self.event.synchronize()
        if self.stage.status is not None and int(self.stage.status.item()):
            raise RuntimeError('oa_place_records: %d records fell outside the output'
                               % int(self.stage.status.item()))
        if not self.root:
            return np.zeros(len(self.off), np.int64), np.zeros(0, dt), np.zeros(0, np.float16)
        t_end = time.time() + self.stage.timeout
        while not self.query():
            if time.time() > t_end:
                raise RuntimeError('sharded records: a rank did not store its records within '
                                   '%.0f s' % self.stage.timeout)
            time.sleep(2e-5)
        slot = self.slot
        if slot.linked:                   # every rank has it mapped now
            self.stage._unlink(slot)
        n = self.total
        slot.busy -= 1                    # in flight since _choose
        if n == 0:
            return self.off, np.zeros(0, dt), np.zeros(0, np.float16)
        # the arrays are exported by two ctypes holders over the mapping: every array or
        # view derived from them keeps its holder alive, and the slot is reused only once
        # both holders are gone (the savefile has dropped the records)
        import ctypes
        hi = (ctypes.c_char * (n * slot.ib)).from_buffer(slot.mm, slot.ids_off)
        ha = (ctypes.c_char * (2 * n)).from_buffer(slot.mm, slot.ang_off)
        slot.busy += 2
        for h in (hi, ha):
            weakref.finalize(h, self.stage._free, slot)
        ids_v = np.frombuffer(hi, dtype=slot.ids.dtype)
        ang_v = np.frombuffer(ha, dtype=np.float16)
        return self.off, ids_as(ids_v, dt), ang_v


class SharedRecordStage:
    """The shared output buffers of one ``ShardedEngine`` (see module docstring)."""

    def __init__(self, group, rank, world, root=0, timeout=None):
        self.group, self.rank, self.world, self.root = group, rank, world, root
        self.slots = {}                   # slot index -> _Slot (this rank's mappings)
        self.gens = {}                    # slot index -> generation mapped here
        self.epoch = 0
        self.name = None                  # (pid, nonce) of rank 0's files
        self.status = None                # device word: records outside the output
        self.timeout = float(timeout if timeout is not None else
                             os.environ.get('ORBIT_FETCH_TIMEOUT', 600))
        self.lib = None
        atexit.register(self.close)

    # ------------------------------------------------------------ slots (rank 0 decides)
    def _path(self, slot, gen):
        pid, nonce = self.name
        return os.path.join(_shm_dir(), 'oa_rec_%d_%d_%d_%d' % (pid, nonce, slot, gen))

    def _free(self, slot):
        slot.busy -= 1

    def _unlink(self, slot):
        try:
            os.unlink(slot.path)
        except OSError:
            pass
        slot.linked = False

    def _choose(self, total, ib):
        """Rank 0: (slot, generation, capacity) for this fetch; creates the file.  The
        slot is busy from here until this fetch's arrays are dropped (a fetch in flight
        counts once, each handed-out array once)."""
        fit = [k for k, s in self.slots.items() if s.busy == 0 and s.ib == ib and s.cap >= total]
        if fit:
            k = min(fit, key=lambda k: self.slots[k].cap)
        else:
            free = [k for k, s in self.slots.items() if s.busy == 0]
            k = free[0] if free else len(self.slots)
            self._map(k, self.gens.get(k, -1) + 1, _pow2(total), ib, create=True)
        self.slots[k].busy += 1
        return k, self.gens[k], self.slots[k].cap

    def _map(self, k, gen, cap, ib, create):
        old = self.slots.get(k)
        if old is not None:
            old.release(self.lib)
        self.slots[k] = _Slot(self._path(k, gen), self.world, cap, ib, create)
        self.gens[k] = gen

    def _agree(self, total, ib, comm_dev):
        """One broadcast from rank 0: the slot this fetch stores into (opened here)."""
        import torch.distributed as dist
        if self.rank == self.root:
            if self.name is None:
                self.name = (os.getpid(), secrets.randbits(31))
            k, gen, cap = self._choose(total, ib)
            msg = [k, gen, cap, ib, self.name[0], self.name[1]]
        else:
            msg = [0] * 6
        t = torch.tensor(msg, dtype=torch.int64).to(comm_dev)
        src = dist.get_global_rank(self.group, self.root) if self.group is not None else self.root
        dist.broadcast(t, src=src, group=self.group)
        k, gen, cap, ib, pid, nonce = (int(x) for x in t.cpu())
        if self.rank != self.root:
            self.name = (pid, nonce)
            if self.gens.get(k) != gen:
                self._map(k, gen, cap, ib, create=False)
        return self.slots[k]

    # ------------------------------------------------------------ one fetch
    def fetch(self, lib, side, done, offs, a_ids, a_ang, total_local, C_local, n_slots,
              ids_dtype, rows=None, n_rows=None, comm_dev=None, profile=None):
        """Place this rank's ``total_local`` records (device tensors ``a_ids``,
        ``a_ang``, which may be None: IDs alone; per-slot counts ``C_local``) into the
        shared buffer.  ``rows``: the records' global previous rows (stripe layout), else
        presharded.  Returns a ``StageFetch``."""
        import torch.distributed as dist
        self.lib = lib
        self.epoch += 1
        epoch = self.epoch
        dev = a_ids.device
        S = n_slots
        on_gpu = dev.type == 'cuda'
        # 1. the count matrix on every rank (one all-gather)
        cl = C_local.to(torch.int64).reshape(S).to(comm_dev)
        allc = torch.empty(self.world * S, dtype=torch.int64, device=comm_dev)
        dist.all_gather_into_tensor(allc, cl.contiguous(), group=self.group)
        C = allc.view(self.world, S)
        Ch = C.cpu().numpy()
        tot_slot = Ch.sum(0)
        total = int(tot_slot.sum())
        off = np.zeros(S + 1, np.int64)
        np.cumsum(tot_slot, out=off[1:])
        ib = a_ids.element_size()
        # 2. the slot (rank 0 chooses, one broadcast)
        slot = self._agree(total, ib, comm_dev)
        n = int(total_local)
        t0 = time.perf_counter() if profile is not None else 0.0
        # 3. this rank's records' positions (the counts are checked on the host first: a
        # count matrix that disagrees with the record total would place records outside
        # their runs)
        loc_h = Ch[self.rank]
        if (Ch < 0).any() or int(loc_h.sum()) != n or n > slot.cap or total > slot.cap:
            raise RuntimeError('sharded records: rank %d holds %d records but its per-halo '
                               'counts sum to %d (min count %d, output capacity %d)'
                               % (self.rank, n, int(loc_h.sum()), int(Ch.min(initial=0)),
                                  slot.cap))
        if rows is None:
            before_h = Ch[:self.rank].sum(0)
            D_h = off[:S] + before_h - (np.cumsum(loc_h) - loc_h)
            dst = torch.arange(n, dtype=torch.int64, device=dev) + \
                torch.repeat_interleave(torch.from_numpy(D_h).to(dev),
                                        torch.from_numpy(loc_h).to(dev), output_size=n) if n else \
                torch.zeros(0, dtype=torch.int64, device=dev)
        else:
            dst = self._rank_by_row(rows[:n].to(dev).to(torch.int64), int(n_rows), comm_dev)
        # 4. the stores, and this rank's epoch in the header when they are done
        if on_gpu:
            import ctypes
            if self.status is None:
                self.status = torch.zeros(1, dtype=torch.int32, device=dev)
            base = slot.register(lib)
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            from . import _native as N
            has_ang = a_ang is not None
            N.check(lib.oa_place_records(
                ctypes.c_void_p(a_ids.data_ptr()),
                ctypes.c_void_p(a_ang.data_ptr()) if has_ang else None,
                ctypes.c_void_p(dst.data_ptr()), n, ib,
                ctypes.c_void_p(base + slot.ids_off),
                ctypes.c_void_p(base + slot.ang_off) if has_ang else None,
                slot.cap, ctypes.c_void_p(self.status.data_ptr()), st), 'oa_place_records')
            flag = slot.flag(self.rank)
            N.check(lib.oa_stream_set_flag(st, ctypes.c_void_p(flag.ctypes.data), epoch),
                    'oa_stream_set_flag')
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
        else:
            if n:
                d = dst.numpy()
                if d.min() < 0 or d.max() >= slot.cap:
                    raise RuntimeError('sharded records: positions outside the output')
                slot.ids[d] = a_ids[:n].numpy().view(slot.ids.dtype)
                if a_ang is not None:
                    slot.ang[d] = a_ang[:n].numpy().view(np.int16)
            slot.flag(self.rank)[0] = epoch
            ev = None
        if profile is not None:
            if on_gpu:
                torch.cuda.current_stream(dev).synchronize()
            profile.update(records=total, own_records=n, place_ms=(time.perf_counter() - t0) * 1e3,
                           bytes_moved=n * (ib + (2 if a_ang is not None else 0)),
                           layout='stripes' if rows is not None
                           else 'presharded')
        return StageFetch(self, slot, epoch, ev, off, total, ids_dtype,
                          self.rank == self.root, n * (ib + (2 if a_ang is not None else 0)))

    def place_rows(self, lib, vals, rows, n_total, comm_dev):
        """Checkpoint angles (track_orbits.py:390-394): this rank's f16 bits ``vals`` at
        their global snapshot rows ``rows`` (every row held by exactly one rank) into a
        shared buffer of ``n_total`` angles (a slot without an ID region); returns the
        float16 array on rank 0 (a view of the buffer, the slot busy while it lives),
        None elsewhere.  Synchronous: each rank's stores are done before its epoch is
        published."""
        import ctypes
        self.lib = lib
        self.epoch += 1
        epoch = self.epoch
        dev = vals.device
        slot = self._agree(int(n_total), 0, comm_dev)
        n = int(vals.shape[0])
        if dev.type == 'cuda':
            from . import _native as N
            if self.status is None:
                self.status = torch.zeros(1, dtype=torch.int32, device=dev)
            base = slot.register(lib)
            v16 = vals.to(torch.int16).contiguous()
            r64 = rows.to(dev).to(torch.int64).contiguous()
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            N.check(lib.oa_place_records(None, ctypes.c_void_p(v16.data_ptr()),
                                         ctypes.c_void_p(r64.data_ptr()), n, 8, None,
                                         ctypes.c_void_p(base + slot.ang_off), slot.cap,
                                         ctypes.c_void_p(self.status.data_ptr()), st),
                    'oa_place_records')
            torch.cuda.current_stream(dev).synchronize()
            if int(self.status.item()):
                raise RuntimeError('checkpoint angles: rows outside the snapshot')
        elif n:
            r = rows.numpy().astype(np.int64)
            if r.min() < 0 or r.max() >= slot.cap:
                raise RuntimeError('checkpoint angles: rows outside the snapshot')
            slot.ang[r] = vals.numpy().astype(np.int64).astype(np.uint16).view(np.int16)
        slot.flag(self.rank)[0] = epoch
        return self._collect(slot, epoch, slot.ang_off, int(n_total), np.float16,
                             'checkpoint angles')

    def place_ranked(self, lib, vals, rows, n_rows, comm_dev):
        """The on-the-fly angle changes (track_orbits_onthefly.py:154-174): this rank's
        values ``vals`` (4- or 8-byte elements, device or CPU) among every rank's,
        ordered by their global previous rows ``rows`` (disjoint over the ranks, in
        [0, n_rows)).  A bitmap rank gives each value its position and every rank the
        total; each rank stores its values there, over its own link.  Returns the values
        (``vals``' dtype) on rank 0, a view of the buffer (the slot busy while it lives);
        None elsewhere.  Synchronous."""
        import ctypes
        self.lib = lib
        self.epoch += 1
        epoch = self.epoch
        dev = vals.device
        n = int(vals.shape[0])
        dst, total = self._rank_by_row(rows[:n].to(dev).to(torch.int64), int(n_rows), comm_dev,
                                       with_total=True)
        ib = vals.element_size()
        if ib not in (4, 8):
            raise ValueError('place_ranked: 4- or 8-byte values, got %d bytes' % ib)
        slot = self._agree(total, ib, comm_dev)
        if total > slot.cap:
            raise RuntimeError('sharded outputs: %d values, output capacity %d'
                               % (total, slot.cap))
        if dev.type == 'cuda':
            from . import _native as N
            if self.status is None:
                self.status = torch.zeros(1, dtype=torch.int32, device=dev)
            base = slot.register(lib)
            v = vals.contiguous()
            d = dst.contiguous()
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            N.check(lib.oa_place_records(ctypes.c_void_p(v.data_ptr()), None,
                                         ctypes.c_void_p(d.data_ptr()), n, ib,
                                         ctypes.c_void_p(base + slot.ids_off), None, slot.cap,
                                         ctypes.c_void_p(self.status.data_ptr()), st),
                    'oa_place_records')
            torch.cuda.current_stream(dev).synchronize()
            if int(self.status.item()):
                raise RuntimeError('sharded outputs: values outside the output')
        elif n:
            d = dst.numpy()
            if d.min() < 0 or d.max() >= slot.cap:
                raise RuntimeError('sharded outputs: values outside the output')
            slot.ids[d] = vals.numpy().view(slot.ids.dtype)
        slot.flag(self.rank)[0] = epoch
        return self._collect(slot, epoch, slot.ids_off, total,
                             torch.empty(0, dtype=vals.dtype).numpy().dtype, 'sharded outputs')

    def _collect(self, slot, epoch, off, n, dtype, what):
        """Rank 0 of a synchronous placement: wait for every rank's epoch, then the first
        ``n`` values of ``dtype`` at byte ``off`` of the slot as an array backed by a ctypes
        holder (the slot stays busy while it lives); None on the other ranks."""
        import ctypes
        if self.rank != self.root:
            return None
        t_end = time.time() + self.timeout
        while not all(int(slot.flag(q)[0]) == epoch for q in range(self.world)):
            if time.time() > t_end:
                raise RuntimeError('%s: a rank did not store its values within %.0f s'
                                   % (what, self.timeout))
            time.sleep(2e-5)
        if slot.linked:
            self._unlink(slot)
        slot.busy -= 1                    # in flight since _choose
        dt = np.dtype(dtype)
        if not n:
            return np.zeros(0, dt)
        h = (ctypes.c_char * (int(n) * dt.itemsize)).from_buffer(slot.mm, off)
        slot.busy += 1
        weakref.finalize(h, self._free, slot)
        return np.frombuffer(h, dtype=dt)

    def probe(self, lib, comm_dev, on_gpu):
        """Whether every rank can map a shared segment and page-lock it for device
        stores (one 1-element all-reduce): a caller that cannot rely on the stage (a
        benchmark pass) checks this first, so no rank is left in a collective alone."""
        import ctypes
        import tempfile
        import torch.distributed as dist
        ok = 1
        try:
            fd, path = tempfile.mkstemp(prefix='oa_probe_', dir=_shm_dir())
            os.ftruncate(fd, 1 << 16)
            mm = mmap.mmap(fd, 1 << 16, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
            os.close(fd)
            os.unlink(path)
            if on_gpu:
                base = np.frombuffer(mm, dtype=np.uint8).ctypes.data
                p = ctypes.c_void_p()
                if lib.oa_host_register(ctypes.c_void_p(base), 1 << 16, ctypes.byref(p)) != 0:
                    ok = 0
                else:
                    lib.oa_host_unregister(ctypes.c_void_p(base))
        except Exception:
            ok = 0
        t = torch.tensor([ok], dtype=torch.int32).to(comm_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(t.item()))

    def _rank_by_row(self, rows, n_rows, comm_dev, with_total=False):
        """Every record's position among all ranks' records ordered by global previous
        row: bits of the rows each rank holds, OR-ed over the ranks by one all-reduce
        (the ranks' rows are disjoint: a byte sum is the OR), then prefix popcounts.
        The bitmap is built and ranked on the rows' device; only its bytes travel
        through ``comm_dev``.  ``with_total``: also the number of records over all
        ranks."""
        import torch.distributed as dist
        nb = max((n_rows + 7) // 8, 1)
        dev = rows.device
        r = rows.to(torch.int64)
        bits = torch.zeros(nb, dtype=torch.int32, device=dev)
        bits.index_add_(0, r >> 3, (1 << (r & 7)).to(torch.int32))
        b = bits.to(torch.uint8).to(comm_dev)
        dist.all_reduce(b, op=dist.ReduceOp.SUM, group=self.group)
        bl = b.to(dev).long()
        lut = torch.from_numpy(_POP8).to(dev)
        pc = lut[bl]
        pre = torch.cumsum(pc, 0) - pc
        byte = r >> 3
        pos = pre[byte] + lut[bl[byte] & ((1 << (r & 7)) - 1)]
        if with_total:
            return pos, int((pre[-1] + pc[-1]).item())
        return pos

    def close(self):
        for s in self.slots.values():
            try:
                s.release(self.lib)
            except Exception:
                pass
