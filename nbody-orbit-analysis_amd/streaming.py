"""Double-buffered snapshot H2D for the on-the-fly stream (BASELINE configs[4],
SURVEY.md §7 item 8, §8(f) f1).

The reference's on-the-fly driver calls ``load_snapshot_data(s, ...)`` once per call
(track_orbits_onthefly.py:22-34) and works on host arrays.  At 1e8+ particles per
snapshot the host-to-device copy (32 B per particle, ~70 ms per 1.25e8 over PCIe 5.0)
outweighs the device work, so a reader that streams should keep the copy of snapshot
s+1 in flight while snapshot s is compared.  ``PinnedRing`` does that:

  * every snapshot's arrays sit in page-locked host memory (a reader fills them);
  * ``prefetch(k)`` starts the H2D of snapshot k into device slot k % slots on a
    high-priority copy stream (a normal-priority stream can share the compute stream's
    hardware queue and hold its kernels behind the copy: INTEGRATION.md, deployment
    note);
  * ``get(k)`` makes the compute stream wait for snapshot k's copy and returns device
    views of the slot, in the loader's dict layout;
  * ``loader`` is a ``load_snapshot_data`` for ``track_orbits_onthefly.track_orbits``:
    it hands out snapshot s and starts the copy of s + 1.

Three slots: snapshot s is compared against s - 1, whose device arrays (the carried
frame state keeps its IDs) must stay intact while s + 1 is copied.  A snapshot may
hold only this rank's stripe of the global one (``sharding.STRIPE``, a striped
reader for ``ShardedOnTheFly``)."""
import numpy as np
import torch


class PinnedRing:
    KEYS = ('ids', 'coordinates', 'velocities')

    def __init__(self, host, extra=None, device=None, slots=3):
        """``host``: {snapshot number: {'ids', 'coordinates', 'velocities' (page-locked
        host tensors), 'region_offsets', ...}}; ``extra``: keys added to every dict
        handed out (masses, box_size, ...)."""
        if slots < 3:
            raise ValueError('the ring needs 3 slots: s - 1 (carried), s, s + 1 (in flight)')
        self.host = host
        self.extra = dict(extra or {})
        self.device = torch.device(device if device is not None else 'cuda')
        first = next(iter(host.values()))
        nmax = max(int(h['ids'].shape[0]) for h in host.values())
        self.slots = [{k: torch.empty((nmax,) + tuple(first[k].shape[1:]), dtype=first[k].dtype,
                                      device=self.device) for k in self.KEYS}
                      for _ in range(slots)]
        self.stream = torch.cuda.Stream(device=self.device, priority=-1)
        self.events = {}
        self.slot_of = {}
        self.h2d_bytes = 0

    def prefetch(self, k):
        """Start the H2D of snapshot ``k`` (no-op if it is in flight / resident or not
        held).  The copy waits for the compute stream's work queued so far, so a slot
        is never overwritten under a kernel still reading it."""
        if k in self.events or k not in self.host:
            return
        i = k % len(self.slots)                 # s - 1, s, s + 1: three distinct slots
        for old, j in list(self.slot_of.items()):
            if j == i:                          # the slot's previous snapshot leaves
                del self.slot_of[old]
                self.events.pop(old, None)
        self.slot_of[k] = i
        src, dst = self.host[k], self.slots[i]
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            for key in self.KEYS:
                n = int(src[key].shape[0])
                dst[key][:n].copy_(src[key], non_blocking=True)
                self.h2d_bytes += src[key].numel() * src[key].element_size()
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.events[k] = ev

    def get(self, k):
        """Snapshot ``k`` as device views (the compute stream waits for its copy)."""
        self.prefetch(k)
        torch.cuda.current_stream(self.device).wait_event(self.events[k])
        src = self.host[k]
        m = int(src['ids'].shape[0])
        d = {key: self.slots[self.slot_of[k]][key][:m] for key in self.KEYS}
        for key, v in src.items():
            if key not in self.KEYS:
                d[key] = v
        d.update(self.extra)
        return d

    def loader(self, s, positions=None, radii=None):
        """``load_snapshot_data``: snapshot s on the device, and s + 1 on its way."""
        d = self.get(s)
        self.prefetch(s + 1)
        return d


def pin_snapshot(snap):
    """A loader dict with its per-particle arrays copied to page-locked host tensors."""
    out = dict(snap)
    for k in PinnedRing.KEYS:
        v = snap[k]
        t = v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t)
        out[k] = h
    return out
