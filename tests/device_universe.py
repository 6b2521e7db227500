"""Test helper: BASELINE-sized synthetic universes (synthetic_device.DevicePlummer) behind
the reference's callback API (track_orbits.py:118-122 / track_orbits_onthefly.py:28-34).

``DeviceUniverse`` generates every snapshot once (the generator only moves forward) and
hands out device tensors; ``RankMajorUniverse`` is the global snapshot a set of
presharded ranks forms (each rank's DevicePlummer draws its own ID range; every block is
the ranks' blocks concatenated in rank order), for single-process reference runs."""
import numpy as np
import torch


class DeviceUniverse:
    def __init__(self, n_snapshots, **kw):
        from orbitanalysis_amd.synthetic_device import DevicePlummer
        self.gen = DevicePlummer(**kw)
        self.n_halos = self.gen.n_halos
        self.snapshot_numbers = np.arange(n_snapshots)
        self.snaps = [self.gen.snapshot(s) for s in range(n_snapshots)]
        self.cats = [self.gen.catalogue(s) for s in range(n_snapshots)]
        self.loads = []

    def main_branches(self):
        return np.tile(np.arange(self.n_halos), (len(self.snapshot_numbers), 1))

    def regions(self, s, halo_ids):
        c = self.cats[s]
        return c[0][halo_ids], c[1][halo_ids], c[2][halo_ids]

    def regions_otf(self, s, halo_ids):
        c = self.cats[s]
        return c[0][halo_ids], c[1][halo_ids]

    def load_snapshot_data(self, s, pos, rad):
        self.loads.append(int(s))
        return dict(self.snaps[s])

    def host_blocks(self, s, k):
        """Host copy of the first k blocks of snapshot s (oracle samples)."""
        snap = self.snaps[s]
        off = np.append(snap['region_offsets'], snap['ids'].numel())
        end = int(off[k])
        d = {key: snap[key][:end].cpu().numpy() for key in ('ids', 'coordinates', 'velocities')}
        d.update(masses=snap['masses'], box_size=snap['box_size'],
                 region_offsets=off[:k].copy())
        return d


def rank_major(snaps):
    """One snapshot from the ranks' snapshots: every block = the ranks' rows of that
    block in rank order (what ShardedEngine(presharded=True) treats as global)."""
    nh = len(snaps[0]['region_offsets'])
    dev = snaps[0]['ids'].device
    parts = []
    for r, sn in enumerate(snaps):
        n = sn['ids'].numel()
        cnt = np.diff(np.append(sn['region_offsets'], n))
        h = torch.repeat_interleave(torch.arange(nh, device=dev), torch.from_numpy(cnt).to(dev))
        parts.append((h * len(snaps) + r, sn, cnt))
    key = torch.cat([p[0] for p in parts])
    order = torch.sort(key, stable=True)[1]
    out = dict(snaps[0])
    for k in ('ids', 'coordinates', 'velocities'):
        out[k] = torch.cat([p[1][k] for p in parts])[order].contiguous()
    tot = sum(p[2] for p in parts)
    out['region_offsets'] = np.concatenate([[0], np.cumsum(tot)[:-1]]).astype(np.int64)
    return out


def digest(groups):
    """sha256 of every dataset (dtype, shape and bytes) of a savefile's groups."""
    import hashlib
    out = {}
    for g, ds in groups.items():
        for k, v in ds.items():
            a = np.ascontiguousarray(np.asarray(v))
            h = hashlib.sha256(('%s|%s|' % (a.dtype.str, a.shape)).encode())
            h.update(a.tobytes())
            out[g + '/' + k] = h.hexdigest()
    return out
