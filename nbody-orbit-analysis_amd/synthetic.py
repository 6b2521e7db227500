"""Deterministic synthetic N-body snapshots (host / NumPy) for tests and fixtures.

The reference ships no data and no tests, so every parity case and
benchmark runs on synthetic Plummer spheres as SURVEY.md §8(d) specifies:

* N_h halos, each a Plummer sphere (G = M = a = 1) sampled with the
  Aarseth-Henon-Wielen (1974) rejection method;
* particles orbit in their halo's fixed Plummer potential (kick-drift-kick
  leapfrog), the halo centre drifts with a constant bulk velocity;
* IDs are a seeded permutation of ``arange(N)`` (+ an optional offset);
* the loader cuts a sphere of radius ``r_cut`` around each requested centre from
  the *whole* population (regions may overlap, so one ID can sit in several
  blocks) and returns every block in a per-snapshot shuffled order.

``regions`` / ``load_snapshot_data`` follow the reference's callback contracts
(``track_orbits.py:27-61``, ``:118-122``; onthefly ``track_orbits_onthefly.py:28,34``).
This module is product-side tooling (used by ``bench.py`` at small sizes and by
the tests); the large-scale device generator lives in ``synthetic_device.py``.
"""
import numpy as np


def plummer_sample(n, rng):
    """Positions/velocities of an isotropic Plummer sphere, G = M = a = 1 (AHW 1974)."""
    x1 = rng.uniform(1e-10, 1.0, n)
    r = 1.0 / np.sqrt(x1 ** (-2.0 / 3.0) - 1.0)
    r = np.minimum(r, 30.0)
    pos = _isotropic(r, rng)
    q = np.empty(n)
    todo = np.arange(n)
    while todo.size:
        x4 = rng.uniform(0.0, 1.0, todo.size)
        x5 = rng.uniform(0.0, 0.1, todo.size)
        ok = x5 < x4 ** 2 * (1.0 - x4 ** 2) ** 3.5
        q[todo[ok]] = x4[ok]
        todo = todo[~ok]
    vesc = np.sqrt(2.0) * (1.0 + r ** 2) ** (-0.25)
    vel = _isotropic(q * vesc, rng)
    return pos, vel


def _isotropic(mag, rng):
    n = mag.size
    cz = rng.uniform(-1.0, 1.0, n)
    ph = rng.uniform(0.0, 2.0 * np.pi, n)
    sz = np.sqrt(1.0 - cz ** 2)
    return mag[:, None] * np.stack([sz * np.cos(ph), sz * np.sin(ph), cz], axis=1)


def plummer_accel(x):
    r2 = np.einsum('ij,ij->i', x, x)
    return -x / (r2 + 1.0)[:, None] ** 1.5


class PlummerSnapshots:
    """A seeded, fully deterministic sequence of synthetic snapshots.

    Parameters mirror the knobs the parity cases need:
    dtype of particle data and of the catalogue centres, scalar vs array masses,
    catalogue vs computed bulk velocity, periodic box, Hubble term, halo births.
    """

    def __init__(self, n_halos=1, n_per_halo=10000, n_snapshots=10, seed=0,
                 dt=0.5, substeps=10, r_cut=4.0, box_size=None, centres=None,
                 halo_velocity=0.3, dtype=np.float64, centre_dtype=None,
                 masses='scalar', bulk='computed', cosmology=None,
                 births=None, id_offset=0, id_dtype=np.int64, first_snapshot=0,
                 shuffle=True, region_returns=3, absent=None, empty=None):
        self.n_halos = int(n_halos)
        sizes = np.broadcast_to(np.asarray(n_per_halo, dtype=np.int64), (self.n_halos,))
        self.sizes = sizes.copy()
        self.n_total = int(sizes.sum())
        self.n_snapshots = int(n_snapshots)
        self.seed = int(seed)
        self.dtype = np.dtype(dtype)
        self.centre_dtype = np.dtype(centre_dtype) if centre_dtype is not None else self.dtype
        self.masses_mode = masses
        self.bulk_mode = bulk
        self.r_cut = float(r_cut)
        self.box_size = box_size
        self.cosmology = cosmology
        self.first_snapshot = int(first_snapshot)
        self.shuffle = shuffle
        self.region_returns = region_returns
        self.snapshot_numbers = np.arange(self.n_snapshots) + self.first_snapshot

        rng = np.random.default_rng(self.seed)
        halo_of = np.repeat(np.arange(self.n_halos), sizes)
        self.halo_of = halo_of
        pos = np.empty((self.n_total, 3))
        vel = np.empty((self.n_total, 3))
        for h in range(self.n_halos):
            sl = halo_of == h
            p, v = plummer_sample(int(sizes[h]), rng)
            pos[sl], vel[sl] = p, v
        if centres is None:
            span = 10.0 * max(1.0, self.n_halos ** (1.0 / 3.0))
            if box_size is not None:
                span = float(np.max(box_size))
            centres = rng.uniform(0.0, span, (self.n_halos, 3))
        self.centres0 = np.asarray(centres, dtype=np.float64).reshape(self.n_halos, 3)
        self.halo_vel = rng.normal(0.0, halo_velocity, (self.n_halos, 3))
        perm = rng.permutation(self.n_total)
        if np.dtype(id_dtype).kind == 'u':
            self.ids = (perm.astype(np.uint64) + np.uint64(id_offset)).astype(id_dtype)
        else:
            self.ids = (perm.astype(np.int64) + np.int64(id_offset)).astype(id_dtype)
        if masses == 'array':
            self.mass_values = (rng.uniform(0.5, 1.5, self.n_total) / self.n_total).astype(self.dtype)
        else:
            self.mass_values = 1.0 / self.n_total
        if births is None:
            births = np.zeros(self.n_halos, dtype=np.int64)
        self.births = np.asarray(births, dtype=np.int64)
        # edge cases: (snapshot index, halo) pairs that are -1 in main_branches
        # (gaps, deaths, all-absent rows) / whose region radius is 0 (empty blocks; a
        # snapshot whose every region is empty loads 0 particles)
        self.absent = [tuple(int(v) for v in p) for p in (absent or [])]
        self.empty = {tuple(int(v) for v in p) for p in (empty or [])}

        # integrate all snapshots once (relative coordinates about each halo centre)
        self._rel_pos, self._rel_vel = [], []
        h_step = dt / substeps
        x, v = pos.copy(), vel.copy()
        for s in range(self.n_snapshots):
            self._rel_pos.append(x.copy())
            self._rel_vel.append(v.copy())
            for _ in range(substeps):
                v += 0.5 * h_step * plummer_accel(x)
                x += h_step * v
                v += 0.5 * h_step * plummer_accel(x)
        self.dt = dt

    # ------------------------------------------------------------------ state
    def _index(self, snapshot_number):
        return int(snapshot_number) - self.first_snapshot

    def halo_centres(self, snapshot_number):
        t = self._index(snapshot_number) * self.dt
        c = self.centres0 + self.halo_vel * t
        if self.box_size is not None:
            c = np.mod(c, np.asarray(self.box_size, dtype=np.float64))
        return c

    def absolute(self, snapshot_number):
        s = self._index(snapshot_number)
        c = self.halo_centres(snapshot_number)
        x = self._rel_pos[s] + c[self.halo_of]
        v = self._rel_vel[s] + self.halo_vel[self.halo_of]
        if self.box_size is not None:
            x = np.mod(x, np.asarray(self.box_size, dtype=np.float64))
        return x, v

    def main_branches(self):
        """(n_snap, n_halo) main-branch table, halo id = column, -1 before birth."""
        mb = np.tile(np.arange(self.n_halos, dtype=np.int64), (self.n_snapshots, 1))
        for h in range(self.n_halos):
            mb[:self.births[h], h] = -1
        for s, h in self.absent:
            mb[s, h] = -1
        return mb

    # --------------------------------------------------------------- callbacks
    def regions(self, snapshot_number, halo_ids):
        halo_ids = np.atleast_1d(np.asarray(halo_ids, dtype=np.int64))
        c = self.halo_centres(snapshot_number)[halo_ids].astype(self.centre_dtype)
        radii = np.full(halo_ids.size, self.r_cut, dtype=self.centre_dtype)
        if self.empty:
            s = self._index(snapshot_number)
            radii[[(s, int(h)) in self.empty for h in halo_ids]] = 0
        if self.region_returns == 2:
            return c, radii
        bulk = None
        if self.bulk_mode == 'catalogue':
            bulk = self.halo_vel[halo_ids].astype(self.centre_dtype)
        return c, radii, bulk

    def load_snapshot_data(self, snapshot_number, region_positions, region_radii):
        s = self._index(snapshot_number)
        x, v = self.absolute(snapshot_number)
        blocks = []
        for k, (c, rad) in enumerate(zip(np.atleast_2d(region_positions),
                                         np.atleast_1d(region_radii))):
            d = x - np.asarray(c, dtype=np.float64)
            if self.box_size is not None:
                L = np.asarray(self.box_size, dtype=np.float64)
                d = d - L * np.round(d / L)
            inds = np.flatnonzero(np.einsum('ij,ij->i', d, d) < float(rad) ** 2)
            if self.shuffle:
                prng = np.random.default_rng(
                    (self.seed * 7919 + 1234 + s * 1000003 + k) % (2 ** 63))
                inds = inds[prng.permutation(inds.size)]
            blocks.append(inds)
        lens = [b.size for b in blocks]
        sel = np.concatenate(blocks) if blocks else np.zeros(0, dtype=np.int64)
        snap = {
            'ids': self.ids[sel],
            'coordinates': x[sel].astype(self.dtype),
            'velocities': v[sel].astype(self.dtype),
            'masses': (self.mass_values[sel] if isinstance(self.mass_values, np.ndarray)
                       else self.mass_values),
            'region_offsets': np.cumsum([0] + lens)[:-1].astype(np.int64),
        }
        if self.box_size is not None:
            snap['box_size'] = self.box_size
        cosmo = self.cosmology or {}
        snap['redshift'] = float(cosmo.get('redshift', 0.0)) + 0.01 * (self.n_snapshots - 1 - s) \
            if cosmo else 0.0
        snap['H0'] = float(cosmo.get('H0', 0.0))
        snap['Omega_m'] = float(cosmo.get('Omega_m', 0.3))
        snap['Omega_L'] = float(cosmo.get('Omega_L', 0.7))
        if 'Omega_k' in cosmo:
            snap['Omega_k'] = float(cosmo['Omega_k'])
        return snap

    def input_digest(self):
        """sha256 over every snapshot the loader would return for all halos (fixture pin)."""
        import hashlib
        h = hashlib.sha256()
        mb = self.main_branches()
        for s, row in zip(self.snapshot_numbers, mb):
            ex = np.flatnonzero(row != -1)
            if ex.size == 0:
                continue
            reg = self.regions(s, row[ex])
            snap = self.load_snapshot_data(s, reg[0], reg[1])
            for key in ('ids', 'coordinates', 'velocities', 'region_offsets'):
                h.update(np.ascontiguousarray(snap[key]).tobytes())
        return h.hexdigest()
