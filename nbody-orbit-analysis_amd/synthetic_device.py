"""Large synthetic Plummer-sphere snapshots generated on the GPU (benchmark inputs).

Same model as ``synthetic.PlummerSnapshots`` at 1e8+ particles:
N_h Plummer spheres (G = M = a = 1, Aarseth-Henon-Wielen sampling), kick-drift-kick
leapfrog in each halo's fixed potential, halo centres drifting with a catalogue bulk
velocity in a periodic box, a region cut r < r_cut (≈1 % of particles enter/leave a
region per snapshot), every block shuffled per snapshot.

Multi-GPU (ID-range sharding): rank r owns the IDs
[r*R, (r+1)*R).  Halo centres/velocities come from a seed shared by all ranks; each
rank draws its own particles of every halo, which is statistically identical to
drawing the global population and keeping the IDs in the rank's range.
"""
import math

import numpy as np
import torch


def _isotropic(mag, gen):
    n = mag.numel()
    cz = torch.rand(n, generator=gen, device=mag.device, dtype=torch.float32) * 2 - 1
    ph = torch.rand(n, generator=gen, device=mag.device, dtype=torch.float32) * (2 * math.pi)
    sz = torch.sqrt(torch.clamp(1 - cz * cz, min=0))
    return torch.stack([sz * torch.cos(ph), sz * torch.sin(ph), cz], dim=1) * mag[:, None]


def plummer_sample_device(n, gen, device):
    x1 = torch.rand(n, generator=gen, device=device, dtype=torch.float32).clamp_(1e-7, 1.0)
    r = torch.rsqrt(x1.pow(-2.0 / 3.0) - 1.0).clamp_(max=30.0)
    pos = _isotropic(r, gen)
    q = torch.empty(n, device=device, dtype=torch.float32)
    todo = torch.arange(n, device=device)
    while todo.numel():
        x4 = torch.rand(todo.numel(), generator=gen, device=device)
        x5 = torch.rand(todo.numel(), generator=gen, device=device) * 0.1
        ok = x5 < x4 * x4 * (1 - x4 * x4).pow(3.5)
        q[todo[ok]] = x4[ok]
        todo = todo[~ok]
    vesc = math.sqrt(2.0) * (1 + r * r).pow(-0.25)
    return pos, _isotropic(q * vesc, gen)


class DevicePlummer:
    """Resident snapshot generator.  ``snapshot(s)`` returns device tensors in the
    loader's layout plus the catalogue rows for every halo."""

    def __init__(self, n_halos=10000, n_particles=100_000_000, seed=0, rank=0, world=1,
                 r_cut=4.0, dt=0.5, substeps=5, box_size=None, halo_velocity=0.3,
                 device='cuda', cosmology=None, dtype='float32'):
        self.device = torch.device(device)
        self.np_dtype = np.dtype(dtype)             # loader dtype of coordinates / velocities
        self.t_dtype = torch.float64 if self.np_dtype == np.float64 else torch.float32
        self.n_halos = int(n_halos)
        # population per halo so that ≈ n_particles sit inside the region cuts:
        # Plummer M(<r) = r^3 / (r^2 + 1)^1.5
        inside = r_cut ** 3 / (r_cut ** 2 + 1) ** 1.5
        self.pop = int(math.ceil(n_particles / inside / self.n_halos))
        self.n_pop = self.pop * self.n_halos
        self.r_cut, self.dt, self.substeps = float(r_cut), float(dt), int(substeps)
        self.box = float(box_size if box_size is not None
                         else 25.0 * max(1.0, self.n_halos ** (1.0 / 3.0)))
        self.cosmology = cosmology or dict(redshift=0.5, H0=0.07, Omega_m=0.3, Omega_L=0.7)
        hg = np.random.default_rng(seed)                      # shared halo catalogue
        self.centres0 = hg.uniform(0, self.box, (self.n_halos, 3))
        self.halo_vel = hg.normal(0, halo_velocity, (self.n_halos, 3))
        gen = torch.Generator(device=self.device)
        gen.manual_seed(1_000_003 * (rank + 1) + seed)
        self.gen = gen
        self.x, self.v = plummer_sample_device(self.n_pop, gen, self.device)
        self.halo_of = torch.arange(self.n_halos, device=self.device,
                                    dtype=torch.int64).repeat_interleave(self.pop)
        self.ids = torch.randperm(self.n_pop, generator=gen, device=self.device) + rank * self.n_pop
        self.d_c0 = torch.tensor(self.centres0, device=self.device, dtype=torch.float64)
        self.d_hv = torch.tensor(self.halo_vel, device=self.device, dtype=torch.float64)
        self.s = 0

    def _advance(self):
        h = self.dt / self.substeps
        x, v = self.x, self.v
        for _ in range(self.substeps):
            r2 = (x * x).sum(1, keepdim=True)
            v.add_(x * (-0.5 * h) * (r2 + 1).pow(-1.5))
            x.add_(v * h)
            r2 = (x * x).sum(1, keepdim=True)
            v.add_(x * (-0.5 * h) * (r2 + 1).pow(-1.5))
        self.s += 1

    def catalogue(self, s):
        t = s * self.dt
        c = np.mod(self.centres0 + self.halo_vel * t, self.box)
        dt = self.np_dtype
        return c.astype(dt), np.full(self.n_halos, self.r_cut, dt), self.halo_vel.astype(dt)

    def snapshot(self, s):
        """Snapshot s (s must not decrease between calls)."""
        while self.s < s:
            self._advance()
        inside = (self.x * self.x).sum(1) < self.r_cut ** 2
        sel = torch.nonzero(inside).squeeze(1)
        key = self.halo_of[sel] * (1 << 31) + torch.randint(
            0, 1 << 31, (sel.numel(),), generator=self.gen, device=self.device)
        sel = sel[torch.argsort(key)]
        h = self.halo_of[sel]
        t = s * self.dt
        c = torch.remainder(self.d_c0 + self.d_hv * t, self.box)
        coords = torch.remainder(self.x[sel].double() + c[h], self.box).to(self.t_dtype).contiguous()
        vels = (self.v[sel].double() + self.d_hv[h]).to(self.t_dtype).contiguous()
        counts = torch.bincount(h, minlength=self.n_halos).cpu().numpy()
        offsets = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
        snap = {'ids': self.ids[sel].contiguous(), 'coordinates': coords, 'velocities': vels,
                'masses': 1.0 / self.n_pop, 'region_offsets': offsets,
                'box_size': self.box, 'redshift': float(self.cosmology['redshift']),
                'H0': float(self.cosmology['H0']), 'Omega_m': float(self.cosmology['Omega_m']),
                'Omega_L': float(self.cosmology['Omega_L'])}
        return snap
