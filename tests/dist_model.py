"""Slab-z domain-decomposed multigrid cycle over torch.distributed (TEST INFRASTRUCTURE ONLY).

A rank-local NumPy model of the schedule that libmgpoisson.so runs with world > 1
(csrc/mgp_api.cpp: smooth / residual_restrict / prolong_correct / cycle_rec / one_cycle):

* each rank owns nz/world contiguous z-planes of a distributed level and sees its z-neighbours'
  boundary planes as ghost planes, refreshed by a send/recv pair per neighbour before every
  red/black half-sweep that reads them (exchange / exchange_buf), zero at the physical boundary;
* the residual is restricted locally; at the first replicated level of the plan the coarse
  right-hand sides are all-gathered and the rest of the hierarchy runs redundantly on every rank
  (cf. the level hand-off of cpu-gpu.lua:17-52);
* linear prolongation from a distributed coarse level reads one coarse ghost plane per side;
* err = sqrt(allreduce(sum (psi - psiOld)^2) / N) in fp64 (cpu.lua:200-203).

The level plan comes from the library's own host logic (mgp_plan), so a CPU world-2 run of this
model checks the decomposition the GPU path uses: the gathered psi must be bit-identical to the
single-domain NumPy oracle (mgp_oracle_np.Multigrid), because exchanges only move values.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

import mgp_oracle_np as N


def _halo(u: np.ndarray, rank: int, world: int):
    """(lower ghost, upper ghost) planes of u from the z-neighbours; zeros at the box faces."""
    lo = np.zeros_like(u[0])
    hi = np.zeros_like(u[0])
    ops = []
    t_lo = torch.from_numpy(lo)
    t_hi = torch.from_numpy(hi)
    if rank > 0:
        ops.append(dist.P2POp(dist.isend, torch.from_numpy(np.ascontiguousarray(u[0])), rank - 1))
        ops.append(dist.P2POp(dist.irecv, t_lo, rank - 1))
    if rank < world - 1:
        ops.append(dist.P2POp(dist.isend, torch.from_numpy(np.ascontiguousarray(u[-1])), rank + 1))
        ops.append(dist.P2POp(dist.irecv, t_hi, rank + 1))
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    return t_lo.numpy(), t_hi.numpy()


def _nbsum_ghost(u, lo, hi):
    """((((xl + xr) + yl) + yr) + zl) + zr with z-neighbours from the ghost planes."""
    ext = np.concatenate([lo[None], u, hi[None]], axis=0)
    p = np.pad(ext, ((0, 0), (1, 1), (1, 1)))
    xl, xr = p[1:-1, 1:-1, :-2], p[1:-1, 1:-1, 2:]
    yl, yr = p[1:-1, :-2, 1:-1], p[1:-1, 2:, 1:-1]
    zl, zr = p[:-2, 1:-1, 1:-1], p[2:, 1:-1, 1:-1]
    return ((((xl + xr) + yl) + yr) + zl) + zr


def _relax(u, f, h, cl, z0, gnz, lo, hi):
    hsq, _ = N._consts(h, 3, u.dtype)
    return (f - _nbsum_ghost(u, lo, hi) / hsq) / N.diag(u.shape, h, 3, u.dtype, cl, z0, gnz)


def _prolong_slab(Vsrc, vbase, fine_shape, z0, gnzc, kind, cl):
    """N.prolong restricted to fine planes z0 .. z0 + nz - 1; Vsrc[0] is global coarse plane vbase."""
    nz, ny, nx = fine_shape
    K = np.arange(nz) + z0
    parent = K >> 1
    if kind == N.PROLONG_PC:
        v = np.repeat(np.repeat(Vsrc[parent - vbase], 2, axis=2), 2, axis=1)
        return v
    dt = Vsrc.dtype.type
    w0, w1, c = dt(0.75), dt(0.25), dt(cl)
    cy, cx = Vsrc.shape[1:]
    xi = N._axis_idx(nx, cx)
    yi = N._axis_idx(ny, cy)
    nb = np.where(K & 1, parent + 1, parent - 1)
    zout = (nb < 0) | (nb >= gnzc)
    zi = (parent - vbase, np.clip(nb, 0, gnzc - 1) - vbase, zout)

    def val(px, py, pz):
        I = xi[px][None, None, :]
        J = yi[py][None, :, None]
        Kc = zi[pz][:, None, None]
        s = np.ones((nz, ny, nx), dtype=Vsrc.dtype)
        if px:
            s = np.where(xi[2][None, None, :], -c * s, s)
        if py:
            s = np.where(yi[2][None, :, None], -c * s, s)
        if pz:
            s = np.where(zi[2][:, None, None], -c * s, s)
        return s * Vsrc[Kc, J, I]

    a00 = w0 * val(0, 0, 0) + w1 * val(1, 0, 0)
    a10 = w0 * val(0, 1, 0) + w1 * val(1, 1, 0)
    a01 = w0 * val(0, 0, 1) + w1 * val(1, 0, 1)
    a11 = w0 * val(0, 1, 1) + w1 * val(1, 1, 1)
    b0 = w0 * a00 + w1 * a10
    b1 = w0 * a01 + w1 * a11
    return w0 * b0 + w1 * b1


class SlabMultigrid:
    """One rank's share of a 3D box: ``rows`` is this rank's mgp_plan() output."""

    def __init__(self, rows, dtype=np.float64, nu1=2, nu2=2, smoother=N.RBGS, cycle=N.CYCLE_V,
                 prolong_kind=N.PROLONG_LINEAR, coarse_init=N.COARSE_FRESH, coarse_sweeps=48,
                 coarse_bc=N.BC_CONSISTENT):
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.rows = rows
        self.dt = np.dtype(dtype)
        self.nu1, self.nu2, self.smoother, self.cycle = nu1, nu2, smoother, cycle
        self.prolong_kind, self.coarse_init, self.coarse_sweeps, self.coarse_bc = \
            prolong_kind, coarse_init, coarse_sweeps, coarse_bc
        self.u = [np.zeros((r["nz_local"], r["ny"], r["nx"]), self.dt) for r in rows]
        self.f = [np.zeros_like(u) for u in self.u]

    def init_point_charge(self):
        r = self.rows[0]
        self.f[0][...] = 0
        c = (r["nz_global"] // 2, r["ny"] // 2, r["nx"] // 2)
        k = c[0] - r["z0"]
        if 0 <= k < r["nz_local"]:
            self.f[0][k, c[1], c[2]] = self.dt.type(-1e6)
        self.u[0] = -self.f[0]

    # -- level operations (distributed or replicated) --
    def _smooth(self, l, sweeps, h):
        r = self.rows[l]
        cl = N.coarse_coef(self.coarse_bc, l)
        u, f = self.u[l], self.f[l]
        if not r["distributed"]:
            self.u[l] = N.smooth(u, f, h, 3, self.smoother, sweeps, cl)
            return
        z0, gnz = r["z0"], r["nz_global"]
        red = N.color_mask(u.shape, z0)
        for _ in range(sweeps):
            if self.smoother == N.JACOBI:
                lo, hi = _halo(u, self.rank, self.world)
                u = _relax(u, f, h, cl, z0, gnz, lo, hi)
                continue
            lo, hi = _halo(u, self.rank, self.world)  # red reads black
            u = np.where(red, _relax(u, f, h, cl, z0, gnz, lo, hi), u)
            lo, hi = _halo(u, self.rank, self.world)  # black reads the new red planes
            u = np.where(~red, _relax(u, f, h, cl, z0, gnz, lo, hi), u)
        self.u[l] = u

    def _residual_restrict(self, l, h):
        r, rc = self.rows[l], self.rows[l + 1]
        cl = N.coarse_coef(self.coarse_bc, l)
        u, f = self.u[l], self.f[l]
        if not r["distributed"]:
            self.f[l + 1] = N.restrict(N.residual(u, f, h, 3, cl), 3)
            return
        lo, hi = _halo(u, self.rank, self.world)
        hsq, _ = N._consts(h, 3, u.dtype)
        askew = _nbsum_ghost(u, lo, hi) / hsq
        res = f - (askew + N.diag(u.shape, h, 3, u.dtype, cl, r["z0"], r["nz_global"]) * u)
        R = N.restrict(res, 3)
        if rc["distributed"]:
            self.f[l + 1] = R
        else:  # agglomerate (ncclAllGather in the library)
            parts = [torch.empty(R.shape, dtype=torch.from_numpy(R).dtype) for _ in range(self.world)]
            dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(R)))
            self.f[l + 1] = np.concatenate([p.numpy() for p in parts], axis=0)

    def _prolong_correct(self, l):
        r, rc = self.rows[l], self.rows[l + 1]
        clc = N.coarse_coef(self.coarse_bc, l + 1)
        u, V = self.u[l], self.u[l + 1]
        if not r["distributed"]:
            self.u[l] = u + N.prolong(V, u.shape, 3, self.prolong_kind, clc)
            return
        if rc["distributed"]:
            if self.prolong_kind == N.PROLONG_LINEAR:
                lo, hi = _halo(V, self.rank, self.world)
            else:
                lo = hi = np.zeros_like(V[0])
            src, base = np.concatenate([lo[None], V, hi[None]], axis=0), rc["z0"] - 1
        else:
            src, base = V, 0
        self.u[l] = u + _prolong_slab(src, base, u.shape, r["z0"], rc["nz_global"], self.prolong_kind, clc)

    def _cycle(self, l, h, fcycle):
        if l == len(self.rows) - 1:
            r = self.rows[l]
            cells = r["nx"] * r["ny"] * r["nz_global"]
            self._smooth(l, 1 if cells == 1 else self.coarse_sweeps, h)
            return
        self._smooth(l, self.nu1, h)
        self._residual_restrict(l, h)
        if self.coarse_init == N.COARSE_FRESH:
            self.u[l + 1] = np.zeros_like(self.u[l + 1])
        if fcycle:
            self._cycle(l + 1, 2 * h, True)
        self._cycle(l + 1, 2 * h, False)
        self._prolong_correct(l)
        self._smooth(l, self.nu2, h)

    def step(self) -> float:
        r = self.rows[0]
        old = self.u[0].copy()
        self._cycle(0, 1.0 / r["nx"], self.cycle == N.CYCLE_F)
        d = self.u[0].astype(np.float64) - old.astype(np.float64)
        s = torch.tensor([float(np.sum(d * d))], dtype=torch.float64)
        dist.all_reduce(s)
        return float(np.sqrt(s.item() / (r["nx"] * r["ny"] * r["nz_global"])))


def run_rank(rank, world, port, plans, cfg, cycles, out_dir):
    """torch.multiprocessing entry: run `cycles` outer iterations, save psi slab and errs."""
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        mg = SlabMultigrid(plans[rank], **cfg)
        mg.init_point_charge()
        errs = [mg.step() for _ in range(cycles)]
        np.savez(f"{out_dir}/rank{rank}.npz", psi=mg.u[0], errs=np.array(errs))
    finally:
        dist.destroy_process_group()
