"""World-size-2 (and 4) CPU tests of the slab-z decomposition with the gloo backend.

The library's multi-GPU path (RCCL halo exchange, all-gather agglomeration, err all-reduce) needs
one GPU per rank, so on CPU the same schedule runs in tests/dist_model.py over torch.distributed
gloo, driven by the level plan the library itself computes (mgp_plan, host logic).  Bar: the
gathered psi is bit-identical to the single-domain NumPy oracle after every cycle (exchanges only
move values); err agrees to fp64 summation order (1e-12 relative).
"""
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import dist_model
import mgp_oracle_np as N


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _mg():
    import mgpoisson

    return mgpoisson


CASES = [
    # box (nx, ny, nz_global), world, gather_cells, model config
    ((16, 16, 32), 2, 64, dict(dtype=np.float64)),
    ((16, 16, 32), 2, 64, dict(dtype=np.float32, cycle=N.CYCLE_F)),
    ((8, 16, 16), 2, 16, dict(dtype=np.float64, smoother=N.JACOBI, nu1=3, nu2=3, prolong_kind=N.PROLONG_PC,
                              coarse_bc=N.BC_ZERO, coarse_init=N.COARSE_WARM)),
    ((16, 8, 32), 4, 32, dict(dtype=np.float64, prolong_kind=N.PROLONG_PC)),
]


@pytest.mark.parametrize("box,world,gather,cfg", CASES,
                         ids=["rbgs-lin-V-f64", "rbgs-lin-F-f32", "jac-pc-warm-f64", "w4-rbgs-pc"])
def test_slab_decomposition_matches_single_domain(box, world, gather, cfg, tmp_path):
    mg = _mg()
    names = {N.RBGS: "rbgs", N.JACOBI: "jacobi"}
    plans = [mg.plan(mg.make_opts(dim=3, n=box, rank=r, world=world, gather_cells=gather,
                                  smoother=names[cfg.get("smoother", N.RBGS)], comm_id=b"\0" * 128))
             for r in range(world)]
    assert sum(lv["distributed"] for lv in plans[0]) >= 2, "case should keep >= 2 distributed levels"
    cycles = 3
    mp.spawn(dist_model.run_rank, args=(world, _free_port(), plans, cfg, cycles, str(tmp_path)), nprocs=world,
             join=True)
    outs = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    psi = np.concatenate([o["psi"] for o in outs], axis=0)

    ref = N.Multigrid(3, box, cfg.get("dtype", np.float64), cfg.get("nu1", 2), cfg.get("nu2", 2),
                      cfg.get("smoother", N.RBGS), cfg.get("cycle", N.CYCLE_V),
                      cfg.get("prolong_kind", N.PROLONG_LINEAR), cfg.get("coarse_init", N.COARSE_FRESH),
                      coarse_bc=cfg.get("coarse_bc", N.BC_CONSISTENT))
    # the single-domain oracle's hierarchy must be the plan's
    assert [s[::-1] for s in ref.shapes] == [(lv["nx"], lv["ny"], lv["nz_global"]) for lv in plans[0]]
    ref.init_point_charge()
    errs = [ref.step() for _ in range(cycles)]
    assert psi.dtype == ref.psi.dtype
    assert np.array_equal(psi, ref.psi), float(np.max(np.abs(psi - ref.psi)))
    for o in outs:
        np.testing.assert_allclose(o["errs"], errs, rtol=1e-12, atol=0)
