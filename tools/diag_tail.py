#!/usr/bin/env python3
"""Diagnostic: 2D 256^2 Jacobi 7+7 with every level per piece (set_coarse_level(0)) once disagreed with the
oracle (test_coarse_level_switch_is_exact[2d-jacobi]).  For each configuration: a reference run, then TRIALS
runs on device memory just released by other work, comparing psi and err with the reference after every
cycle; prints the first cycle of each disagreement."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lua-multigrid-poisson_amd"), os.path.join(ROOT, "tests")]
import mgpoisson as mg  # noqa: E402
import torch  # noqa: E402

CYC = int(os.environ.get("CYC", "3"))
TRIALS = int(os.environ.get("TRIALS", "6"))
CONFIGS = {
    "2d-jacobi-all-pieces": (dict(dim=2, n=(256, 256, 1), real="double"), 0),
    "2d-jacobi-tail16": (dict(dim=2, n=(256, 256, 1), real="double"), 16),
    "2d-jacobi-tail8": (dict(dim=2, n=(256, 256, 1), real="double"), 8),
    "2d-jacobi-tail4": (dict(dim=2, n=(256, 256, 1), real="double"), 4),
    "2d-jacobi-tail2": (dict(dim=2, n=(256, 256, 1), real="double"), 2),
    "2d-jacobi-f32-all-pieces": (dict(dim=2, n=(256, 256, 1), real="float"), 0),
    "2d-jacobi-64-all-pieces": (dict(dim=2, n=(64, 64, 1), real="double"), 0),
    "2d-jacobi-warm-all-pieces": (dict(dim=2, n=(256, 256, 1), real="double", coarse_init="warm"), 0),
    "2d-jacobi-noerr-all-pieces": (dict(dim=2, n=(256, 256, 1), real="double", err_mode=0), 0),
    "2d-rbgs-all-pieces": (dict(dim=2, n=(256, 256, 1), real="double", smoother="rbgs", nu1=2, nu2=2,
                                prolong="linear", coarse_bc="consistent"), 0),
    "3d-jacobi-all-pieces": (dict(dim=3, n=(64, 64, 64), real="float"), 0),
}


def run(kw, size, churn):
    if churn:
        t = torch.randn((32 << 20,), dtype=torch.float64, device="cuda:0")
        torch.cuda.synchronize()
        del t
        torch.cuda.empty_cache()
    ctx = mg.Context(mg.make_opts(device=0, **kw))
    ctx.set_coarse_level(size)
    ctx.init_point_charge()
    out = []
    for _ in range(CYC):
        e = ctx.cycles(1)[0]
        out.append((e, ctx.get_psi()))
    ctx.close()
    return out


sel = os.environ.get("CONFIGS")
for name, (kw, size) in CONFIGS.items():
    if sel and name not in sel.split(","):
        continue
    ref = run(kw, size, False)
    bad = []
    for t in range(TRIALS):
        got = run(kw, size, t % 2 == 0)
        for cyc, ((er, pr), (eg, pg)) in enumerate(zip(ref, got)):
            if not (er == eg or (er != er and eg != eg)) or not np.array_equal(pr, pg):
                bad.append((t, cyc, er == eg, float(np.nanmax(np.abs(pr - pg)))))
                break
    print(f"{name}: {len(bad)} of {TRIALS} trials disagree {bad}", flush=True)
