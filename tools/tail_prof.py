#!/usr/bin/env python3
"""Timing experiment: run one 512^3 V-cycle with a TAIL_PROF library (MGP_LIBRARY) and print the
shader cycles of each k_tail op (written into f of the first tail level, plane 0, colour 0)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lua-multigrid-poisson_amd"))
import mgpoisson as M  # noqa: E402
import mgpoisson._lib as L  # noqa: E402

from mgpoisson.context import make_opts  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
ctx = M.Context(make_opts(dim=3, n=(n, n, n), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
                          coarse_bc="consistent"))
ctx.init_point_charge()
for _ in range(3):
    ctx.cycle()
lv = [i for i, x in enumerate(ctx.levels) if x["nx"] == 16][0]
f = ctx.get_field(L.FIELD_F, lv)
vals = [f[0, j, 2 * m + (j & 1)] for j in range(16) for m in range(8)]
tot = 0
for i, v in enumerate(vals):
    if v == 0:
        break
    tot += v
    print(i, int(v))
print("total cycles", int(tot), "us at 2.4 GHz ~", tot / 2400, "(s_memtime ticks at 100 MHz:", tot / 100, "us)")
