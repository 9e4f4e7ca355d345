#!/usr/bin/env python3
"""Timing experiment: run cycles with a TC_PROF library (MGP_LIBRARY) and print the wall-clock ticks
(100 MHz) of each k_tail_c op, read back from f of the first tail level (rows 0-1: ticks, rows 2-3: op code).
usage: tools/tail_prof_c.py dim n"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lua-multigrid-poisson_amd"))
import mgpoisson as M  # noqa: E402
import mgpoisson._lib as L  # noqa: E402

from mgpoisson.context import make_opts  # noqa: E402

dim = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
box = (n, n, n) if dim == 3 else (n, n, 1)
ctx = M.Context(make_opts(dim=dim, n=box, real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
                          coarse_bc="consistent"))
ctx.init_point_charge()
for _ in range(3):
    ctx.cycle()
top = 16 if dim == 3 else 64
lv = [i for i, x in enumerate(ctx.levels) if x["nx"] == top][0]
f = ctx.get_field(L.FIELD_F, lv)
plane = f[0] if dim == 3 else f
names = {1: "smooth", 2: "rr", 3: "zero", 4: "prolong"}
tot = 0
for q in range(2 * top):
    t = plane[q // top, q % top]
    code = int(plane[2 + q // top, q % top])
    if code == 0:
        break
    code -= 1
    tot += t
    print(q, f"{names.get(code & 15, code & 15)} level {code >> 4}", int(t), "ticks", f"{t / 100:.2f} us")
print("total", int(tot), "ticks =", tot / 100, "us")
