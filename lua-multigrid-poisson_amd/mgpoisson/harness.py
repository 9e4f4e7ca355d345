"""Benchmark harness and convergence report in the reference's formats.

``python -m mgpoisson.harness bench`` reproduces test/test.lua:8-63.  For sizes 2^lo .. 2^hi it
constructs the solver with the positional protocol ``MG(size, real, cpuDepth)``, times
``mg:run()`` (two outer iterations, cpu-raw.lua:239-258), keeps the best of ``--tries`` and
writes ``#size<TAB>col...`` rows to ``cpu-vs-gpu.txt``.  The reference times with ``os.clock``
(CPU time); this harness uses wall-clock time with a device synchronisation, since the work runs
on the GPU.  The reference's harness calls ``run`` on ``multigrid-poisson.cpu``, which only has
``solve``.  Here every column is a solver whose class has ``run``.

The reference's table is cpu against gpu (its column list, test/test.lua:8-14, is 'cpu', 'cpu-raw', 'gpu',
...).  The GPU columns are built in (``COLUMNS``); CPU columns are plugged in by the caller, because this
package holds no CPU solver (there is deliberately no CPU fallback): ``register_column(name, factory)`` or
``--plugin module`` (a module whose ``columns()`` returns ``{name: factory}``), where
``factory(size, real, cpudepth)`` returns an object with ``run()``.  The reference's own Lua classes
bound from Python, or the test suite's C restatement of cpu-raw.lua (tests/harness_columns.py: column
``cpu-raw``), fit that slot.

``python -m mgpoisson.harness converge`` reproduces the multigrid half of
test/converge-multigrid-vs-krylov.lua:15-89.  For sizes 4 .. 128 it runs ``solve()`` with
``epsilon = 1e-20`` and records ``|psi|_inf`` per iteration from the ``errorCallback``.  It adds a
conjugate-gradient column on the same system (the reference's ``solver.conjgrad`` with
``x0 = -f``, ``b = f``, ``A`` = the 5-point operator with zero ghosts), computed on the device by
``mgp_cg_solve`` (matrix-free CG, fp64 dot products) as the cross-check.  Both columns are shifted by
their common minimum and written to ``converge/<size>.txt``.
"""
from __future__ import annotations

import argparse
import importlib
import os
import sys
import time

import numpy as np

COLUMNS = {
    # column name -> (real, build options); 'hip' is the reference configuration on the GPU
    "hip": ("double", {}),
    # gpu.lua's float column (test/test.lua's 'gpu'): every operation in float (gpu.lua:32); cpu-raw.lua's float
    # arithmetic (double expressions over float images) is the 'hip-raw-f32' column
    "hip-f32": ("float", dict(arith="real")),
    "hip-raw-f32": ("float", dict(arith="double")),
    "hip-rbgs": ("double", dict(smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent")),
}
# caller-supplied columns: name -> factory(size, real, cpudepth) returning an object with run()
EXTRA_COLUMNS = {}


def register_column(name, factory):
    """Add a column (e.g. a CPU solver of the positional protocol, test/test.lua:8-14's 'cpu' / 'cpu-raw')."""
    EXTRA_COLUMNS[name] = factory


def _make(col, size, cpudepth):
    if col in EXTRA_COLUMNS:
        return EXTRA_COLUMNS[col](size, None, cpudepth)  # test/test.lua:54: cl(size, nil, cpudepth)
    from .solver import MultigridHIPRaw

    real, build = COLUMNS[col]
    return MultigridHIPRaw(size, real, cpudepth, **build)


def bench(lo=5, hi=10, tries=1, cols=("hip",), cpudepth=3, out="cpu-vs-gpu.txt", quiet=False):
    """test/test.lua: best-of-tries wall time of MG(size, real, cpudepth):run() per size and column."""
    rows = []
    with open(out, "w") as fh:
        def write(s):
            fh.write(s)
            fh.flush()
            if not quiet:
                sys.stdout.write(s)
                sys.stdout.flush()

        write("#size" + "".join("\t" + c for c in cols) + "\n")
        for log2size in range(lo, hi + 1):
            size = 1 << log2size
            write(str(size))
            row = [size]
            for col in cols:
                best = float("inf")
                for _ in range(tries):
                    mg = _make(col, size, cpudepth)
                    mg.quiet = True
                    t0 = time.perf_counter()
                    mg.run()
                    ctx = getattr(mg, "ctx", None)
                    if ctx is not None:
                        ctx.sync()
                    best = min(best, time.perf_counter() - t0)
                    if ctx is not None:
                        ctx.close()
                write(f"\t{best}")
                row.append(best)
            write("\n")
            rows.append(row)
    return rows


def converge(sizes=(4, 8, 16, 32, 64, 128), epsilon=1e-20, outdir="converge", maxiter=1000, quiet=False,
             cg_maxiter=20000):
    """converge-multigrid-vs-krylov.lua: |psi|_inf per multigrid iteration next to CG's (both on the GPU)."""
    from .solver import MultigridHIP

    os.makedirs(outdir, exist_ok=True)
    report = {}
    for size in sizes:
        if not quiet:
            print(f"solving for size {size}")
        data = []
        mg = None

        def cb(it, err):
            data.append(float(np.max(np.abs(mg.psi))))
            return False

        mg = MultigridHIP(size=size, epsilon=epsilon, errorCallback=cb, maxiter=maxiter)
        mg.solve()
        # the conjugate-gradient column on the device (mgp_cg_solve: x0 = -f, b = f, converge...lua:38-69)
        _, _, _, hist = mg.ctx.cg_solve(epsilon=epsilon, maxiter=cg_maxiter, history=True)
        cg = [float(v) for v in hist]
        n = max(len(data), len(cg))
        cols = [data + [float("nan")] * (n - len(data)), cg + [float("nan")] * (n - len(cg))]
        finite = [v for c in cols for v in c if np.isfinite(v)]
        lo = min(finite) if finite else 0.0
        with open(os.path.join(outdir, f"{size}.txt"), "w") as fh:
            fh.write("\n".join("\t".join(repr(c[i] - lo) for c in cols) for i in range(n)))
        report[size] = (data, cg)
    return report


def main(argv=None):
    p = argparse.ArgumentParser(prog="python -m mgpoisson.harness")
    sub = p.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("bench", help="test/test.lua: TSV of best-of-tries run() times")
    b.add_argument("--lo", type=int, default=5)
    b.add_argument("--hi", type=int, default=10)
    b.add_argument("--tries", type=int, default=1)
    b.add_argument("--cols", default="hip", help="comma list of " + ",".join(COLUMNS) + " and plugged-in columns")
    b.add_argument("--plugin", action="append", default=[],
                   help="module whose columns() returns {name: factory(size, real, cpudepth)} (e.g. a CPU solver)")
    b.add_argument("--cpudepth", type=int, default=3)
    b.add_argument("--out", default="cpu-vs-gpu.txt")
    c = sub.add_parser("converge", help="converge-multigrid-vs-krylov.lua: |psi|_inf histories")
    c.add_argument("--sizes", default="4,8,16,32,64,128")
    c.add_argument("--epsilon", type=float, default=1e-20)
    c.add_argument("--outdir", default="converge")
    a = p.parse_args(argv)
    if a.cmd == "bench":
        for mod in a.plugin:
            for name, factory in importlib.import_module(mod).columns().items():
                register_column(name, factory)
        bench(a.lo, a.hi, a.tries, tuple(a.cols.split(",")), a.cpudepth, a.out)
    else:
        converge(tuple(int(s) for s in a.sizes.split(",")), a.epsilon, a.outdir)


if __name__ == "__main__":
    main()
