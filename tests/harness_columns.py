"""CPU column of the TSV harness (TEST INFRASTRUCTURE ONLY): the C restatement of MultigridCPURaw.

test/test.lua:8-14 tabulates 'cpu' / 'cpu-raw' next to 'gpu'.  The product package holds no CPU solver,
so the test suite plugs its oracle in (``python -m mgpoisson.harness bench --plugin harness_columns``
with tests/ on the path, or ``harness.register_column``).  ``cpu-raw`` follows the positional protocol
MultigridCPURaw(size, real) (cpu-raw.lua:142-258): warm coarse buffers, Jacobi 7+7, injection, two
outer iterations in run(), real = 'float' with cpu-raw.lua's double arithmetic.
"""
from __future__ import annotations

from oracle_lib import Oracle


class CpuRaw:
    """MultigridCPURaw(size, real):run() on the host, one thread (cpu-raw.lua:102-114 loops)."""

    def __init__(self, size, real=None, cpudepth=None):
        real = real or "double"  # cpu-raw.lua:143
        self.o = Oracle(dim=2, n=(size, size, 1), real=real, arith="double", coarse_init="warm")
        self.o.init_point_charge()
        self.quiet = False

    def run(self):
        errs = []
        for it in range(1, 3):  # cpu-raw.lua:245
            errs.append(self.o.step())
            if not self.quiet:
                print(it, errs[-1])
            if not errs[-1] < float("inf") or errs[-1] < 1e-10:
                break
        return errs


def columns():
    return {"cpu-raw": CpuRaw}
