"""ctypes binding of libmgpoisson.so (include/mgpoisson.h).

The product path: every call goes to the HIP library.  There is no CPU fallback — if the
library is missing this module raises at import time, and if no GPU is present
``mgp_create`` fails with MGP_ERR_HIP, which surfaces as :class:`MGPError`.

HIP runtime note: ``import torch`` loads PyTorch's own copy of libamdhip64.so.7 (and
librccl.so.1).  To keep ONE HIP runtime per process, torch is imported (when installed)
before the library is loaded, so that the library binds to the already-loaded copies by
SONAME instead of loading /opt/rocm's second copy beside them.
"""
from __future__ import annotations

import ctypes
import os

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the product path
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MGP_LIBRARY", os.path.join(_HERE, "libmgpoisson.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libmgpoisson.so not found at {LIB_PATH}: the HIP extension is not built. "
        "Run `python -c 'import __graft_entry__ as g; g.build()'` from the repo root "
        "(there is deliberately no CPU fallback)."
    )

lib = ctypes.CDLL(LIB_PATH)

MGP_OK = 0
STATUS = {-1: "MGP_ERR_ARG", -2: "MGP_ERR_HIP", -3: "MGP_ERR_RCCL", -4: "MGP_ERR_OOM", -5: "MGP_ERR_STATE"}
JACOBI, RBGS, GS_LEX = 0, 1, 2
CYCLE_V, CYCLE_F = 0, 1
PROLONG_PC, PROLONG_LINEAR = 0, 1
COARSE_FRESH, COARSE_WARM = 0, 1
BC_ZERO, BC_CONSISTENT = 0, 1
RESTRICT_AVERAGE, RESTRICT_FULL_WEIGHTING = 0, 1
ARITH_REAL, ARITH_DOUBLE = 0, 1
API_VERSION = 3
FIELD_U, FIELD_F = 0, 1
FIELD_RESIDUAL, FIELD_CORRECTION, FIELD_PSI_OLD, FIELD_ERROR, FIELD_TMP = 2, 3, 4, 5, 6
# cpu-raw.lua:148-171 names of the level fields (Vs/Rs are U/F below the finest level)
FIELDS = {"psi": FIELD_U, "f": FIELD_F, "Vs": FIELD_U, "Rs": FIELD_F, "rs": FIELD_RESIDUAL, "vs": FIELD_CORRECTION,
          "psiOld": FIELD_PSI_OLD, "errorBuf": FIELD_ERROR, "tmpU": FIELD_TMP}
MEM_HOST, MEM_DEVICE = 0, 1
# int fn(void* user, double h, void* u, const void* f, int64_t size)
COARSE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_int64)
TIMING_HALF_SWEEP, TIMING_FUSED_PRE, TIMING_FUSED_POST, TIMING_EXCHANGE, TIMING_COLLECTIVE = 0, 1, 2, 3, 4
TIMING_KINDS = {TIMING_HALF_SWEEP: "half_sweep", TIMING_FUSED_PRE: "fused_pre", TIMING_FUSED_POST: "fused_post",
                TIMING_EXCHANGE: "exchange", TIMING_COLLECTIVE: "collective"}
COMM_OPS = {0: "exchange", 1: "allgather", 2: "allreduce"}
COMM_ID_BYTES = 128


class MGPOpts(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_int32),
        ("dim", ctypes.c_int32),
        ("n", ctypes.c_int64 * 3),
        ("real_bytes", ctypes.c_int32),
        ("nu1", ctypes.c_int32),
        ("nu2", ctypes.c_int32),
        ("smoother", ctypes.c_int32),
        ("cycle", ctypes.c_int32),
        ("prolong", ctypes.c_int32),
        ("coarse_init", ctypes.c_int32),
        ("coarse_bc", ctypes.c_int32),
        ("coarse_sweeps", ctypes.c_int32),
        ("err_mode", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("world", ctypes.c_int32),
        ("restriction", ctypes.c_int32),
        ("gather_cells", ctypes.c_int64),
        ("comm_id", ctypes.c_uint8 * COMM_ID_BYTES),
        ("arith", ctypes.c_int32),
        ("api_version", ctypes.c_int32),
    ]


_vp, _i32, _i64, _dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
_P = ctypes.POINTER

SIGNATURES = {
    "mgp_version": (ctypes.c_int, []),
    "mgp_opts_default": (None, [_P(MGPOpts)]),
    "mgp_comm_unique_id": (ctypes.c_int, [_vp, _i64]),
    "mgp_create": (ctypes.c_int, [_P(_vp), _P(MGPOpts)]),
    "mgp_loopback_create": (ctypes.c_int, [_P(_vp), ctypes.c_int]),
    "mgp_loopback_destroy": (None, [_vp]),
    "mgp_create_loopback": (ctypes.c_int, [_P(_vp), _P(MGPOpts), _vp]),
    "mgp_destroy": (None, [_vp]),
    "mgp_last_error": (ctypes.c_char_p, [_vp]),
    "mgp_num_levels": (ctypes.c_int, [_vp]),
    "mgp_level_info": (ctypes.c_int, [_vp, ctypes.c_int, _P(_i64)]),
    "mgp_plan": (ctypes.c_int, [_P(MGPOpts), _P(_i64), ctypes.c_int]),
    "mgp_init_point_charge": (ctypes.c_int, [_vp]),
    "mgp_set_field": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, _i64, ctypes.c_int]),
    "mgp_get_field": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, _i64, ctypes.c_int]),
    "mgp_cycle": (ctypes.c_int, [_vp, _P(_dbl)]),
    "mgp_cycles": (ctypes.c_int, [_vp, _i32, _P(_dbl)]),
    "mgp_two_grid": (ctypes.c_int, [_vp, _dbl, _vp, _vp, _i64, ctypes.c_int]),
    "mgp_set_planes": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _i64, _i64, _vp, ctypes.c_int]),
    "mgp_get_planes": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _i64, _i64, _vp, ctypes.c_int]),
    "mgp_field_stats": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _P(ctypes.c_uint64), _P(_dbl)]),
    "mgp_smooth": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    "mgp_residual_restrict": (ctypes.c_int, [_vp, ctypes.c_int]),
    "mgp_prolong_correct": (ctypes.c_int, [_vp, ctypes.c_int]),
    "mgp_coarse_solve": (ctypes.c_int, [_vp]),
    "mgp_sync": (ctypes.c_int, [_vp]),
    "mgp_metrics": (ctypes.c_int, [_vp, _P(_dbl), _P(_i64), _P(_dbl)]),
    "mgp_set_coarse_level": (ctypes.c_int, [_vp, _i64]),
    "mgp_residual_norm": (ctypes.c_int, [_vp, ctypes.c_int, _P(_dbl), _P(_dbl)]),
    "mgp_cg_solve": (ctypes.c_int, [_vp, _dbl, _i32, _vp, ctypes.c_int, _P(_i32), _P(_dbl), _P(_dbl)]),
    "mgp_set_coarse_handoff": (ctypes.c_int, [_vp, _i64, COARSE_FN, _vp]),
    "mgp_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
    "mgp_set_debug": (ctypes.c_int, [_vp, ctypes.c_int]),
    "mgp_timing_read": (ctypes.c_int, [_vp, ctypes.c_int, _P(_dbl), _P(_i64), _P(_dbl)]),
    "mgp_timing_kernel": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, _P(_i64)]),
    "mgp_comm_log": (ctypes.c_int, [_vp, _P(_i64), ctypes.c_int, ctypes.c_int]),
    "mgp_plan_comm": (ctypes.c_int, [_P(MGPOpts), _i32, _P(_i64), ctypes.c_int]),
    "mgp_copy_bandwidth": (ctypes.c_int, [ctypes.c_int, _i64, _i32, _P(_dbl)]),
    "mgp_group_create": (ctypes.c_int, [_P(_vp), _P(MGPOpts), ctypes.c_int, _P(ctypes.c_int)]),
    "mgp_group_destroy": (None, [_vp]),
    "mgp_group_last_error": (ctypes.c_char_p, [_vp]),
    "mgp_group_size": (ctypes.c_int, [_vp]),
    "mgp_group_rank": (_vp, [_vp, ctypes.c_int]),
    "mgp_group_init_point_charge": (ctypes.c_int, [_vp]),
    "mgp_group_cycle": (ctypes.c_int, [_vp, _P(_dbl)]),
    "mgp_group_cycles": (ctypes.c_int, [_vp, _i32, _P(_dbl)]),
    "mgp_group_set_field": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, _i64, ctypes.c_int]),
    "mgp_group_get_field": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, _i64, ctypes.c_int]),
    "mgp_group_residual_norm": (ctypes.c_int, [_vp, ctypes.c_int, _P(_dbl), _P(_dbl)]),
    "mgp_group_field_stats": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _P(ctypes.c_uint64), _P(_dbl)]),
}

for _name, (_res, _args) in SIGNATURES.items():
    _fn = getattr(lib, _name)  # AttributeError here = library/header skew: fail loudly
    _fn.restype = _res
    _fn.argtypes = _args


class MGPError(RuntimeError):
    """A negative mgp_status from the library, with mgp_last_error's message."""

    def __init__(self, code: int, message: str):
        super().__init__(f"{STATUS.get(code, code)}: {message}")
        self.code = code


def check(code: int, ctx=None) -> int:
    if code < 0:
        msg = lib.mgp_last_error(ctx)
        raise MGPError(code, msg.decode() if msg else "")
    return code


def check_group(code: int, group=None) -> int:
    if code < 0:
        msg = lib.mgp_group_last_error(group)
        raise MGPError(code, msg.decode() if msg else "")
    return code


def default_opts() -> MGPOpts:
    o = MGPOpts()
    lib.mgp_opts_default(ctypes.byref(o))
    return o


def comm_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
    check(lib.mgp_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p), COMM_ID_BYTES))
    return bytes(buf)


def plan(opts: MGPOpts, max_levels: int = 48):
    """Host-only level plan: list of dicts (nx, ny, nz_global, nz_local, z0, distributed, engine), engine =
    how mgp_create would run the level's phases ("piece", "tail", "zs", "blk", "zpost": PRE per piece, POST k_zs)."""
    rows = (ctypes.c_int64 * (8 * max_levels))()
    n = check(lib.mgp_plan(ctypes.byref(opts), rows, max_levels))
    keys = ("nx", "ny", "nz_global", "nz_local", "z0", "distributed")
    out = [dict(zip(keys, [rows[8 * l + i] for i in range(6)])) for l in range(n)]
    for l, d in enumerate(out):
        d["engine"] = ("piece", "tail", "zs", "blk", "zpost")[rows[8 * l + 6]]
    return out


def plan_comm(opts: MGPOpts, cycles: int = 1, max_rows: int = 1 << 14):
    """Host-only schedule of the exchanges / collectives a rank with these options issues in `cycles` outer
    iterations (mgp_plan_comm): [(op, side, level, msgs, bytes)], as Context.comm_log reports them."""
    rows = (ctypes.c_int64 * (5 * max_rows))()
    n = check(lib.mgp_plan_comm(ctypes.byref(opts), int(cycles), rows, max_rows))
    return [(COMM_OPS[rows[5 * i]],) + tuple(rows[5 * i + k] for k in range(1, 5)) for i in range(min(n, max_rows))]


def copy_bandwidth(device: int = -1, nbytes: int = 2 << 30, reps: int = 10) -> float:
    """Measured 16-byte streaming copy bandwidth of the device in GB/s (read + write bytes, best of reps)."""
    g = ctypes.c_double()
    check(lib.mgp_copy_bandwidth(int(device), int(nbytes), int(reps), ctypes.byref(g)))
    return g.value
