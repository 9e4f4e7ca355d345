"""mgpoisson — MI355X-native multigrid Poisson solver (host layer over libmgpoisson.so).

Importing this package loads the HIP library and fails loudly if it is missing.
"""
from ._lib import (FIELD_CORRECTION, FIELD_ERROR, FIELD_F, FIELD_PSI_OLD, FIELD_RESIDUAL, FIELD_TMP,  # noqa: F401
                   FIELD_U, MGPError, comm_unique_id, copy_bandwidth, default_opts, plan, plan_comm)
from .context import Context, Group, Loopback, make_opts  # noqa: F401
from .solver import MultigridHIP, MultigridHIPHybrid, MultigridHIPRaw  # noqa: F401

__all__ = ["Context", "Group", "Loopback", "MGPError", "MultigridHIP", "MultigridHIPHybrid", "MultigridHIPRaw", "comm_unique_id", "copy_bandwidth",
           "default_opts", "make_opts", "plan", "plan_comm"]
