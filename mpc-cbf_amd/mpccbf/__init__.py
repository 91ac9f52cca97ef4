"""Python host binding of libmpccbf.so (include/mpccbf.h) — the MI355X batched MPC-CBF solver.

The product is the C ABI + HIP kernels; this module only marshals torch device tensors (device
memory, streams) into it. There is no CPU fallback: without the built library, or without a
GPU, every solve raises.
"""
from ._lib import (  # noqa: F401
    LIB_PATH, MpccbfError, Params, Options, Context, status_name, build_library, load,
    dense_qp_solve, dense_qp_solve_batch, STATUS_NAMES, OPTIMAL, FEASIBLE, UNBOUNDED, INFEASIBLE, ERROR, UNKNOWN,
    INFEASIBLEORUNBOUNDED, Comm, comm_unique_id, fov_control_solve, fov_control_params,
    connectivity_control_solve,
)
from . import swarm  # noqa: F401
