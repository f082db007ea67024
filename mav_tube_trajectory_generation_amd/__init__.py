"""MI355X-native batched polynomial trajectory optimizer.

Drop-in for the linear-constrained / tube-QCQP solve path of
NilsFunk/mav_tube_trajectory_generation.  The product is libmtg_hip.so
(hand-written gfx950 HIP kernels behind the C ABI in include/mtg_hip.h) and
the C++ host API in include/mav_tube_trajectory_generation_amd/.  This Python
package is the batched front end used by tests and bench.py.
"""
from ._abi import (COLL_DEFAULTS, LIB_PATH, MTGError, lib, make_coll_params,  # noqa: F401
                   make_collision_params, make_time_params)
from .batch import (Context, LinearPlan, coll_field, generate_random_problems,  # noqa: F401
                    magnitude_candidates,
                    max_magnitude,
                    min_max_magnitude, sample_trajectories, segment_matrices, soft_constraint_cost,
                    tube_num_constraints, tube_residuals, tube_solve, tube_time_cost,
                    tube_time_optimize, tube_time_workspace_bytes)

__all__ = ["Context", "LinearPlan", "MTGError", "coll_field", "generate_random_problems",
           "magnitude_candidates",
           "max_magnitude",
           "min_max_magnitude", "make_coll_params", "make_collision_params", "make_time_params",
           "COLL_DEFAULTS",
           "sample_trajectories", "segment_matrices", "soft_constraint_cost",
           "tube_num_constraints", "tube_residuals", "tube_solve", "tube_time_cost",
           "tube_time_optimize", "tube_time_workspace_bytes", "lib", "LIB_PATH"]
