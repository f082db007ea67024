"""Fixtures of the collision-driven objectives (the reference demo's path,
src/main.cpp): the demo's 4-segment vertex set and parameters, and synthetic
occupancy maps standing in for its private supereight map (main.cpp:17-19,
a "forest"; the file is not in the reference).

Maps are dense float32 grids [nz, ny, nx] of log-odds (occupied iff >= 0) with
voxel (x, y, z) covering [x, x+1) * res etc. from the world origin, the
layout of mtg_collision_cost."""
import numpy as np

import pyoracle
# The demo's geometry, parameters and synthetic map are product-side data
# (mav_tube_trajectory_generation_amd/demo.py, also used by bench.py).
from mav_tube_trajectory_generation_amd.demo import (MAIN_PARAMS, MAIN_POSITIONS,  # noqa: F401
                                                     MAIN_RADII, NEAR_TREES, coll_params,
                                                     forest_map, perturbed_starts)

N, R, D = 10, 4, 3
M = N // 2


def vertices_with_positions(positions):
    """Vertices of the demo: start/end fixed to derivative 0..M-1 (rest), the
    intermediate vertices fixing only their position."""
    S = len(positions) - 1
    mask = np.zeros((S + 1, M), np.uint8)
    vals = np.zeros((S + 1, M, D))
    mask[0, :] = mask[S, :] = 1
    mask[1:S, 0] = 1
    vals[:, 0, :] = positions
    return pyoracle.Vertices(mask, vals)


def tube_pattern(v):
    """The fork's nonlinear problem: every intermediate derivative free, the
    positions included (setupConstraintReorderingMatrixkDim, qcqp_impl:18-118)."""
    mask = v.mask.copy()
    mask[1:v.S, :] = 0
    return pyoracle.Vertices(mask, v.vals)


def main_problem():
    """(vertices with positions, tube-pattern vertices, segment times,
    initial x = the tube QCQP solution's d_p) of main.cpp."""
    v = vertices_with_positions(MAIN_POSITIONS)
    t = pyoracle.estimate_segment_times(v, 2.0, 2.0)  # main.cpp:51-53
    sol = pyoracle.tube_solve(N, R, v, t, MAIN_RADII)
    return v, tube_pattern(v), t, sol["x"]
