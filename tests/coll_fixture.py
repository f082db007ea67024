"""Fixtures of the collision-driven objectives (the reference demo's path,
src/main.cpp): the demo's 4-segment vertex set and parameters, and synthetic
occupancy maps standing in for its private supereight map (main.cpp:17-19,
a "forest"; the file is not in the reference).

Maps are dense float32 grids [nz, ny, nx] of log-odds (occupied iff >= 0) with
voxel (x, y, z) covering [x, x+1) * res etc. from the world origin, the
layout of mtg_collision_cost."""
import numpy as np

import pyoracle

N, R, D = 10, 4, 3
M = N // 2

# main.cpp:26-53 (start, middle1..3, end); makeStartOrEnd fixes derivatives
# 0..SNAP at the start and end vertex.
MAIN_POSITIONS = np.array([[2.7, 9.5, 4.8], [3.50796, 4.34802, 4.56653],
                           [3.95552, 3.23008, 4.75131], [5.06673, 2.31032, 4.79433],
                           [7.0, 2.2, 4.8]])
MAIN_RADII = np.full((4, 2), 0.15)  # main.cpp:56-67

# main.cpp:75-110 (the fields the collision objective reads).
MAIN_PARAMS = dict(max_iterations=25, f_rel=1e-6, x_rel=0.01, soft_constraint_weight=100.0,
                   initial_stepsize_rel=0.1, w_d=50.0, w_c=50.0, w_t=0.1, w_sc=1.0,
                   increment_time=1e-6, epsilon=0.3, coll_pot_multiplier=20.0,
                   is_collision_safe=True, simple_numgrad_time=True,
                   simple_numgrad_constraints=True, coll_check_time_increment=0.1,
                   is_coll_raise_first_iter=True, robot_radius=0.15, add_coll_raise=1e-7,
                   map_resolution=0.1, min_bound=(1.4, 1.4, 3.9), max_bound=(11.3, 11.3, 8.8))


def coll_params(**over):
    """MAIN_PARAMS as keys of COLL_DEFAULTS (the objective's fields)."""
    keys = set(pyoracle.COLL_DEFAULTS)
    d = {k: v for k, v in MAIN_PARAMS.items() if k in keys}
    d.update(over)
    return d


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


def _dist_to_polyline(c, pts):
    best = np.inf
    for a, b in zip(pts[:-1], pts[1:]):
        ab = b - a
        u = np.clip(np.dot(c - a, ab) / np.dot(ab, ab), 0.0, 1.0)
        best = min(best, np.linalg.norm(c - (a + u * ab)))
    return best


# Beside the demo's QCQP path, about 0.6 m from it: the potential is non-zero
# there (distance - robot_radius <= epsilon) without a collision.
NEAR_TREES = ((3.73, 6.57), (4.28, 3.60), (6.74, 2.78))


def forest_map(seed=7, n_trees=40, res=0.1, extent=(12.0, 12.0, 9.0), radius=0.25,
               near=NEAR_TREES, clearance=1.2):
    """Vertical cylinders ("trees") of `radius` metres: `near` places some
    beside the demo path, the rest are random and at least `clearance`
    metres from the demo's vertex polyline.  Returns float32 [nz, ny, nx]."""
    rng = np.random.default_rng(seed)
    poly = MAIN_POSITIONS[:, :2]
    nx, ny, nz = (int(round(e / res)) for e in extent)
    occ = np.full((nz, ny, nx), -1.0, np.float32)
    xs = (np.arange(nx) + 0.5) * res
    ys = (np.arange(ny) + 0.5) * res
    X, Y = np.meshgrid(xs, ys)  # [ny, nx]
    centres = [np.array(c) for c in near]
    while len(centres) < n_trees:
        c = rng.uniform(1.6, 11.0, size=2)
        if _dist_to_polyline(c, poly) > clearance:
            centres.append(c)
    col = np.zeros((ny, nx), bool)
    for c in centres:
        col |= (X - c[0]) ** 2 + (Y - c[1]) ** 2 <= radius ** 2
    occ[:, col] = rng.uniform(0.0, 3.0, size=(nz, int(col.sum()))).astype(np.float32)
    return occ


def perturbed_starts(x0, n, scale, seed=11):
    rng = np.random.default_rng(seed)
    return [x0 + scale * rng.standard_normal(x0.shape) * (1.0 + np.abs(x0)) for _ in range(n)]
