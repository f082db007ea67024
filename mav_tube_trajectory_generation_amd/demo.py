"""The reference's demo problem (src/main.cpp) as data: its 4-segment vertex
set, tube radii and optimiser parameters (main.cpp:26-110), the segment-time
estimate it uses (estimateSegmentTimes, vertex.cpp:252-269), and a synthetic
occupancy map standing in for its private supereight "forest" map
(main.cpp:17-19; the map file is not in the reference).

Used by bench.py's collision workload and by the tests' fixtures.  Maps are
dense float32 grids [nz, ny, nx] of log-odds (occupied iff >= 0), voxel
(x, y, z) covering [x, x+1) * res etc. from the world origin: the layout of
mtg_collision_cost / mtg_coll_optimize.
"""
import numpy as np

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
    """MAIN_PARAMS restricted to the collision objective's fields
    (mav_tube_trajectory_generation_amd.COLL_DEFAULTS), with overrides."""
    from ._abi import COLL_DEFAULTS
    d = {k: v for k, v in MAIN_PARAMS.items() if k in COLL_DEFAULTS}
    d.update(over)
    return d


def estimate_segment_times(positions, v_max, a_max, magic_fabian_constant=6.5):
    """estimateSegmentTimes (vertex.cpp:252-269, the Nfabian estimate main.cpp
    uses): t = d / v_max * 2 * (1 + c v_max / a_max exp(-d / v_max * 2))."""
    p = np.asarray(positions, dtype=np.float64)
    d = np.linalg.norm(np.diff(p, axis=0), axis=1)
    return d / v_max * 2.0 * (1.0 + magic_fabian_constant * v_max / a_max *
                              np.exp(-d / v_max * 2.0))


def tube_pattern(positions):
    """The fork's nonlinear problem over the demo vertices: start and end
    fix derivatives 0..M-1 (position, rest), every intermediate derivative is
    free, positions included (setupConstraintReorderingMatrixkDim,
    qcqp_impl:18-118).  Returns (mask [(S+1), M], fixed values [D, 2M] in
    (vertex, derivative) order)."""
    p = np.asarray(positions, dtype=np.float64)
    S = p.shape[0] - 1
    mask = np.zeros((S + 1, M), np.uint8)
    mask[0, :] = mask[S, :] = 1
    df = np.zeros((D, 2 * M))
    df[:, 0] = p[0]
    df[:, M] = p[S]
    return mask, df


NEAR_TREES = ((3.73, 6.57), (4.28, 3.60), (6.74, 2.78))


def _dist_to_polyline(c, pts):
    best = np.inf
    for a, b in zip(pts[:-1], pts[1:]):
        ab = b - a
        u = np.clip(np.dot(c - a, ab) / np.dot(ab, ab), 0.0, 1.0)
        best = min(best, np.linalg.norm(c - (a + u * ab)))
    return best


def forest_map(seed=7, n_trees=40, res=0.1, extent=(12.0, 12.0, 9.0), radius=0.25,
               near=NEAR_TREES, clearance=1.2):
    """Vertical cylinders ("trees") of `radius` metres: `near` places some
    about 0.6 m beside the demo path (the potential is non-zero there without
    a collision), the rest are random and at least `clearance` metres from the
    demo's vertex polyline.  Returns float32 [nz, ny, nx]."""
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
    """n copies of x0 with relative Gaussian perturbations of `scale`."""
    rng = np.random.default_rng(seed)
    return [x0 + scale * rng.standard_normal(x0.shape) * (1.0 + np.abs(x0)) for _ in range(n)]
