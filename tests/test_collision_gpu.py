"""Collision cost over an occupancy map (mtg_collision_cost; SURVEY.md 8f
rank 4: getCostAndGradientCollision, nonlinear_impl:1609-1780, with the
nearest-occupied search of :1782-2043 and getCostPotential :2660-2684)
against the oracle restatement on the same dense grid.  supereight is absent,
so parity with the reference's octree is unpinned; the oracle follows the
reference's arithmetic with the dense grid in place of the octree."""
import numpy as np
import pytest

from helpers import compact_fixed, rel_err, standard_vertices

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N, R, D = 10, 4, 3
OFFSET = 20.0  # trajectories in the positive octant of a [0, 40)^3 map


def _map(seed, n=160, n_obst=6000, n_blob=30):
    rng = np.random.default_rng(seed)
    occ = np.full((n, n, n), -1.0, np.float32)
    idx = rng.integers(0, n, size=(n_obst, 3))
    occ[idx[:, 2], idx[:, 1], idx[:, 0]] = rng.uniform(0.0, 2.0, n_obst)
    for _ in range(n_blob):  # a few solid blocks
        c = rng.integers(10, n - 10, size=3)
        occ[c[2] - 2:c[2] + 3, c[1] - 2:c[1] + 3, c[0] - 2:c[0] + 3] = 1.0
    return occ


def _problems(oracle, S, seeds, pattern):
    vs, ts = [], []
    for sd in seeds:
        v = standard_vertices(N, S, D, sd)
        v.vals[:, 0, :] += OFFSET
        t = oracle.estimate_segment_times(v, 3.0, 5.0)
        if pattern == "tube":
            v.mask[1:S, :] = 0
        vs.append(v)
        ts.append(t)
    return vs, np.array(ts)


@pytest.mark.parametrize("pattern,radius,n_obst", [("standard", 0.1, 6000),
                                                   ("tube", 0.1, 6000),
                                                   ("standard", 0.6, 600)])
def test_collision_cost_vs_oracle(ctx, dev, oracle, pattern, radius, n_obst):
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 6, 24
    vs, times = _problems(oracle, S, range(300, 300 + B), pattern)
    mask, _ = compact_fixed(vs[0], N)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    occ = _map(5, n_obst=n_obst, n_blob=n_obst // 200)
    prm = dict(map_resolution=0.25, min_bound=[0.0] * 3, max_bound=[40.0] * 3, epsilon=0.5,
               robot_radius=radius, coll_pot_multiplier=1.0, coll_check_time_increment=0.1)
    dps, coeffs = [], []
    for v, t in zip(vs, times):
        sol = oracle.linear_solve(N, R, v, t)
        dps.append(sol["dp"])
        coeffs.append(sol["coeffs"])
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    out = plan.collision_cost(T(np.array(coeffs)), T(times), T(occ),
                              mtg.make_collision_params(**prm))
    got = {k: v.cpu().numpy() for k, v in out.items()}
    n_coll = 0
    for b in range(B):
        J, c, gc, gf = oracle.collision_cost(N, R, vs[b], times[b], dps[b], occ, prm)
        assert got["collision"][b] == c, b
        n_coll += c
        assert rel_err(got["cost"][b], J) <= 1e-9 or abs(got["cost"][b] - J) <= 1e-12, b
        sc = max(np.max(np.abs(gc)), 1e-300)
        assert np.max(np.abs(got["grad_coeffs"][b] - gc)) <= 1e-8 * sc, b
        sf = max(np.max(np.abs(gf)), 1e-300)
        assert np.max(np.abs(got["grad_free"][b] - gf)) <= 1e-7 * sf, b
    # the map yields both outcomes
    assert 0 < n_coll < B, n_coll


def test_collision_free_map_and_bounds(ctx, dev, oracle):
    """An empty map costs nothing; a map whose bounds the trajectory leaves
    reports a collision (is_valid_state, nonlinear_impl:1803-1811)."""
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 5, 4
    vs, times = _problems(oracle, S, range(40, 40 + B), "standard")
    mask, _ = compact_fixed(vs[0], N)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    coeffs = np.array([oracle.linear_solve(N, R, v, t)["coeffs"] for v, t in zip(vs, times)])
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    empty = np.full((8, 8, 8), -1.0, np.float32)
    ok = plan.collision_cost(T(coeffs), T(times), T(empty),
                             mtg.make_collision_params(0.25, [0.0] * 3, [40.0] * 3))
    assert (ok["collision"].cpu().numpy() == 0).all()
    assert (ok["cost"].cpu().numpy() == 0).all()
    tight = plan.collision_cost(T(coeffs), T(times), T(empty),
                                mtg.make_collision_params(0.25, [OFFSET - 1.0] * 3,
                                                          [OFFSET + 1.0] * 3))
    assert (tight["collision"].cpu().numpy() == 1).all()
    assert (tight["grad_free"].cpu().numpy() == 0).all()
