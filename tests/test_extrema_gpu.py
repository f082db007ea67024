"""GPU magnitude extrema (mtg_max_magnitude, mtg_soft_constraint_cost)
against the oracle's restatement of computeMaximumOfMagnitude
(linear_impl:455-487, segment.cpp:82-133, polynomial.cpp:32-81) and of
evaluateMaximumMagnitudeAsSoftConstraint (nonlinear_impl:2735-2766).

The oracle finds all roots (companion-matrix eigenvalues standing in for
Jenkins-Traub, pinned to numpy.roots in test_oracle.py); the kernel isolates
only the real roots in [0, T] by Bernstein subdivision.  Both evaluate the
magnitude at their roots, so values agree to rounding: 1e-10 relative.  The
argmax agrees exactly except where the maximum sits on a vertex, whose two
sides (end of segment s, start of s+1) are equal up to rounding and either
may win the reference's strict comparison.
"""
import math

import numpy as np
import pytest

from helpers import standard_vertices

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _problems(oracle, N, D, S, seeds, r=None):
    r = N // 2 - 1 if r is None else r
    vs = [standard_vertices(N, S, D, s) for s in seeds]
    times = np.stack([oracle.estimate_segment_times(v, 3.0, 5.0) for v in vs])
    coeffs = np.stack([oracle.linear_solve(N, r, v, t)["coeffs"] for v, t in zip(vs, times)])
    return coeffs, times


def _magnitude(c, t, k):
    from numpy.polynomial import polynomial as P
    return np.sqrt(sum(P.polyval(t, P.polyder(c[d], k) if k else c[d]) ** 2
                       for d in range(c.shape[0])))


def _check_argmax(got_t, got_s, ref, coeffs, times, k):
    """The reported (segment, time) attains the reference's value.  The
    segment equals the reference's, or the maximum sits on a vertex (end of
    s vs start of s + 1, equal up to rounding).  The time equals the
    reference's unless the maximum is flat (then any time attaining the value
    to rounding is the same extremum)."""
    if got_s != ref["segment"]:
        a, b = sorted([(got_s, got_t), (ref["segment"], ref["time"])])
        assert b[0] == a[0] + 1, (got_t, got_s, ref)
        assert abs(a[1] - times[a[0]]) <= 1e-9 * times[a[0]] and abs(b[1]) <= 1e-9, \
            (got_t, got_s, ref)
    assert 0.0 <= got_t <= times[got_s]
    val = _magnitude(coeffs[got_s], got_t, k)
    assert abs(val - ref["value"]) <= 1e-9 * max(ref["value"], 1e-300), (got_t, got_s, ref)


@pytest.mark.parametrize("N,D,S", [(10, 3, 10), (10, 1, 5), (10, 2, 3), (6, 3, 4), (8, 4, 6),
                                   (12, 3, 7), (4, 2, 3), (10, 3, 40)])
def test_max_magnitude_vs_oracle(ctx, dev, oracle, N, D, S):
    import mav_tube_trajectory_generation_amd as mtg
    seeds = list(range(700, 712))
    coeffs, times = _problems(oracle, N, D, S, seeds)
    cd = torch.from_numpy(coeffs).to(dev)
    td = torch.from_numpy(times).to(dev)
    for k in range(0, min(4, N - 2) + 1):
        out = mtg.max_magnitude(cd, td, k)
        torch.cuda.synchronize()
        t, v, s = (out[x].cpu().numpy() for x in ("time", "value", "segment"))
        for b in range(len(seeds)):
            ref = oracle.max_magnitude(N, coeffs[b], times[b], k)
            assert abs(v[b] - ref["value"]) <= 1e-10 * max(ref["value"], 1e-300), (N, D, S, k, b)
            _check_argmax(float(t[b]), int(s[b]), ref, coeffs[b], times[b], k)


def test_max_magnitude_full_batch_vs_sampling(ctx, dev):
    """Config-2 batch (1024 x 10 segments): the analytic maximum bounds the
    densely sampled magnitude from above and agrees within the reference
    test's 0.01 (test_polynomial_optimization.cpp:396-400); the reported
    time attains the value."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S, B = 10, 3, 10, 1024
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=105)
    plan = mtg.LinearPlan(ctx, N, D, 4, S, mask)
    td = torch.from_numpy(times).to(dev)
    sol = plan.solve(torch.from_numpy(fixed).to(dev), td)
    coeffs = sol["coeffs"]
    dt = 0.005
    smp, _, cnt = mtg.sample_trajectories(coeffs, td, dt, max_derivative=2, with_times=False)
    for k in (1, 2):
        out = mtg.max_magnitude(coeffs, td, k)
        torch.cuda.synchronize()
        ch = smp[:, k * D:(k + 1) * D, :]
        n = cnt.long()
        idx = torch.arange(ch.shape[2], device=dev)[None, :] < n[:, None]
        mag = torch.where(idx, torch.sqrt((ch ** 2).sum(dim=1)), torch.zeros((), dtype=ch.dtype, device=dev))
        sampled = mag.max(dim=1).values.cpu().numpy()
        v = out["value"].cpu().numpy()
        assert np.all(v >= sampled - 1e-12)
        assert np.all(v - sampled <= 0.01)
        # the reported (segment, time) attains the value
        c = coeffs.cpu().numpy()
        seg = out["segment"].cpu().numpy()
        tt = out["time"].cpu().numpy()
        for b in range(0, B, 97):
            val = 0.0
            for d in range(D):
                p = np.polynomial.polynomial.polyder(c[b, seg[b], d], k)
                val += np.polynomial.polynomial.polyval(tt[b], p) ** 2
            assert abs(np.sqrt(val) - v[b]) <= 1e-10 * v[b]


def test_soft_constraint_cost_vs_oracle(ctx, dev, oracle):
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S = 10, 3, 10
    seeds = list(range(720, 736))
    coeffs, times = _problems(oracle, N, D, S, seeds)
    cd = torch.from_numpy(coeffs).to(dev)
    td = torch.from_numpy(times).to(dev)
    ders, lims = [1, 2], [3.0, 1.5]  # v_max, a_max of estimateSegmentTimes scale
    out = mtg.soft_constraint_cost(cd, td, ders, lims, weight=100.0)
    torch.cuda.synchronize()
    cost = out["cost"].cpu().numpy()
    maxima = out["maxima"].cpu().numpy()
    for b in range(len(seeds)):
        rc, rm = oracle.soft_constraint_cost(N, coeffs[b], times[b], ders, lims, 100.0)
        assert np.allclose(maxima[b], rm, rtol=1e-10, atol=0)
        # exp(100 x) amplifies the maxima's rounding by 100 / limit
        assert abs(cost[b] - rc) <= 1e-8 * rc, (b, cost[b], rc)
    # the 1e12 cap (maximum_cost)
    out = mtg.soft_constraint_cost(cd, td, [1], [0.01], weight=100.0)
    assert torch.all(out["cost"] == 1.0e12)


@pytest.mark.parametrize("S,ders,lims,B", [
    (2, [0, 1, 2, 3, 4], [20.0, 3.0, 1.5, 5.0, 9.0], 24),   # one launch, 5 lane groups
    (20, [1, 2, 3], [3.0, 1.5, 4.0], 16),                   # one launch, fewer parts
    (10, [2, 1], [1.5, 3.0], 4100),                          # per-constraint launches
])
def test_soft_constraint_cost_launch_shapes(ctx, dev, oracle, S, ders, lims, B):
    """Both launch organisations of mtg_soft_constraint_cost (all constraints
    in one workgroup per trajectory below 4096 trajectories, one launch per
    constraint above) against the oracle, with up to five constraints."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D = 10, 3
    n_ref = 12
    coeffs, times = _problems(oracle, N, D, S, list(range(900, 900 + n_ref)))
    reps = (B + n_ref - 1) // n_ref
    cb = np.ascontiguousarray(np.tile(coeffs, (reps, 1, 1, 1))[:B])
    tb = np.ascontiguousarray(np.tile(times, (reps, 1))[:B])
    out = mtg.soft_constraint_cost(torch.from_numpy(cb).to(dev), torch.from_numpy(tb).to(dev),
                                   ders, lims, weight=100.0)
    torch.cuda.synchronize()
    cost = out["cost"].cpu().numpy()
    maxima = out["maxima"].cpu().numpy()
    for b in list(range(n_ref)) + [B - 1]:
        rc, rm = oracle.soft_constraint_cost(N, cb[b], tb[b], ders, lims, 100.0)
        assert np.allclose(maxima[b], rm, rtol=1e-10, atol=0), b
        assert abs(cost[b] - rc) <= 1e-8 * rc, (b, cost[b], rc)


def test_extrema_zero_and_edge_inputs(ctx, dev, oracle):
    """Identically-zero derivative (no roots; Extremum stays {0, 0, 0}) and a
    maximum forced onto the end of the last segment."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S = 10, 3, 4
    c = np.zeros((1, S, D, N))
    t = np.full((1, S), 2.0)
    out = mtg.max_magnitude(torch.from_numpy(c).to(dev), torch.from_numpy(t).to(dev), 1)
    assert float(out["value"][0]) == 0.0 and int(out["segment"][0]) == 0
    assert float(out["time"][0]) == 0.0
    # p(t) = t^2 in x on every segment: |v| = 2t grows to the segment end.
    c[0, :, 0, 2] = 1.0
    t[0, S - 1] = 3.0
    out = mtg.max_magnitude(torch.from_numpy(c).to(dev), torch.from_numpy(t).to(dev), 1)
    ref = oracle.max_magnitude(N, c[0], t[0], 1)
    assert int(out["segment"][0]) == S - 1 == ref["segment"]
    assert float(out["time"][0]) == 3.0 and abs(float(out["value"][0]) - 6.0) <= 1e-12


def test_extrema_rejects_bad_arguments(ctx, dev):
    import mav_tube_trajectory_generation_amd as mtg
    from mav_tube_trajectory_generation_amd._abi import MTGError
    c = torch.zeros((1, 3, 3, 10), dtype=torch.float64, device=dev)
    t = torch.ones((1, 3), dtype=torch.float64, device=dev)
    with pytest.raises(MTGError):
        mtg.max_magnitude(c, t, 5)   # only POSITION..SNAP
    with pytest.raises(MTGError):
        mtg.max_magnitude(c, t, -1)
    c4 = torch.zeros((1, 3, 3, 4), dtype=torch.float64, device=dev)
    with pytest.raises(MTGError):
        mtg.max_magnitude(c4, t, 3)  # N - derivative - 1 <= 0
    with pytest.raises(MTGError):
        mtg.soft_constraint_cost(c, t, [1], [-1.0])


@pytest.mark.parametrize("N,D,S,K", [(12, 4, 256, 2), (8, 3, 100, 1), (10, 3, 33, 0)])
def test_max_magnitude_random_polynomials(ctx, dev, oracle, N, D, S, K):
    """Random coefficients (not minimum-snap solutions: no smoothness across
    vertices), long trajectories: S = 256 stages 100 KB of LDS per workgroup
    and runs one part per segment; S = 100 two; S = 33 four."""
    import mav_tube_trajectory_generation_amd as mtg
    rng = np.random.default_rng(N * 1000 + S)
    B = 3
    coeffs = rng.standard_normal((B, S, D, N)) / np.array([math.factorial(k) for k in range(N)])
    times = rng.uniform(0.2, 3.0, (B, S))
    out = mtg.max_magnitude(torch.from_numpy(coeffs).to(dev), torch.from_numpy(times).to(dev), K)
    torch.cuda.synchronize()
    for b in range(B):
        ref = oracle.max_magnitude(N, coeffs[b], times[b], K)
        assert abs(float(out["value"][b]) - ref["value"]) <= 1e-10 * ref["value"]
        _check_argmax(float(out["time"][b]), int(out["segment"][b]), ref, coeffs[b], times[b], K)


@pytest.mark.parametrize("N,D,S", [(10, 3, 10), (10, 2, 4), (8, 3, 6)])
def test_min_max_magnitude(ctx, dev, oracle, N, D, S):
    """mtg_min_max_magnitude (Trajectory::computeMinMaxMagnitude,
    trajectory.cpp:184-220): the maximum is mtg_max_magnitude's bit for bit;
    the minimum is attained at its reported (segment, time), is no larger than
    the minimum over 2000 samples per segment, and no smaller by more than
    the sampling resolution (the test_polynomial_optimization.cpp:307-406
    check, 1e-2 there)."""
    import mav_tube_trajectory_generation_amd as mtg
    seeds = list(range(900, 908))
    coeffs, times = _problems(oracle, N, D, S, seeds)
    c_d = torch.from_numpy(coeffs).to(dev)
    t_d = torch.from_numpy(times).to(dev)
    for k in range(0, 4):
        mm = {key: v.cpu().numpy() for key, v in mtg.min_max_magnitude(c_d, t_d, k).items()}
        mx = {key: v.cpu().numpy() for key, v in mtg.max_magnitude(c_d, t_d, k).items()}
        assert np.array_equal(mm["max_value"], mx["value"])
        assert np.array_equal(mm["max_time"], mx["time"])
        assert np.array_equal(mm["max_segment"], mx["segment"])
        for b in range(len(seeds)):
            smin = min(np.min(_magnitude(coeffs[b, s], np.linspace(0, times[b, s], 2000), k))
                       for s in range(S))
            vmax = mm["max_value"][b]
            s_, t_ = int(mm["min_segment"][b]), mm["min_time"][b]
            assert 0.0 <= t_ <= times[b, s_]
            got = _magnitude(coeffs[b, s_], t_, k)
            assert abs(got - mm["min_value"][b]) <= 1e-9 * max(vmax, 1.0)
            assert mm["min_value"][b] <= smin + 1e-12 * max(vmax, 1.0)
            assert smin - mm["min_value"][b] <= 1e-2 * max(vmax, 1.0)
