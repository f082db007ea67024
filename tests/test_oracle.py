"""CPU tests that pin the oracle (oracle/liboracle.so) to the reference.

The reference cannot be built here, so the oracle is pinned by
the reference's own known answers and property tests
(test/test_polynomial_optimization.cpp) and by an independent NumPy
restatement (tests/numpy_ref.py) plus the committed golden fixtures.
"""
import json
import os

import numpy as np
import pytest

import numpy_ref
from helpers import check_path, cost_numeric, rel_err, rel_err_coeffs, standard_vertices

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_two_vertices_known_answer(oracle):
    """TwoVerticesSetup (test_polynomial_optimization.cpp:707-751): the Matlab
    coefficients of the 1-D rest-to-rest 0 -> 5 m, T = 5 s snap solution."""
    mask = np.ones((2, 5), np.uint8)
    vals = np.zeros((2, 5, 1))
    vals[1, 0, 0] = 5.0
    sol = oracle.linear_solve(10, 4, oracle.Vertices(mask, vals), [5.0])
    matlab = np.array([-0.000000000000004, 0.000000000000004, -0.000000000000006,
                       0.000000000000003, -0.000000000000001, 0.201600000000015,
                       -0.134400000000012, 0.034560000000004, -0.004032000000000,
                       0.000179200000000])
    assert sol["np"] == 0 and sol["nf"] == 10
    assert np.max(np.abs(sol["coeffs"][0, 0] - matlab)) < 1e-13


def test_base_coefficients(oracle):
    """computeBaseCoefficients: base(n, i) = i!/(i-n)! (polynomial.cpp:145-161)."""
    B = oracle.base_coefficients(22)
    for n in range(22):
        for i in range(22):
            assert B[n, i] == numpy_ref.falling(n, i)


@pytest.mark.parametrize("N", [4, 6, 8, 10])
def test_a_matrix_inversion(oracle, N):
    """AMatrixInversion (test_polynomial_optimization.cpp:695-705), 1e-10
    (the reference runs it for its N = 10; at N = 12 numpy's dense inverse
    itself is only ~1e-8 accurate at T = 1)."""
    for t in np.arange(1.0, 61.0):
        _, A, Ai, _ = oracle.segment_matrices(N, N // 2 - 1, t)
        assert np.array_equal(A, numpy_ref.mapping_matrix(N, t))
        assert np.max(np.abs(Ai - np.linalg.inv(A))) < 1e-10, t


def test_constraint_packing(oracle):
    """ConstraintPacking (test_polynomial_optimization.cpp:510-570): [d_f; d_p]
    -> p = A^-1 M d -> M_pinv A p round trip, p equals segment coefficients."""
    for D, S in ((1, 10), (3, 10), (3, 5)):
        for i in range(4):
            v = oracle.random_vertices(4, S, D, -50.0, 50.0, 12345 + i)
            t = oracle.estimate_segment_times(v, 3.0, 5.0)
            m = oracle.linear_matrices(10, 4, v, t)
            for d in range(D):
                d_all = np.concatenate([m["df"][d], m["dp"][d]])
                p = m["Ainv"] @ m["M"] @ d_all
                back = m["Mpinv"] @ (m["A"] @ p)
                assert np.max(np.abs(back - d_all)) < 1e-6
                for s in range(S):
                    assert np.max(np.abs(p[s * 10:(s + 1) * 10] - m["coeffs"][s, d])) < 1e-6


REF_PARAMS = [
    (1, 4, 1, 100, 3.0, 5.0), (1, 4, 10, 102, 3.0, 5.0), (1, 4, 50, 103, 3.0, 5.0),
    (3, 4, 1, 104, 3.0, 5.0), (3, 4, 10, 105, 3.0, 5.0), (3, 4, 50, 106, 3.0, 5.0),
    (3, 4, 75, 106, 3.0, 5.0), (1, 2, 5, 107, 1.0, 2.0), (3, 2, 1, 108, 1.0, 2.0),
    (3, 2, 5, 109, 1.0, 2.0), (3, 3, 5, 110, 1.0, 2.0),
]


@pytest.mark.parametrize("D,r,S,seed,vmax,amax", REF_PARAMS)
def test_reference_fixture_properties(oracle, D, r, S, seed, vmax, amax):
    """checkPath + checkCost (test_polynomial_optimization.cpp:113-195) and
    VertexGeneration (:249-268) on the reference's parameter sets."""
    v = standard_vertices(10, S, D, seed)
    assert v.mask[0].sum() == 5 and v.mask[-1].sum() == 5
    assert np.all(np.abs(v.vals[:, 0, :]) <= 10.0)
    t = oracle.estimate_segment_times(v, vmax, amax)
    sol = oracle.linear_solve(10, r, v, t)
    check_path(v, sol["coeffs"], t, 10)
    if S <= 10:
        num = cost_numeric(sol["coeffs"], t, r)
        assert abs(num - sol["cost"]) <= 0.1 * num


@pytest.mark.parametrize("D,r,S,seed,vmax,amax", REF_PARAMS[:9])
def test_numpy_cross_check(oracle, D, r, S, seed, vmax, amax):
    """Oracle vs the independent NumPy restatement (dense KKT)."""
    v = standard_vertices(10, S, D, seed)
    t = oracle.estimate_segment_times(v, vmax, amax)
    sol = oracle.linear_solve(10, r, v, t)
    c, cost = numpy_ref.solve_linear(10, r, v.mask[:, :5], v.vals[:, :5, :], t)
    assert rel_err_coeffs(sol["coeffs"], c) <= 1e-7
    assert rel_err(sol["cost"], cost) <= 1e-7


@pytest.mark.parametrize("seed", [0, 1, 105, 4242, 2**31 + 5])
def test_generator_matches_libstdcxx_semantics(oracle, seed):
    """createRandomVertices positions vs a pure-Python std::mt19937 +
    generate_canonical<double, 53> emulation (bit-exact)."""
    v = oracle.random_vertices(4, 10, 3, -10.0, 10.0, seed & 0xFFFFFFFF)
    ref = numpy_ref.random_positions(10, 3, -10.0, 10.0, seed & 0xFFFFFFFF)
    assert np.array_equal(v.positions(), ref)


def test_time_estimates(oracle):
    """estimateSegmentTimesNfabian / VelocityRamp formulas (vertex.cpp:252-287)."""
    v = standard_vertices(10, 6, 3, 7)
    p = v.positions()
    d = np.linalg.norm(np.diff(p, axis=0), axis=1)
    t0 = oracle.estimate_segment_times(v, 3.0, 5.0)
    assert np.allclose(t0, d / 3.0 * 2 * (1.0 + 6.5 * 3.0 / 5.0 * np.exp(-d / 3.0 * 2)),
                       rtol=1e-15)
    t1 = oracle.estimate_segment_times(v, 3.0, 5.0, method=1, magic=1.0)
    acc_t, acc_d = 3.0 / 5.0, 0.5 * 3.0 * 3.0 / 5.0
    exp = np.where(d < 2 * acc_d, 2 * np.sqrt(d / 5.0), 2 * acc_t + (d - 2 * acc_d) / 3.0)
    assert np.allclose(t1, exp, rtol=1e-15)


def test_time_cost_modes(oracle):
    """objectiveFunctionTime value and the two gradient forms are consistent:
    mode 2 (re-solved central differences) ~ analytic envelope derivative,
    mode 1 = w_d dJ_d/dT + w_t with fixed d (getCostAndGradientTime)."""
    v = standard_vertices(10, 5, 3, 105)
    t = oracle.estimate_segment_times(v, 3.0, 5.0)
    J0, _ = oracle.time_cost(10, 4, v, t)
    sol = oracle.linear_solve(10, 4, v, t)
    assert abs(J0 - (sol["cost"] + 500.0 * t.sum() ** 2)) <= 1e-12 * J0
    _, g2 = oracle.time_cost(10, 4, v, t, grad_mode=2, increment=1e-4)
    # Envelope theorem: d(min_x J)/dT = dJ/dT at fixed x, so mode 1 with
    # w_d = 0.5 (J_d = 2 computeCost) and w_t = 0 plus the penalty
    # derivative equals mode 2 up to O(increment^2).
    _, g1 = oracle.time_cost(10, 4, v, t, grad_mode=1, increment=1e-4, w_d=0.5, w_t=0.0)
    pen = 2 * 500.0 * t.sum()
    assert np.allclose(g1 + pen, g2, rtol=1e-5, atol=1e-6 * np.abs(g2).max())


def test_golden_fixtures(oracle):
    """Committed fixtures (tests/golden/make_golden.py) reproduce."""
    path = os.path.join(GOLDEN, "linear_golden.json")
    with open(path) as f:
        cases = json.load(f)["cases"]
    assert cases
    for c in cases:
        mask = np.array(c["mask"], np.uint8)
        vals = np.array(c["vals"])
        t = np.array(c["times"])
        sol = oracle.linear_solve(c["N"], c["r"], oracle.Vertices(mask, vals), t)
        assert rel_err_coeffs(sol["coeffs"], np.array(c["coeffs"])) <= 1e-12, c["name"]
        assert rel_err(sol["cost"], c["cost"]) <= 1e-12, c["name"]


def _evaluate_range_py(coeffs, times, t_start, t_end, dt, k):
    """Independent pure-Python restatement of Trajectory::evaluateRange
    (trajectory.cpp:74-134) with Polynomial::evaluate (polynomial.h:135-149)."""
    S, D, N = coeffs.shape
    acc, i = 0.0, 0
    for i in range(S):
        acc += times[i]
        if acc > t_start:
            break
    acc -= times[i]
    tin = t_start - acc
    out, ts = [], []
    while acc < t_end:
        if tin > times[i]:
            tin -= times[i]
            i += 1
            if i >= S:
                break
            continue
        row = []
        for d in range(D):
            c = coeffs[i, d]
            f = [numpy_ref.falling(k, j) for j in range(N)]
            v = f[N - 1] * c[N - 1]
            for j in range(N - 2, k - 1, -1):
                v = v * tin + f[j] * c[j]
            row.append(v if k < N else 0.0)
        out.append(row)
        ts.append(acc)
        tin += dt
        acc += dt
    return np.array(out), np.array(ts)


@pytest.mark.parametrize("k", [0, 1, 4])
def test_evaluate_range(oracle, k):
    """orc_evaluate_range against an independent Python loop (bit-exact:
    same operation order, -ffp-contract=off in the oracle)."""
    v = oracle.random_vertices(4, 4, 3, -10.0, 10.0, 123)
    t = oracle.estimate_segment_times(v, 3.0, 5.0)
    coeffs = oracle.linear_solve(10, 4, v, t)["coeffs"]
    for t0, t1 in ((0.0, float(t.sum())), (float(t[0]) + 0.21, float(t.sum()) - 0.5)):
        ref, rt = _evaluate_range_py(coeffs, t, t0, t1, 0.03, k)
        got, gt, n = oracle.evaluate_range(10, coeffs, t, t0, t1, 0.03, k)
        assert n == len(ref)
        assert np.array_equal(got, ref) and np.array_equal(gt, rt)


@pytest.mark.parametrize("seed", [900, 901, 902])
def test_time_optimize_port_matches_driver(oracle, seed):
    """orc_time_optimize (the C++ port timed as bench's time-workload CPU
    baseline) takes the same steps as the Python driver of the GPU
    optimiser, on the same oracle objective."""
    from helpers import optimize_reference
    N, R, S = 10, 4, 6
    v = standard_vertices(N, S, 3, seed)
    t0 = oracle.estimate_segment_times(v, 3.0, 5.0)
    Tr, fr, er = optimize_reference(oracle, N, R, v, t0, 20)
    Tc, fc, ec = oracle.time_optimize(N, R, v, t0, 20)
    assert ec == er
    assert np.max(np.abs(Tc - Tr) / Tr) <= 1e-12
    assert abs(fc - fr) <= 1e-12 * abs(fr)


def test_bench_workload_baselines(oracle):
    """The three CPU-baseline legs run and count units (tiny budgets)."""
    N, R, S, D = 10, 4, 4, 3
    K = N // 2
    B = 2
    masks = np.zeros((B, S + 1, K), np.uint8)
    vals = np.zeros((B, S + 1, K, D))
    times = np.zeros((B, S))
    for b in range(B):
        v = standard_vertices(N, S, D, 105 + b)
        masks[b], vals[b] = v.mask, v.vals
        times[b] = oracle.estimate_segment_times(v, 3.0, 5.0)
    n, sec = oracle.bench_workload(1, N, D, R, S, K, masks, vals, times, param_i=5, seconds=0.01)
    assert n >= 1 and sec > 0
    tm = masks.copy()
    tm[:, :, :] = 0
    tm[:, :, 0] = 1
    tm[:, 0, :] = 1
    tm[:, S, :] = 1
    tv = np.zeros_like(vals)
    tv[:, :, 0, :] = vals[:, :, 0, :]
    radii = np.full((B, S, 2), 0.15)
    n, sec = oracle.bench_workload(2, N, D, R, S, K, tm, tv, times, radii=radii, seconds=0.01)
    assert n >= 1
    n, sec = oracle.bench_workload(3, N, D, R, S, K, masks, vals, times, param_i=4, param_d=0.01,
                                   seconds=0.01)
    assert n >= int(times[0].sum() / 0.01)


def test_poly_roots_match_numpy(oracle):
    """The oracle's root finder (companion eigenvalues, standing in for
    findRootsJenkinsTraub, rpoly_ak1.cpp:70-117) against numpy.roots,
    including zero roots and dropped highest-order zeros."""
    rng = np.random.default_rng(3)
    for it in range(300):
        n = int(rng.integers(2, 19))
        c = rng.standard_normal(n)
        if it % 5 == 0:
            c[0] = 0.0
        if it % 7 == 0:
            c[-1] = 0.0
        got = np.sort_complex(oracle.poly_roots(c))
        if not np.any(c):
            assert len(got) == 0
            continue
        last = np.nonzero(c)[0].max()
        ref = np.sort_complex(np.roots(c[:last + 1][::-1])) if last > 0 else np.array([])
        assert len(got) == len(ref)
        if len(ref):
            assert np.max(np.abs(got - ref) / np.maximum(1, np.abs(ref))) <= 1e-10


def _max_magnitude_numpy(N, coeffs, times, k):
    """computeMaximumOfMagnitude (linear_impl:455-487) restated with numpy:
    convolution of segment.cpp:101-116, numpy.roots, the candidate filter of
    polynomial.cpp:32-63."""
    from numpy.polynomial import polynomial as P
    S, D, _ = coeffs.shape
    best = (0.0, 0.0, 0)
    for s in range(S):
        f = np.zeros(2 * (N - k) - 2)
        for d in range(D):
            dv = P.polyder(coeffs[s, d], k) if k else coeffs[s, d]
            ddv = P.polyder(coeffs[s, d], k + 1)
            dv = np.pad(dv, (0, N - k - len(dv)))[:N - k]
            ddv = np.pad(ddv, (0, N - k - 1 - len(ddv)))[:N - k - 1]
            f += np.convolve(dv, ddv)
        nz = np.nonzero(np.abs(f) >= np.finfo(float).tiny)[0]
        roots = np.roots(f[:nz.max() + 1][::-1]) if len(nz) and nz.max() > 0 else []
        cands = [0.0, 0.0, times[s]] + [r.real for r in roots
                                        if abs(r.imag) <= np.finfo(float).eps
                                        and 0.0 <= r.real <= times[s]]
        for t in cands:
            v = np.sqrt(sum(P.polyval(t, P.polyder(coeffs[s, d], k) if k else coeffs[s, d]) ** 2
                            for d in range(D)))
            if v > best[0]:
                best = (v, t, s)
    return best


@pytest.mark.parametrize("k", [0, 1, 2, 3, 4])
def test_max_magnitude_matches_numpy_restatement(oracle, k):
    N, S, D = 10, 10, 3
    for seed in (105, 106, 111):
        v = standard_vertices(N, S, D, seed)
        t = oracle.estimate_segment_times(v, 3.0, 5.0)
        c = oracle.linear_solve(N, 4, v, t)["coeffs"]
        got = oracle.max_magnitude(N, c, t, k)
        val, tm, seg = _max_magnitude_numpy(N, c, t, k)
        assert abs(got["value"] - val) <= 1e-12 * val
        assert got["segment"] == seg and abs(got["time"] - tm) <= 1e-9 * t[seg]
        # candidates: 0, 0, T and the real roots in [0, T] per segment, + the end
        assert got["n_candidates"] >= 3 * S + 1


def test_soft_constraint_cost_formula(oracle):
    N, S, D = 10, 6, 3
    v = standard_vertices(N, S, D, 140)
    t = oracle.estimate_segment_times(v, 3.0, 5.0)
    c = oracle.linear_solve(N, 4, v, t)["coeffs"]
    cost, maxima = oracle.soft_constraint_cost(N, c, t, [1, 2], [2.0, 1.0], 100.0)
    vm = oracle.max_magnitude(N, c, t, 1)["value"]
    am = oracle.max_magnitude(N, c, t, 2)["value"]
    assert np.allclose(maxima, [vm, am], rtol=0, atol=0)
    ref = min(1e12, np.exp((vm - 2.0) / 2.0 * 100.0)) + min(1e12, np.exp((am - 1.0) / 1.0 * 100.0))
    assert abs(cost - ref) <= 1e-12 * ref


def test_free_objectives_oracle(oracle):
    """orc_free_cost pinned by identities of the reference's definitions:
    J_d = d^T R d = 2 computeCost() (getCostAndGradientDerivative,
    nonlinear_impl:1537-1606), its gradient 2 (R_pf d_f + R_pp d_p) vanishes
    at the linear solution and equals central differences elsewhere;
    objectiveFunctionTimeAndConstraints = computeCost + time_penalty (sum T)^2
    (:947-1019); the optimiser restatement's Newton step lands on d*."""
    from helpers import standard_vertices
    N, R, D, S = 10, 4, 3, 5
    for pattern in ("standard", "tube"):
        v = standard_vertices(N, S, D, 321)
        t = oracle.estimate_segment_times(v, 3.0, 5.0)
        if pattern == "tube":
            v.mask[1:S, :] = 0
        ref = oracle.linear_solve(N, R, v, t)
        J, g = oracle.free_cost(N, R, v, t, ref["dp"])
        assert abs(J - 2 * ref["cost"]) <= 1e-9 * J
        assert np.max(np.abs(g)) <= 1e-7 * (1 + J)
        J1, _ = oracle.free_cost(N, R, v, t, ref["dp"], mode=1, time_penalty=500.0)
        assert abs(J1 - (ref["cost"] + 500.0 * t.sum() ** 2)) <= 1e-12 * J1
        dp = ref["dp"] + np.random.default_rng(2).normal(scale=0.2, size=ref["dp"].shape)
        J2, g2 = oracle.free_cost(N, R, v, t, dp)
        h = 1e-4
        for idx in [(0, 0), (1, dp.shape[1] // 2), (2, dp.shape[1] - 1)]:
            a, b = dp.copy(), dp.copy()
            a[idx] += h
            b[idx] -= h
            num = (oracle.free_cost(N, R, v, t, a)[0] - oracle.free_cost(N, R, v, t, b)[0]) / (2 * h)
            assert abs(num - g2[idx]) <= 1e-6 * np.max(np.abs(g2))
        d3, J3, e3 = oracle.free_optimize(N, R, v, t, dp, 10)
        assert np.max(np.abs(d3 - ref["dp"])) <= 1e-8 * (1 + np.max(np.abs(ref["dp"])))
        assert J3 <= J2 and 2 <= e3 <= 10


def test_hard_constraint_optimizer_descends_violation(oracle):
    """The device optimiser's hard-constraint mode (use_soft_constraints =
    false, nonlinear_impl:861-872; oracle port orc_time_optimize_hard) steps
    along the violation's central-difference gradient while the incumbent is
    infeasible, so from an infeasible start the violation falls (the plain
    -grad J direction shortens the times and raises |v|, |a|)."""
    N, R, D, S, tol = 10, 4, 3, 6, 0.1
    for seed in (960, 961, 962):
        v = standard_vertices(N, S, D, seed)
        t0 = oracle.estimate_segment_times(v, 3.0, 5.0)
        c0 = oracle.linear_solve(N, R, v, t0)["coeffs"]
        lims = [(1, 0.8 * oracle.max_magnitude(N, c0, t0, 1)["value"]),
                (2, 0.8 * oracle.max_magnitude(N, c0, t0, 2)["value"])]
        T, _, _ = oracle.time_optimize(N, R, v, t0, 20, soft=lims, hard=True,
                                       hard_tolerance=tol)

        def viol(c, t):
            return max(oracle.max_magnitude(N, c, t, k)["value"] - lim - tol for k, lim in lims)

        v0 = viol(c0, t0)
        v1 = viol(oracle.linear_solve(N, R, v, T)["coeffs"], T)
        assert v0 > 0.0 and v1 < 0.5 * v0, (seed, v0, v1)
