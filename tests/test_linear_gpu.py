"""GPU parity of the batched linear solve (libmtg_hip.so) against the oracle.

Cases mirror the reference's parameterised fixture
(test/test_polynomial_optimization.cpp:753-851) plus the batched
configurations of BASELINE.json.
"""
import numpy as np
import pytest

from helpers import (REL_TOL, check_path, compact_fixed, cost_numeric, rel_err,
                     rel_err_coeffs, standard_vertices)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(params=["auto", "generic"])
def kernel(request):
    """Every parity case runs twice: with the kernel AUTO selects (the
    standard-pattern kernel wherever the pattern allows it) and with the
    generic kernel forced."""
    return request.param


def _solve_gpu(ctx, dev, N, r, mask, df_batch, times_batch, kernel="auto"):
    import mav_tube_trajectory_generation_amd as mtg
    S = times_batch.shape[1]
    D = df_batch.shape[1]
    plan = mtg.LinearPlan(ctx, N, D, r, S, mask).set_kernel(kernel)
    out = plan.solve(torch.from_numpy(np.ascontiguousarray(df_batch)).to(dev),
                     torch.from_numpy(np.ascontiguousarray(times_batch)).to(dev), free=True)
    torch.cuda.synchronize()
    return plan, {k: v.cpu().numpy() for k, v in out.items()}


def test_two_vertices_known_answer(ctx, dev):
    """TwoVerticesSetup (test_polynomial_optimization.cpp:707-751)."""
    N = 10
    mask = np.ones((2, 5), np.uint8)
    df = np.zeros((1, 1, 10))
    df[0, 0, 5] = 5.0  # goal position; everything else zero
    _, out = _solve_gpu(ctx, dev, N, 4, mask, df, np.array([[5.0]]))
    matlab = np.array([-0.000000000000004, 0.000000000000004, -0.000000000000006,
                       0.000000000000003, -0.000000000000001, 0.201600000000015,
                       -0.134400000000012, 0.034560000000004, -0.004032000000000,
                       0.000179200000000])
    got = out["coeffs"][0, 0, 0]
    assert np.max(np.abs(got - matlab)) < 1e-13
    assert out["status"][0] == 0


# (D, derivative, segments, seed, v_max, a_max) from
# test_polynomial_optimization.cpp:753-839.
REF_PARAMS = [
    (1, 4, 1, 100, 3.0, 5.0), (1, 4, 10, 102, 3.0, 5.0), (1, 4, 50, 103, 3.0, 5.0),
    (3, 4, 1, 104, 3.0, 5.0), (3, 4, 10, 105, 3.0, 5.0), (3, 4, 50, 106, 3.0, 5.0),
    (3, 4, 75, 106, 3.0, 5.0), (1, 2, 5, 107, 1.0, 2.0), (3, 2, 1, 108, 1.0, 2.0),
    (3, 2, 5, 109, 1.0, 2.0), (3, 3, 5, 110, 1.0, 2.0),
]


@pytest.mark.parametrize("D,r,S,seed,vmax,amax", REF_PARAMS)
def test_reference_fixture_parity(ctx, dev, oracle, D, r, S, seed, vmax, amax, kernel):
    N = 10
    v = standard_vertices(N, S, D, seed)
    times = oracle.estimate_segment_times(v, vmax, amax)
    ref = oracle.linear_solve(N, r, v, times)
    mask, df = compact_fixed(v, N)
    _, out = _solve_gpu(ctx, dev, N, r, mask, df[None], times[None], kernel)
    assert out["status"][0] == 0
    assert rel_err_coeffs(out["coeffs"][0], ref["coeffs"]) <= REL_TOL
    assert rel_err(out["cost"][0], ref["cost"]) <= REL_TOL
    if ref["np"]:
        assert rel_err_coeffs(out["free"][0], ref["dp"]) <= REL_TOL
    check_path(v, out["coeffs"][0], times, N)
    # checkCost: 10 % vs the numeric integral (test_polynomial_optimization.cpp:174-195).
    if S <= 10:
        # computeCost() = 0.5 c^T Q c with Q carrying the factor 2
        # (linear_impl:570) = the integral of ||p^(r)||^2.
        num = cost_numeric(out["coeffs"][0], times, r)
        assert abs(num - out["cost"][0]) <= 0.1 * num


def _exact_cases():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "exact_linear.json")) as f:
        return json.load(f)["cases"]


def _golden_cases():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "linear_golden.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", _golden_cases(), ids=lambda c: c["name"])
def test_committed_golden_vectors(ctx, dev, oracle, case, kernel):
    """The committed golden vectors (tests/golden/linear_golden.json, made by
    make_golden.py: the reference's TwoVerticesSetup Matlab solution and
    reference-fixture problems) read directly, not through the oracle, so a
    drift in the oracle cannot move the GPU's target.  Batched 2x (and, where
    the pattern allows, through the lane kernels at a batch of 70)."""
    import mav_tube_trajectory_generation_amd as mtg
    N, r = case["N"], case["r"]
    # oracle.Vertices is only the dense (mask, vals) container
    v = oracle.Vertices(np.array(case["mask"], np.uint8), np.array(case["vals"]))
    times = np.array(case["times"])
    want_c, want_J = np.array(case["coeffs"]), case["cost"]
    mask, df = compact_fixed(v, N)
    _, out = _solve_gpu(ctx, dev, N, r, mask, np.stack([df, df]), np.stack([times, times]), kernel)
    for b in range(2):
        assert out["status"][b] == 0
        assert rel_err_coeffs(out["coeffs"][b], want_c) <= REL_TOL, case["name"]
        assert rel_err(out["cost"][b], want_J) <= REL_TOL, case["name"]
    S, D = len(times), v.D
    if kernel == "auto" and N == 10 and r == 4 and D == 3 and 2 <= S <= 12:
        plan = mtg.LinearPlan(ctx, N, D, r, S, mask)
        try:
            plan.set_kernel("lane_pair")
        except mtg.MTGError:
            return  # not the standard pattern
        for k in ("lane", "lane_pair"):
            plan.set_kernel(k)
            o = plan.solve(torch.from_numpy(np.repeat(df[None], 70, 0)).to(dev),
                           torch.from_numpy(np.repeat(times[None], 70, 0)).to(dev))
            c = o["coeffs"].cpu().numpy()
            J = o["cost"].cpu().numpy()
            for b in (0, 33, 69):
                assert rel_err_coeffs(c[b], want_c) <= REL_TOL, (k, case["name"])
                assert rel_err(J[b], want_J) <= REL_TOL, (k, case["name"])


@pytest.mark.parametrize("case", _exact_cases(), ids=lambda c: f"N{c['N']}_r{c['r']}")
def test_orders_vs_exact(ctx, dev, oracle, case, kernel):
    """Every supported N (4..12) and derivative order against the exact
    rational solution (tests/golden/make_exact.py).  Where the
    reference-faithful oracle is itself accurate (< 1e-7 from the truth) the
    GPU must match it to the 1e-6 parity bar; everywhere the GPU must be at
    least as accurate as the reference algorithm in FP64."""
    N, r = case["N"], case["r"]
    v = oracle.Vertices(np.array(case["mask"], np.uint8), np.array(case["vals"]))
    times = np.array(case["times"])
    exact = np.array(case["exact"])
    mask, df = compact_fixed(v, N)
    _, out = _solve_gpu(ctx, dev, N, r, mask, df[None], times[None], kernel)
    assert out["status"][0] == 0
    gpu_err = rel_err_coeffs(out["coeffs"][0], exact)
    assert gpu_err <= max(REL_TOL, 2.0 * case["oracle_err"]), gpu_err
    if case["oracle_err"] < 1e-7:
        ref = oracle.linear_solve(N, r, v, times)
        assert rel_err_coeffs(out["coeffs"][0], ref["coeffs"]) <= REL_TOL
        assert rel_err(out["cost"][0], ref["cost"]) <= REL_TOL


@pytest.mark.parametrize("N", [4, 6, 8, 12])
def test_other_orders_3d(ctx, dev, oracle, N, kernel):
    """3-D problems at the orders where FP64 resolves the solution."""
    D, S = 3, 6
    for r in range(max(0, N // 2 - 3), N // 2):
        v = standard_vertices(N, S, D, 200 + N)
        times = oracle.estimate_segment_times(v, 3.0, 5.0)
        ref = oracle.linear_solve(N, r, v, times)
        mask, df = compact_fixed(v, N)
        _, out = _solve_gpu(ctx, dev, N, r, mask, df[None], times[None], kernel)
        assert out["status"][0] == 0, (N, r)
        tol = 1e-5 if (N == 12 and r == 3) else REL_TOL
        assert rel_err_coeffs(out["coeffs"][0], ref["coeffs"]) <= tol, (N, r)
        assert rel_err(out["cost"][0], ref["cost"]) <= tol, (N, r)


def test_irregular_patterns(ctx, dev, oracle):
    """Non-standard constraint maps: free start derivatives, an intermediate
    vertex without position, a fully constrained middle vertex, 1-D and 4-D."""
    N, r = 10, 4
    rng = np.random.default_rng(7)
    for D in (1, 2, 4):
        S = 7
        v = standard_vertices(N, S, D, 300 + D)
        v.mask[0, 3:] = 0           # start jerk/snap free
        v.mask[3, 0] = 0            # vertex 3 without position
        v.mask[5, :] = 1            # vertex 5 fully constrained
        v.vals[5, 1:, :] = rng.normal(size=(4, D))
        times = rng.uniform(0.5, 6.0, size=S)
        ref = oracle.linear_solve(N, r, v, times)
        mask, df = compact_fixed(v, N)
        plan, out = _solve_gpu(ctx, dev, N, r, mask, df[None], times[None])
        assert plan.kernel == "generic"
        assert out["status"][0] == 0
        assert rel_err_coeffs(out["coeffs"][0], ref["coeffs"]) <= REL_TOL, D
        assert rel_err(out["cost"][0], ref["cost"]) <= REL_TOL, D


def test_fully_constrained(ctx, dev, oracle):
    """n_free == 0 path (linear_impl:342-348)."""
    N, D, S = 10, 3, 3
    v = standard_vertices(N, S, D, 42)
    v.mask[:, :] = 1
    v.vals[1:S, 1:, :] = np.random.default_rng(1).normal(size=(S - 1, 4, D))
    times = np.array([2.0, 3.0, 1.5])
    ref = oracle.linear_solve(N, 4, v, times)
    assert ref["np"] == 0
    mask, df = compact_fixed(v, N)
    _, out = _solve_gpu(ctx, dev, N, 4, mask, df[None], times[None])
    assert rel_err_coeffs(out["coeffs"][0], ref["coeffs"]) <= REL_TOL


def test_config2_batch(ctx, dev, oracle, kernel):
    """BASELINE config 2: 1024 x 10-segment N=10 3-D minimum snap."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S, B = 10, 3, 10, 1024
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=105)
    _, out = _solve_gpu(ctx, dev, N, 4, mask, fixed, times, kernel)
    assert (out["status"] == 0).all()
    for b in list(range(0, B, 37)) + [B - 1]:
        v = standard_vertices(N, S, D, 105 + b)
        ref = oracle.linear_solve(N, 4, v, times[b])
        assert rel_err_coeffs(out["coeffs"][b], ref["coeffs"]) <= REL_TOL, b
        assert rel_err(out["cost"][b], ref["cost"]) <= REL_TOL, b
    # Size-independent properties on every trajectory: fixed start/end
    # constraints and C^4 continuity.
    c = out["coeffs"]
    k = np.arange(N)
    for deriv in range(5):
        f = np.ones(N)
        for m in range(deriv):
            f = f * np.maximum(k - m, 0)
        pw_end = times[:, :, None] ** np.maximum(k - deriv, 0)[None, None, :]
        end_val = np.einsum("bsdk,bsk->bsd", c * f, np.where(k >= deriv, pw_end, 0.0))
        start_val = c[:, :, :, deriv] * f[deriv]
        scale = np.maximum(1.0, np.abs(end_val[:, :-1]))
        assert np.all(np.abs(end_val[:, :-1] - start_val[:, 1:]) <= 1e-6 * scale)
    assert np.allclose(c[:, 0, :, 0], fixed[:, :, 0], atol=1e-12)


def test_bad_time_status(ctx, dev, kernel):
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S, B = 10, 3, 4, 3
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=1)
    times[1, 2] = 0.0
    times[2, 0] = -1.0
    _, out = _solve_gpu(ctx, dev, N, 4, mask, fixed, times, kernel)
    assert list(out["status"]) == [0, 1, 1]
    assert np.isnan(out["cost"][1]) and np.isfinite(out["cost"][0])


def test_host_entry_point(ctx, oracle):
    """mtg_linear_solve_host (what the C++ shim calls)."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S, B = 10, 3, 5, 4
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=9)
    plan = mtg.LinearPlan(ctx, N, D, 4, S, mask)
    out = plan.solve_host(fixed, times)
    for b in range(B):
        v = standard_vertices(N, S, D, 9 + b)
        ref = oracle.linear_solve(N, 4, v, times[b])
        assert rel_err_coeffs(out["coeffs"][b], ref["coeffs"]) <= REL_TOL


def _exact_mapping_inverse(N, T):
    from fractions import Fraction as F
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_exact as me
    M = N // 2
    A = [[F(0)] * N for _ in range(N)]
    for l in range(M):
        A[l][l] = F(me.falling(l, l))
        for j in range(l, N):
            A[M + l][j] = F(me.falling(l, j)) * F(T) ** (j - l)
    aug = me.gauss_jordan([row[:] + [F(int(i == j)) for j in range(N)]
                           for i, row in enumerate(A)], N, 2 * N)
    return np.array([[float(x) for x in row[N:]] for row in aug])


def test_segment_matrices(ctx, dev, oracle):
    """AMatrixInversion (test_polynomial_optimization.cpp:695-705) and the
    per-segment Q, A, H against the oracle's reference-faithful versions.
    The reference compares its Schur inverse with Eigen's dense inverse at
    1e-10 absolute; both FP64 LU inverses are themselves ~3e-10 off the exact
    inverse at T = 1 (entries up to 540), so the GPU's closed form is checked
    against the exact rational inverse (1e-12 relative) and against the
    reference's Schur inverse at 1e-9."""
    import mav_tube_trajectory_generation_amd as mtg
    N, r = 10, 4
    ts = np.arange(1.0, 61.0)
    Q, A, Ai, H = (x.cpu().numpy() for x in
                   mtg.segment_matrices(ctx, N, r, torch.from_numpy(ts).to(dev)))
    for i, t in enumerate(ts):
        Qo, Ao, Aio, Ho = oracle.segment_matrices(N, r, t)
        assert np.array_equal(A[i], Ao)
        ex = _exact_mapping_inverse(N, t)
        assert np.max(np.abs(Ai[i] - ex)) <= 1e-12 * np.max(np.abs(ex)), t
        assert np.allclose(Ai[i], Aio, atol=1e-9, rtol=0)
        assert np.allclose(Q[i], Qo, rtol=1e-13, atol=0)
        assert np.max(np.abs(H[i] - Ho)) <= 1e-8 * np.max(np.abs(Ho))


def test_coefficients_from_constraints(ctx, dev, oracle):
    """mtg_coeffs_from_constraints (setFreeConstraints ->
    updateSegmentsFromCompactConstraints, linear_impl:254-275, 497-506):
    feeding the solved d_p back reproduces the solve; a perturbed d_p gives
    the oracle's A^-1 M [d_f; d_p] and a higher cost."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S, B = 10, 3, 10, 64
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=105)
    plan, out = _solve_gpu(ctx, dev, N, 4, mask, fixed, times)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    c, cost, st = plan.coefficients(T(fixed), T(out["free"]), T(times))
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert rel_err_coeffs(c.cpu().numpy(), out["coeffs"]) <= 1e-12
    # The solve (standard-pattern kernel) and the recovery (generic
    # formulation) sum the quadratic form in different orders; the form
    # cancels, so the round trip is held to 1e-9, not the rounding floor.
    assert np.max(np.abs(cost.cpu().numpy() - out["cost"]) / out["cost"]) <= 1e-9
    rng = np.random.default_rng(3)
    dp = out["free"] + rng.normal(0.0, 0.3, out["free"].shape)
    c2, cost2, _ = plan.coefficients(T(fixed), T(dp), T(times))
    c2, cost2 = c2.cpu().numpy(), cost2.cpu().numpy()
    assert np.all(cost2 > out["cost"])
    for b in (0, 17, 63):
        v = standard_vertices(N, S, D, 105 + b)
        m = oracle.linear_matrices(N, 4, v, times[b])
        nf = fixed.shape[2]
        for d in range(D):
            dall = np.concatenate([fixed[b, d], dp[b, d]])
            want = (m["Ainv"] @ m["M"] @ dall).reshape(S, N)
            assert rel_err_coeffs(c2[b, :, d], want) <= 1e-9, (b, d)
        assert nf == m["M"].shape[1] - dp.shape[2]


@pytest.mark.parametrize("N,D,S", [(10, 3, 2), (10, 3, 3), (10, 3, 4), (10, 3, 9), (10, 3, 10),
                                   (10, 3, 17), (10, 3, 18), (10, 3, 33), (10, 3, 64),
                                   (10, 1, 10), (10, 2, 7), (10, 4, 10), (8, 3, 10),
                                   (6, 3, 12), (12, 3, 10), (4, 3, 10)])
def test_standard_kernel_matches_generic(ctx, dev, oracle, N, D, S):
    """The standard-pattern kernel against the generic kernel (and spot
    checks against the oracle) on a random batch: every S parity of the
    twisted sweep, S*D beyond one wave, every N and D.  Same inputs, same
    algorithm family: agreement to 1e-9 normwise."""
    import mav_tube_trajectory_generation_amd as mtg
    B = 64
    r = N // 2 - 1
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=1000 + S)
    plan_s, out_s = _solve_gpu(ctx, dev, N, r, mask, fixed, times, "standard")
    plan_g, out_g = _solve_gpu(ctx, dev, N, r, mask, fixed, times, "generic")
    assert plan_s.kernel == "standard" and plan_g.kernel == "generic"
    assert (out_s["status"] == 0).all() and (out_g["status"] == 0).all()
    tol = 1e-9 if N <= 10 else 1e-6
    worse = []
    for b in range(B):
        assert rel_err_coeffs(out_s["coeffs"][b], out_g["coeffs"][b]) <= tol, b
        assert rel_err_coeffs(out_s["free"][b], out_g["free"][b]) <= tol, b
        # The cost is a cancelling quadratic form summed in a different order
        # by the two kernels (symmetric half vs full rows).
        assert rel_err(out_s["cost"][b], out_g["cost"][b]) <= 100 * tol, b
        v = standard_vertices(N, S, D, 1000 + S + b)
        ref = oracle.linear_solve(N, r, v, times[b])
        assert rel_err_coeffs(out_s["coeffs"][b], ref["coeffs"]) <= REL_TOL, b
        assert rel_err(out_s["cost"][b], ref["cost"]) <= REL_TOL, b
        worse.append(rel_err(out_s["cost"][b], ref["cost"]) /
                     max(rel_err(out_g["cost"][b], ref["cost"]), 1e-15))
    # No systematic accuracy loss against the oracle.
    assert np.median(worse) <= 10.0, np.median(worse)


@pytest.mark.parametrize("N,D,S,kernels", [
    (10, 3, 2, ("standard",)), (10, 3, 3, ("standard", "lane", "lane_pair")),
    (10, 3, 5, ("standard", "lane", "lane_pair")), (10, 3, 6, ("standard", "lane", "lane_pair")),
    (10, 3, 9, ("standard", "lane", "lane_pair")), (10, 3, 10, ("standard", "lane", "lane_pair")),
    (10, 3, 16, ("standard",)), (10, 3, 20, ("standard",)), (10, 2, 10, ("standard",)),
    (8, 3, 7, ("standard",)), (10, 1, 4, ("standard",))])
def test_standard_kernels_nonzero_end_derivatives(ctx, dev, oracle, N, D, S, kernels):
    """The standard pattern with moving end vertices: random non-zero
    derivatives 1..N/2-1 at the start and end vertex (createRandomVertices
    fixes them to zero, so the fixtures never exercise the end vertices'
    share of b, linear_impl:306-379).  Every kernel that runs the pattern —
    the compile-time-S wave kernel (N = 10, D = 3, S <= 16), the runtime-S
    kernel, the lane kernels — against the oracle, 1e-6."""
    M = N // 2
    r = M - 1
    B = 8
    rng = np.random.default_rng(4242 + S)
    dfs, ts, refs = [], [], []
    mask = None
    for b in range(B):
        v = standard_vertices(N, S, D, 7000 + S + b)
        v.vals[0, 1:M, :] = rng.uniform(-2.0, 2.0, (M - 1, D))
        v.vals[S, 1:M, :] = rng.uniform(-2.0, 2.0, (M - 1, D))
        m, df = compact_fixed(v, N)
        mask = m
        t = oracle.estimate_segment_times(v, 3.0, 5.0)
        dfs.append(df)
        ts.append(t)
        refs.append(oracle.linear_solve(N, r, v, t))
    df_b, t_b = np.array(dfs), np.array(ts)
    for kernel in kernels:
        plan, out = _solve_gpu(ctx, dev, N, r, mask, df_b, t_b, kernel)
        assert plan.kernel == kernel
        assert (out["status"] == 0).all(), kernel
        for b in range(B):
            assert rel_err_coeffs(out["coeffs"][b], refs[b]["coeffs"]) <= REL_TOL, (kernel, b)
            assert rel_err(out["cost"][b], refs[b]["cost"]) <= REL_TOL, (kernel, b)


def test_kernel_selection(ctx):
    """AUTO picks the standard-pattern kernel exactly on the standard
    pattern; STANDARD is refused elsewhere."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S = 10, 3, 10
    mask = np.zeros((S + 1, 5), np.uint8)
    mask[0, :] = mask[S, :] = 1
    mask[1:S, 0] = 1
    assert mtg.LinearPlan(ctx, N, D, 4, S, mask).kernel == "standard"
    assert mtg.LinearPlan(ctx, N, D, 4, S, mask).set_kernel("generic").kernel == "generic"
    odd = mask.copy()
    odd[3, 0] = 0
    p = mtg.LinearPlan(ctx, N, D, 4, S, odd)
    assert p.kernel == "generic"
    with pytest.raises(mtg.MTGError):
        p.set_kernel("standard")
    assert mtg.LinearPlan(ctx, N, D, 4, 1, np.ones((2, 5), np.uint8)).kernel == "generic"
