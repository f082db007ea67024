"""CPU checks of the oracle's tube QCQP (oracle/mtg_oracle.cpp, restating
qcqp_impl:18-788).

MOSEK, the reference's solver (qcqp_impl:577-775), is absent, so the solve
is "parity unpinned" against the reference itself.  What is pinned here:
  * the constraint assembly (qcqp_impl:321-474) against an independent
    geometric restatement: Bernstein control points of the recovered
    polynomials, distance to the tube axis, half-spaces and end spheres;
  * the oracle's interior-point solution against SciPy's SLSQP on the same
    convex QCQP (objective agrees; x to the conditioning) and the KKT
    conditions at the oracle's solution.
The GPU tube kernels are then compared with this oracle (test_tube_gpu.py).
"""
import math

import numpy as np
import pytest

from test_tube_gpu import main_cpp_vertices

N, R = 10, 4
M = N // 2


def bernstein_points(coeffs, T):
    """Control points of p(t) = sum_k a_k t^k on [0, T] (degree n = N-1):
    b_j = sum_{k<=j} C(j,k)/C(n,k) a_k T^k."""
    n = len(coeffs) - 1
    a = coeffs * T ** np.arange(n + 1)
    return np.array([sum(math.comb(j, k) / math.comb(n, k) * a[k] for k in range(j + 1))
                     for j in range(n + 1)])


def geometric_residuals(v, coeffs, times, radii):
    """Constraint values in the reference's order (qcqp_impl:321-474): per
    segment i: [sphere if i < S-1], tube j = 1..N-2, then for j = 1..N-2 the
    start and end half-spaces of control point j."""
    S = v.S
    pos = v.vals[:, 0, :]
    out = []
    for i in range(S):
        cps = np.stack([bernstein_points(coeffs[i, d], times[i]) for d in range(3)], axis=1)
        p0, p1 = pos[i], pos[i + 1]
        nvec = (p1 - p0) / np.linalg.norm(p1 - p0)
        r1, r2 = radii[i]
        if i < S - 1:
            out.append(np.sum((cps[N - 1] - p1) ** 2) - r2 ** 2)
        P = np.eye(3) - np.outer(nvec, nvec)
        for j in range(1, N - 1):
            out.append(np.sum((P @ (cps[j] - p0)) ** 2) - r1 ** 2)
        ps = p0 - nvec * (r1 if i == 0 else radii[i - 1][1])
        pe = p1 + nvec * r2
        for j in range(1, N - 1):
            out.append(-nvec @ (cps[j] - ps))
            out.append(nvec @ (cps[j] - pe))
    return np.array(out)


def random_tube(oracle, S, seed):
    mask = np.zeros((S + 1, M), np.uint8)
    rv = oracle.random_vertices(M - 1, S, 3, -10.0, 10.0, seed, K=M)
    mask[:, 0] = 1
    mask[0, :] = 1
    mask[S, :] = 1
    return oracle.Vertices(mask, rv.vals * mask[:, :, None])


@pytest.mark.parametrize("case", ["main_cpp", "random5"])
def test_assembly_matches_geometry(oracle, case):
    v = main_cpp_vertices(oracle) if case == "main_cpp" else random_tube(oracle, 5, 105)
    t = oracle.estimate_segment_times(v, 2.0, 2.0)
    radii = np.full((v.S, 2), 0.15 if case == "main_cpp" else 0.5)
    sol = oracle.tube_solve(N, R, v, t, radii)
    res = oracle.tube_residuals(N, R, v, t, radii, sol["x"])
    geo = geometric_residuals(v, sol["coeffs"], t, radii)
    assert res.shape == geo.shape == (oracle.tube_num_constraints(N, v.S),)
    # The reference zero-snaps entries below 1e-6 / 1e-5 (qcqp_impl:304-309,
    # 388-400); the geometric restatement does not, hence the tolerance.
    assert np.max(np.abs(res - geo)) <= 1e-6


@pytest.mark.parametrize("case", ["main_cpp", "random5"])
def test_ipm_matches_scipy(oracle, case):
    from scipy.optimize import minimize
    v = main_cpp_vertices(oracle) if case == "main_cpp" else random_tube(oracle, 5, 105)
    t = oracle.estimate_segment_times(v, 2.0, 2.0)
    radii = np.full((v.S, 2), 0.15 if case == "main_cpp" else 0.5)
    qp = oracle.tube_assemble(N, R, v, t, radii)
    P, q, Qk, lk, ck = qp["P"], qp["q"], qp["quad"], qp["lin"], qp["cst"]
    sol = oracle.tube_solve(N, R, v, t, radii)
    assert sol["status"] == 0

    f = lambda x: 0.5 * x @ P @ x + q @ x  # noqa: E731
    cons = {"type": "ineq",
            "fun": lambda x: -(0.5 * np.einsum("i,kij,j->k", x, Qk, x) + lk @ x + ck),
            "jac": lambda x: -(np.einsum("kij,j->ki", Qk, x) + lk)}
    x0 = np.linalg.solve(P, -q)  # unconstrained minimiser
    ref = minimize(f, x0, jac=lambda x: P @ x + q, constraints=[cons], method="SLSQP",
                   options={"maxiter": 2000, "ftol": 1e-12})
    assert ref.success, ref.message
    fo, fs = f(sol["x"]), f(ref.x)
    assert abs(fo - fs) <= 1e-6 * abs(fs)
    g = 0.5 * np.einsum("i,kij,j->k", sol["x"], Qk, sol["x"]) + lk @ sol["x"] + ck
    assert g.max() <= 1e-8
    scale = max(1.0, np.abs(ref.x).max())
    assert np.max(np.abs(sol["x"] - ref.x)) <= 1e-3 * scale
    # KKT at the oracle's x: grad f = -sum lambda_k grad g_k over the active
    # set with lambda >= 0 (non-negative least squares residual ~ 0).  The
    # IPM stops at mu <= tol = 1e-10 (its complementarity target is kept at
    # >= 1e-2 x the infeasibility, so mu does not run to 1e-20): the ~100
    # inactive constraints (slack ~0.05) keep lambda ~ mu / s ~ 1e-9 each,
    # which the active-set NNLS leaves out.  The bound is per case, each about
    # 5x the measured residual: main_cpp (6 active constraints) 1.1e-9,
    # random5 (16 active, more inactive multipliers left out) 2.3e-8.
    from scipy.optimize import nnls
    x = sol["x"]
    act = g > -1e-6
    Jg = (np.einsum("kij,j->ki", Qk, x) + lk)[act]
    _, resid = nnls(Jg.T, -(P @ x + q))
    bound = {"main_cpp": 5e-9, "random5": 1e-7}[case]
    assert resid <= bound * max(1.0, np.linalg.norm(P @ x + q))


def test_tube_time_objective_oracle(oracle):
    """objectiveFunctionTime with the QCQP inner solve (nonlinear_impl:877-945,
    solveQCQP at :892): J = computeCost of the QCQP solution + time_penalty
    (sum T)^2; the gradient is the central difference of that J (clamp rule
    :2525-2530); the optimiser only accepts decreases, stays in [0.1, 2 T0]
    and counts its evaluations."""
    S = 4
    v = main_cpp_vertices(oracle)
    t0 = oracle.estimate_segment_times(v, 2.0, 2.0)
    radii = np.full((S, 2), 0.15)
    t = t0 * 1.1
    ref = oracle.tube_solve(N, R, v, t, radii, times_cp=t0)
    J, g = oracle.tube_time_cost(N, R, v, t, radii, times_cp=t0, grad_mode=2)
    assert J == pytest.approx(ref["cost"] + 500.0 * t.sum() ** 2, rel=1e-14)
    h = 0.1
    for n in range(S):
        lo, hi = t.copy(), t.copy()
        lo[n] -= h
        hi[n] += h
        Jl, _ = oracle.tube_time_cost(N, R, v, lo, radii, times_cp=t0)
        Jh, _ = oracle.tube_time_cost(N, R, v, hi, radii, times_cp=t0)
        assert g[n] == pytest.approx((Jh - Jl) / (2 * h), rel=1e-12)
    J0, _ = oracle.tube_time_cost(N, R, v, t0, radii, times_cp=t0)
    topt, Jopt, evals = oracle.tube_time_optimize(N, R, v, t0, radii, max_evals=12)
    assert Jopt <= J0 and 1 <= evals <= 12
    assert np.all(topt >= 0.1) and np.all(topt <= 2 * t0)
    Jchk, _ = oracle.tube_time_cost(N, R, v, topt, radii, times_cp=t0)
    assert Jchk == Jopt
