"""Shared test helpers: oracle problem construction and the parity metric."""
import numpy as np

import pyoracle

# Parity bar (BASELINE.json north_star): within 1e-6 relative on segment
# coefficients and cost.  Coefficients are compared normwise per (segment,
# dimension) because low-order coefficients of rest-to-rest segments are
# roundoff noise (the reference's own TwoVerticesSetup KAT holds 1e-15 values,
# test/test_polynomial_optimization.cpp:740-744).
REL_TOL = 1e-6


def rel_err_coeffs(got, ref):
    """max over (segment, dim) of ||got - ref|| / ||ref|| (abs floor 1e-12)."""
    got = np.asarray(got)
    ref = np.asarray(ref)
    num = np.linalg.norm(got - ref, axis=-1)
    den = np.linalg.norm(ref, axis=-1)
    return float(np.max(num / np.maximum(den, 1e-12)))


def rel_err(got, ref):
    return abs(got - ref) / max(abs(ref), 1e-300)


def standard_vertices(N, S, D, seed, pos_bound=10.0):
    """createRandomVertices(N/2-1, S, +/-pos_bound, seed) as the reference's
    test fixture (test_polynomial_optimization.cpp:75-77)."""
    return pyoracle.random_vertices(N // 2 - 1, S, D, -pos_bound, pos_bound, seed)


def compact_fixed(vertices, N):
    """Pattern mask [(S+1), N/2] and d_f [D, n_f] in (vertex, derivative)
    order, constraints of order > N/2-1 dropped (linear_impl:72-95)."""
    M = N // 2
    S, D = vertices.S, vertices.D
    K = vertices.K
    mask = np.zeros((S + 1, M), np.uint8)
    cols = []
    for v in range(S + 1):
        for k in range(M):
            if k < K and vertices.mask[v, k]:
                mask[v, k] = 1
                cols.append(vertices.vals[v, k, :])
    df = np.array(cols).T.reshape(D, len(cols)) if cols else np.zeros((D, 0))
    return mask, np.ascontiguousarray(df)


def evaluate_poly(c, t, deriv=0):
    """Value of derivative `deriv` of sum c_k t^k."""
    N = len(c)
    acc = 0.0
    for k in range(deriv, N):
        f = 1.0
        for m in range(deriv):
            f *= (k - m)
        acc += c[k] * f * t ** (k - deriv)
    return acc


def check_path(vertices, coeffs, times, N, tol=1e-6):
    """checkPath (test_polynomial_optimization.cpp:113-172): fixed constraints
    met at both segment ends and C^(N/2-1) continuity at vertices.  Tolerance
    relative to the constraint magnitude scale."""
    S, D = vertices.S, vertices.D
    M = N // 2
    for s in range(S):
        for end, v in ((0, s), (1, s + 1)):
            t = 0.0 if end == 0 else times[s]
            for k in range(min(M, vertices.K)):
                if not vertices.mask[v, k]:
                    continue
                for d in range(D):
                    got = evaluate_poly(coeffs[s, d], t, k)
                    want = vertices.vals[v, k, d]
                    assert abs(got - want) <= tol * max(1.0, abs(want)), (s, end, k, d, got, want)
        if s > 0:
            for k in range(M):
                for d in range(D):
                    a = evaluate_poly(coeffs[s - 1, d], times[s - 1], k)
                    b = evaluate_poly(coeffs[s, d], 0.0, k)
                    assert abs(a - b) <= tol * max(1.0, abs(a)), (s, k, d, a, b)


def cost_numeric(coeffs, times, r, dt=1e-3):
    """computeCostNumeric (test_utils.h:56-64): sum over samples of
    ||p^(r)(t)||^2 dt along the trajectory."""
    total = 0.0
    S, D, N = coeffs.shape
    for s in range(S):
        ts = np.arange(0.0, times[s], dt)
        for d in range(D):
            c = coeffs[s, d]
            k = np.arange(r, N)
            f = np.ones_like(k, dtype=float)
            for m in range(r):
                f *= (k - m)
            vals = (c[r:] * f)[None, :] * ts[:, None] ** (k - r)[None, :]
            total += np.sum(vals.sum(axis=1) ** 2) * dt
    return total


def optimize_reference(oracle, N, R, v, t0, max_evals, time_penalty=500.0, inc=0.1):
    """The optimiser of time_optimize_kernel restated on the oracle objective:
    projected scaled steepest descent, expand x1.5 / backtrack x0.5."""
    T0 = np.array(t0, float)
    T = T0.copy()
    f, _ = oracle.time_cost(N, R, v, T, time_penalty=time_penalty)
    _, g = oracle.time_cost(N, R, v, T, time_penalty=time_penalty, grad_mode=2, increment=inc)
    evals, alpha = 1, 0.1
    while evals < max_evals and alpha > 1e-9:
        gmax = np.max(np.abs(g * T0))
        if not gmax > 0:
            break
        trial = np.clip(T - alpha * T0 * (g * T0) / gmax, 0.1, 2.0 * T0)
        if np.array_equal(trial, T):
            break
        ft, _ = oracle.time_cost(N, R, v, trial, time_penalty=time_penalty)
        evals += 1
        if ft < f:
            T, f = trial, ft
            alpha = min(alpha * 1.5, 1.0)
            _, g = oracle.time_cost(N, R, v, T, time_penalty=time_penalty, grad_mode=2,
                                    increment=inc)
        else:
            alpha *= 0.5
    return T, f, evals
