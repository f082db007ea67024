"""The LN_SBPLX restatement (oracle/orc_sbplx.cpp: NLopt's Subplex, the
reference's default optimiser, polynomial_optimization_nonlinear.h:61)
pinned evaluation for evaluation against an independent pure-Python
restatement (tests/sbplx_ref.py), and its time-allocation driver
(orc_time_optimize_sbplx, optimizeTime nonlinear_impl:332-397) checked for
the reference's contract: bounds [0.1, 2 T0], maxeval, a best point no worse
than the start.  NLopt is absent, so parity with NLopt itself is unpinned.
"""
import numpy as np
import pytest

import sbplx_ref


@pytest.mark.parametrize("n,maxeval,ftol", [(1, 30, 0.05), (2, 40, 0.05), (3, 60, 1e-4),
                                            (5, 80, 1e-6), (7, 120, 0.05), (10, 50, 0.05),
                                            (10, 400, 1e-9), (13, 300, 1e-8), (16, 500, -1.0)])
def test_oracle_matches_python_restatement(oracle, n, maxeval, ftol):
    rng = np.random.default_rng(n * 1000 + maxeval)
    x0 = rng.uniform(0.2, 3.0, n)
    lb = np.full(n, 0.1)
    ub = 2.0 * x0
    step = 0.1 * x0
    code, x, minf, nev, hist = oracle.sbplx_test(lb, ub, x0, step, maxeval, ftol, -1.0)
    pcode, px, pminf, phist = sbplx_ref.sbplx(sbplx_ref.test_fn, list(lb), list(ub), list(x0),
                                               list(step), maxeval, ftol, -1.0)
    assert code == pcode
    assert nev == len(phist)
    assert np.array_equal(hist, np.array(phist).reshape(-1, n)), "evaluation sequence differs"
    assert np.array_equal(x, np.array(px))
    assert minf == pminf
    assert (x >= lb).all() and (x <= ub).all()
    assert nev <= maxeval
    assert code in (3, 4, 5)


def test_converges_on_the_test_objective(oracle):
    from scipy.optimize import minimize
    n = 6
    x0 = np.linspace(0.5, 2.0, n)
    lb, ub = np.full(n, -5.0), np.full(n, 5.0)
    code, x, minf, nev, _ = oracle.sbplx_test(lb, ub, x0, 0.1 * x0, 4000, 1e-14, -1.0)
    ref = minimize(lambda z: sbplx_ref.test_fn(list(z)), x0, method="BFGS", tol=1e-12)
    assert minf <= ref.fun + 1e-8 * (1 + abs(ref.fun))
    assert np.allclose(x, ref.x, atol=1e-3)


def test_time_optimize_sbplx_contract(oracle):
    N, D, r, S = 10, 3, 4, 10
    for seed in (105, 106, 107):
        v = oracle.random_vertices(N // 2 - 1, S, D, -10.0, 10.0, seed)
        t0 = oracle.estimate_segment_times(v, 3.0, 5.0)
        J0, _ = oracle.time_cost(N, r, v, t0, grad_mode=0)
        t, J, ev, res, hist = oracle.time_optimize_sbplx(N, r, v, t0, 50)
        assert ev <= 50 and res in (3, 4, 5)
        assert J <= J0
        assert (t >= 0.1 - 1e-15).all() and (t <= 2.0 * t0 + 1e-12).all()
        assert np.array_equal(hist[0], t0)  # the first evaluation is the start
        # the reported cost is the objective at the returned point
        Jt, _ = oracle.time_cost(N, r, v, t, grad_mode=0)
        assert abs(Jt - J) <= 1e-9 * abs(J)


@pytest.mark.parametrize("x0", [[0.5, 0.08, 0.7], [0.04, 1.0, 1.0]], ids=["below_lb", "lb_gt_ub"])
def test_start_out_of_bounds_is_failure(oracle, x0):
    """A start below kOptimizationTimeLowerBound (0.1), or with lb > ub = 2 T0,
    is NLopt's invalid start (NLOPT_INVALID_ARGS before any evaluation, which
    optimizeTime returns as nlopt::FAILURE, nonlinear_impl:389-394): both
    restatements return -1 with no evaluation and x unchanged."""
    x0 = np.array(x0)
    lb, ub, step = np.full(3, 0.1), 2.0 * x0, 0.1 * x0
    code, x, minf, nev, hist = oracle.sbplx_test(lb, ub, x0, step, 40, 0.05, -1.0)
    assert code == -1 and nev == 0 and np.array_equal(x, x0) and np.isnan(minf)
    pcode, px, pminf, phist = sbplx_ref.sbplx(sbplx_ref.test_fn, list(lb), list(ub), list(x0),
                                               list(step), 40, 0.05, -1.0)
    assert pcode == -1 and phist == [] and px == list(x0)
