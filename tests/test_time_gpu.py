"""GPU parity of the time-allocation cost callback and the batched segment
time optimiser (mtg_time_cost / mtg_time_optimize) against the oracle."""
import numpy as np
import pytest

from helpers import optimize_reference, rel_err, standard_vertices

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N, D, R = 10, 3, 4


@pytest.fixture(params=["auto", "generic"])
def kernel(request):
    """Every case runs with the kernel AUTO selects (time_*_std_kernel on the
    standard pattern) and with the generic time_cost_kernel /
    time_optimize_kernel forced."""
    return request.param


def _batch(S, B, seed0):
    import mav_tube_trajectory_generation_amd as mtg
    return mtg.generate_random_problems(N, D, S, B, seed0=seed0)


@pytest.mark.parametrize("grad_mode", [0, 1, 2])
def test_time_cost_vs_oracle(ctx, dev, oracle, grad_mode, kernel):
    """objectiveFunctionTime (nonlinear_impl:877-945) with the gradient forms
    of getCostAndGradientTime (:2495-2584)."""
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 8, 16
    mask, fixed, times, _ = _batch(S, B, 500)
    times[3, 2] = 0.1   # exercise the clamp rule (nonlinear_impl:2529-2530)
    times[5, 0] = 0.07
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    out = plan.time_cost(torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev),
                         grad_mode=grad_mode, increment=0.1, w_d=0.1, w_t=1.0)
    cost = out["cost"].cpu().numpy()
    assert (out["status"].cpu().numpy() == 0).all()
    for b in range(B):
        v = standard_vertices(N, S, D, 500 + b)
        J, g = oracle.time_cost(N, R, v, times[b], grad_mode=grad_mode, increment=0.1,
                                w_d=0.1, w_t=1.0)
        # A segment time of 0.1 s makes A(T) ill-conditioned (cond ~1e10):
        # the reference-faithful oracle then carries ~1e-7 relative error in
        # J, which central differences amplify by J / (2 increment).
        well = times[b].min() > 0.5
        assert rel_err(cost[b], J) <= (1e-9 if well else 1e-6), b
        if grad_mode:
            gg = out["grad"].cpu().numpy()[b]
            if well:
                assert np.max(np.abs(gg - g)) <= 1e-6 * np.max(np.abs(g)) + 1e-9, (b, gg, g)
            elif grad_mode == 1:
                # The reference differences two full J_d sums
                # (nonlinear_impl:2549-2566); with one 0.1 s segment J_d is
                # ~1e14 and that cancels ~1e-3 of the gradient away.  Check
                # against the same derivative formed segment-wise from the
                # oracle's solution and H matrices instead; that solution is
                # itself only ~1e-5 accurate here (cond(A(0.1)) ~ 1e10).
                ref = _grad_mode1_segmentwise(oracle, v, times[b], 0.1, 0.1, 1.0)
                assert np.max(np.abs(gg - ref)) <= 1e-4 * np.max(np.abs(ref)), (b, gg, ref)
            else:
                assert np.max(np.abs(gg - g)) <= 1e-4 * np.max(np.abs(g)), (b, gg, g)


def _vertex_derivs(v, sol, N):
    """All vertex derivatives x[(S+1), M, D] from the oracle's d_f / d_p."""
    M = N // 2
    x = np.zeros((v.S + 1, M, v.D))
    f = p = 0
    for vi in range(v.S + 1):
        for k in range(M):
            if k < v.K and v.mask[vi, k]:
                x[vi, k] = sol["df"][:, f]
                f += 1
            else:
                x[vi, k] = sol["dp"][:, p]
                p += 1
    return x


def _grad_mode1_segmentwise(oracle, v, t, inc, w_d, w_t):
    sol = oracle.linear_solve(N, R, v, t)
    x = _vertex_derivs(v, sol, N)
    g = np.zeros(len(t))
    for n, Tn in enumerate(t):
        ts = 0.1 if Tn <= 0.1 else Tn - inc
        tb = 0.1 if Tn <= 0.1 else Tn + inc
        e = np.concatenate([x[n], x[n + 1]], axis=0)  # [N, D]
        Hs = oracle.segment_matrices(N, R, ts)[3]
        Hb = oracle.segment_matrices(N, R, tb)[3]
        g[n] = w_d * np.einsum("ad,ab,bd->", e, Hb - Hs, e) / (2 * inc) + w_t
    return g


def test_time_optimize_vs_reference_driver(ctx, dev, oracle, kernel):
    import mav_tube_trajectory_generation_amd as mtg
    S, B, E = 6, 8, 20
    mask, fixed, times, _ = _batch(S, B, 900)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    out = plan.time_optimize(torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev),
                             max_evals=E)
    T = out["times"].cpu().numpy()
    cost = out["cost"].cpu().numpy()
    evals = out["evals"].cpu().numpy()
    for b in range(B):
        v = standard_vertices(N, S, D, 900 + b)
        Tr, fr, er = optimize_reference(oracle, N, R, v, times[b], E)
        assert evals[b] == er, b
        assert np.max(np.abs(T[b] - Tr) / Tr) <= 1e-6, (b, T[b], Tr)
        assert rel_err(cost[b], fr) <= 1e-6, b
        Tc, fc, ec = oracle.time_optimize(N, R, v, times[b], E)
        assert ec == evals[b] and np.max(np.abs(T[b] - Tc) / Tc) <= 1e-6, b


def test_time_optimize_properties(ctx, dev, oracle, kernel):
    """BASELINE config 5 shape (reduced batch): 50 evaluations, bounds
    [0.1, 2 T0] (nonlinear_impl:350-378), monotone objective."""
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 10, 256
    mask, fixed, times, _ = _batch(S, B, 105)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    fd = torch.from_numpy(fixed).to(dev)
    td = torch.from_numpy(times).to(dev)
    c0 = plan.time_cost(fd, td)["cost"].cpu().numpy()
    out = plan.time_optimize(fd, td, max_evals=50)
    T = out["times"].cpu().numpy()
    c1 = out["cost"].cpu().numpy()
    assert (out["status"].cpu().numpy() == 0).all()
    assert np.all(out["evals"].cpu().numpy() <= 50)
    assert np.all(T >= 0.1 - 1e-15) and np.all(T <= 2 * times + 1e-12)
    assert np.all(c1 <= c0)
    assert np.mean(c1 / c0) < 0.9
    # The reported cost is the objective at the returned times.
    chk = plan.time_cost(fd, out["times"])["cost"].cpu().numpy()
    assert np.allclose(chk, c1, rtol=1e-12)


def _soft_limits(oracle, v, t):
    """Limits 3% above the start trajectory's max |v| and |a|: the soft cost
    is in its exponential regime (exp(100 * -0.03) ~ 0.05) and grows fast
    when the optimiser shortens the segments."""
    c = oracle.linear_solve(N, R, v, t)["coeffs"]
    return [(1, 1.03 * oracle.max_magnitude(N, c, t, 1)["value"]),
            (2, 1.03 * oracle.max_magnitude(N, c, t, 2)["value"])]


@pytest.mark.parametrize("grad_mode", [0, 2])
def test_time_cost_soft_constraints_vs_oracle(ctx, dev, oracle, grad_mode, kernel):
    """objectiveFunctionTime with use_soft_constraints (nonlinear_impl:907-913):
    J + sum_c min(1e12, exp((max_c - lim_c) / lim_c * 100))."""
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 8, 8
    mask, fixed, times, _ = _batch(S, B, 540)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    for b in range(B):
        v = standard_vertices(N, S, D, 540 + b)
        soft = _soft_limits(oracle, v, times[b])
        out = plan.time_cost(fd[b:b + 1], td[b:b + 1], grad_mode=grad_mode, soft=soft)
        J, g = oracle.time_cost(N, R, v, times[b], grad_mode=grad_mode, soft=soft)
        J0, _ = oracle.time_cost(N, R, v, times[b])
        assert J > J0  # the soft term is present
        assert rel_err(float(out["cost"][0]), J) <= 1e-9, b
        if grad_mode:
            gg = out["grad"].cpu().numpy()[0]
            assert np.max(np.abs(gg - g)) <= 1e-6 * np.max(np.abs(g)) + 1e-9, (b, gg, g)


def test_time_optimize_soft_constraints_vs_oracle(ctx, dev, oracle, kernel):
    """The device optimiser on the soft-constrained objective takes the same
    steps as the oracle port (orc_time_optimize_soft)."""
    import mav_tube_trajectory_generation_amd as mtg
    S, B, E = 6, 6, 20
    mask, fixed, times, _ = _batch(S, B, 940)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    agree = 0
    for b in range(B):
        v = standard_vertices(N, S, D, 940 + b)
        soft = _soft_limits(oracle, v, times[b])
        out = plan.time_optimize(fd[b:b + 1], td[b:b + 1], max_evals=E, soft=soft)
        T = out["times"].cpu().numpy()[0]
        Tc, fc, ec = oracle.time_optimize(N, R, v, times[b], E, soft=soft)
        # the reported cost is the soft objective at the returned times
        chk = plan.time_cost(fd[b:b + 1], out["times"], soft=soft)["cost"].cpu().numpy()[0]
        assert rel_err(float(out["cost"][0]), chk) <= 1e-12
        if int(out["evals"][0]) == ec and np.max(np.abs(T - Tc) / Tc) <= 1e-6:
            assert rel_err(float(out["cost"][0]), fc) <= 1e-6
            agree += 1
    # accept/reject decisions compare objectives whose soft terms amplify
    # rounding by the weight (100); allow one divergent path in six
    assert agree >= B - 1


def test_time_soft_rejects_bad_constraints(ctx, dev, kernel):
    import mav_tube_trajectory_generation_amd as mtg
    from mav_tube_trajectory_generation_amd._abi import MTGError
    S = 4
    mask, fixed, times, _ = _batch(S, 1, 5)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    for soft in ([(5, 1.0)], [(1, 0.0)], [(-1, 1.0)], [(1, 1.0)] * 9):
        with pytest.raises(MTGError):
            plan.time_cost(fd, td, soft=soft)


@pytest.mark.parametrize("start", ["feasible", "infeasible"])
def test_time_optimize_hard_constraints_vs_oracle(ctx, dev, oracle, kernel, start):
    """use_soft_constraints = false (nonlinear_impl:861-872): the magnitude
    constraints are inequalities max |p^(k)| - limit <= tolerance
    (evaluateMaximumMagnitudeConstraint, :2687-2733).  The device optimiser
    takes the oracle port's steps (orc_time_optimize_hard: feasible trials
    must lower J; from an infeasible start the largest violation must drop);
    a feasible start stays feasible.  The cost carries no soft term."""
    import mav_tube_trajectory_generation_amd as mtg
    S, B, E, tol = 6, 6, 20, 0.1
    scale = 1.02 if start == "feasible" else 0.9
    mask, fixed, times, _ = _batch(S, B, 960)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    agree = 0
    for b in range(B):
        v = standard_vertices(N, S, D, 960 + b)
        c0 = oracle.linear_solve(N, R, v, times[b])["coeffs"]
        lims = [(1, scale * oracle.max_magnitude(N, c0, times[b], 1)["value"]),
                (2, scale * oracle.max_magnitude(N, c0, times[b], 2)["value"])]
        J0 = plan.time_cost(fd[b:b + 1], td[b:b + 1], soft=lims, hard=True,
                            hard_tolerance=tol)["cost"].cpu().numpy()[0]
        Jp, _ = oracle.time_cost(N, R, v, times[b])
        assert rel_err(J0, Jp) <= 1e-9  # no soft term
        out = plan.time_optimize(fd[b:b + 1], td[b:b + 1], max_evals=E, soft=lims, hard=True,
                                 hard_tolerance=tol)
        T = out["times"].cpu().numpy()[0]
        Tc, fc, ec = oracle.time_optimize(N, R, v, times[b], E, soft=lims, hard=True,
                                          hard_tolerance=tol)
        c1 = oracle.linear_solve(N, R, v, T)["coeffs"]
        viol = max(oracle.max_magnitude(N, c1, T, k)["value"] - lim - tol for k, lim in lims)
        if start == "feasible":
            assert viol <= 1e-9, viol
        else:
            # From an infeasible start the steps descend the violation.
            viol0 = max(oracle.max_magnitude(N, c0, times[b], k)["value"] - lim - tol
                        for k, lim in lims)
            assert viol0 > 0.0 and viol < viol0, (viol0, viol)
        if int(out["evals"][0]) == ec and np.max(np.abs(T - Tc) / Tc) <= 1e-6:
            assert rel_err(float(out["cost"][0]), fc) <= 1e-6
            agree += 1
    assert agree >= B - 1, agree


def test_hard_constraints_only_where_implemented(ctx, dev):
    import mav_tube_trajectory_generation_amd as mtg
    from mav_tube_trajectory_generation_amd._abi import MTGError
    S = 4
    mask, fixed, times, _ = _batch(S, 1, 5)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    dp = torch.zeros((1, D, plan.n_free), dtype=torch.float64, device=dev)
    from mav_tube_trajectory_generation_amd._abi import check, lib, make_time_params
    import ctypes
    p = make_time_params(soft=[(1, 3.0)], hard=True)
    cost = torch.empty(1, dtype=torch.float64, device=dev)
    rc = lib().mtg_free_cost(plan._h, 1, ctypes.c_void_p(fd.data_ptr()),
                             ctypes.c_void_p(dp.data_ptr()), ctypes.c_void_p(td.data_ptr()),
                             ctypes.byref(p), 1, ctypes.c_void_p(cost.data_ptr()), None, None,
                             None)
    assert rc == -1  # MTG_ERR_INVALID_ARG
    with pytest.raises(MTGError):
        plan.time_cost(fd, td, soft=[(1, 3.0)], hard=True, hard_tolerance=-1.0)
    check(0, "ok")


@pytest.mark.parametrize("S", [2, 3, 5, 7, 11, 13, 16])
def test_time_cost_wave_kernels_every_s(ctx, dev, oracle, S):
    """time_cost_wave_kernel<10, 4, 3, S> (AUTO on the standard pattern,
    S = 2..16) against the oracle's objective and mode-2 gradient."""
    import mav_tube_trajectory_generation_amd as mtg
    B = 4
    mask, fixed, times, _ = _batch(S, B, 900 + 10 * S)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    out = plan.time_cost(torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev),
                         grad_mode=2, increment=0.1, w_d=0.1, w_t=1.0)
    cost = out["cost"].cpu().numpy()
    grad = out["grad"].cpu().numpy()
    assert (out["status"].cpu().numpy() == 0).all()
    for b in range(B):
        v = standard_vertices(N, S, D, 900 + 10 * S + b)
        J, g = oracle.time_cost(N, R, v, times[b], grad_mode=2, increment=0.1, w_d=0.1, w_t=1.0)
        tol = 1e-9 if times[b].min() > 0.5 else 1e-6
        assert rel_err(cost[b], J) <= tol, (S, b)
        assert np.max(np.abs(grad[b] - g)) <= 1e-5 * np.max(np.abs(g)) + 1e-9, (S, b)
