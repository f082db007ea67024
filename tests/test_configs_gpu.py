"""Every BASELINE.json configuration at its stated size on one MI355X.

Config 2 (1024) lives in test_linear_gpu.py.  Here:
  * config 4 on one GPU: one 8192-trajectory shard and the whole 65536 batch;
  * config 3: 4096 tube QCQPs;
  * config 5: 4096 trajectories x 50 objective evaluations.
Each checks the status of every trajectory, the size-independent properties
of the reference's tests on every trajectory (checkPath:
test/test_polynomial_optimization.cpp:113-172 -- fixed constraints met,
C^(N/2-1) continuity; feasibility for the tube; bounds and monotone cost for
the optimiser) and strided oracle spot checks at the 1e-6 parity bar.
"""
import concurrent.futures as cf

import numpy as np
import pytest

from helpers import REL_TOL, optimize_reference, rel_err, rel_err_coeffs, standard_vertices

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N, D, R = 10, 3, 4
M = N // 2


def _pool():
    # ctypes releases the GIL, so oracle calls run in parallel threads.
    return cf.ThreadPoolExecutor(max_workers=8)


def _deriv_factors(deriv):
    k = np.arange(N)
    f = np.ones(N)
    for m in range(deriv):
        f = f * np.maximum(k - m, 0)
    return f


def check_path_batch(coeffs, times, fixed, positions, tol=1e-6):
    """checkPath on every trajectory of a standard-pattern batch, vectorised:
    start/end derivatives 0..M-1 as fixed (start/end fully constrained, the
    rest zero), intermediate positions, and C^(M-1) continuity."""
    k = np.arange(N)
    for deriv in range(M):
        f = _deriv_factors(deriv)
        pw = np.where(k >= deriv, times[:, :, None] ** np.maximum(k - deriv, 0)[None, None, :],
                      0.0)
        end_val = np.einsum("bsdk,bsk->bsd", coeffs * f, pw)
        start_val = coeffs[:, :, :, deriv] * f[deriv]
        scale = np.maximum(1.0, np.abs(end_val[:, :-1]))
        assert np.all(np.abs(end_val[:, :-1] - start_val[:, 1:]) <= tol * scale), deriv
        want_start = positions[:, 0, :] if deriv == 0 else 0.0
        want_end = positions[:, -1, :] if deriv == 0 else 0.0
        assert np.all(np.abs(start_val[:, 0] - want_start) <= tol * np.maximum(1.0, np.abs(
            want_start))), deriv
        assert np.all(np.abs(end_val[:, -1] - want_end) <= tol * np.maximum(1.0, np.abs(
            want_end))), deriv
        if deriv == 0:
            # intermediate vertex positions (fixed in the standard pattern)
            assert np.all(np.abs(start_val[:, 1:] - positions[:, 1:-1, :]) <=
                          tol * np.maximum(1.0, np.abs(positions[:, 1:-1, :])))
    # fixed_vals holds the start derivatives in its first columns
    assert np.allclose(coeffs[:, 0, :, 0], fixed[:, :, 0], atol=1e-12)


@pytest.mark.parametrize("B", [8192, 65536])
def test_config4_linear_at_size(ctx, dev, oracle, B):
    """BASELINE config 4 on one GPU: an 8192-trajectory shard (8-way) and the
    whole 65536 batch, seeds 105 + global index."""
    import mav_tube_trajectory_generation_amd as mtg
    S = 10
    mask, fixed, times, pos = mtg.generate_random_problems(N, D, S, B, seed0=105)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    out = plan.solve(torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev))
    torch.cuda.synchronize()
    st = out["status"].cpu().numpy()
    coeffs = out["coeffs"].cpu().numpy()
    cost = out["cost"].cpu().numpy()
    assert (st == 0).all()
    assert np.all(np.isfinite(cost)) and np.all(cost > 0)
    check_path_batch(coeffs, times, fixed, pos)
    picks = list(range(0, B, B // 64)) + [B - 1]

    def ref(b):
        return b, oracle.linear_solve(N, R, standard_vertices(N, S, D, 105 + b), times[b])

    with _pool() as ex:
        for b, r in ex.map(ref, picks):
            assert rel_err_coeffs(coeffs[b], r["coeffs"]) <= REL_TOL, b
            assert rel_err(cost[b], r["cost"]) <= REL_TOL, b


def _tube_batch(B, S, seed0=105):
    import mav_tube_trajectory_generation_amd as mtg
    mask, fixed, times, pos = mtg.generate_random_problems(N, D, S, B, seed0=seed0)
    tf = np.zeros((B, 3, N))
    tf[:, :, 0] = pos[:, 0, :]
    tf[:, :, M] = pos[:, S, :]
    return times, pos, tf


def test_config3_tube_at_size(ctx, dev, oracle):
    """BASELINE config 3: 4096 x 10-segment tube QCQPs (radii 0.15).  Every
    converged solve is feasible to 1e-7 (1e3 tol); the breakdown rate is no worse than
    the oracle IPM's on the same seeds (every problem re-solved on the CPU);
    32 strided converged problems agree with the oracle at 1e-6."""
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 10, 4096
    times, pos, tf = _tube_batch(B, S)
    radii = np.full((B, S, 2), 0.15)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    out = mtg.tube_solve(ctx, N, R, T(pos), T(tf), T(times), T(times), T(radii))
    res = mtg.tube_residuals(ctx, N, R, T(pos), T(tf), T(times), T(times), T(radii), out["x"])
    torch.cuda.synchronize()
    st = out["status"].cpu().numpy()
    x = out["x"].cpu().numpy()
    coeffs = out["coeffs"].cpu().numpy()
    cost = out["cost"].cpu().numpy()
    resid = res.cpu().numpy()
    conv = st == 0
    near = st == 4  # MTG_TRAJ_NEAR_OPTIMAL: stopped at a breakdown within 1e3 tol
    usable = conv | near
    hist = dict(zip(*np.unique(st, return_counts=True)))
    print("config 3 GPU status histogram", hist)
    assert set(np.unique(st)) <= {0, 2, 3, 4}
    # converged: primal feasible to tol (g_k = -s_k + rp_k, rp <= tol)
    assert resid[conv].max() <= 1e-10
    if near.any():
        assert resid[near].max() <= 1e3 * 1e-10
    print("config 3 max residual (converged)", resid[conv].max())
    assert np.all(np.isfinite(cost[usable]))

    rad1 = np.full((S, 2), 0.15)

    def ref(b):
        v = standard_vertices(N, S, D, 105 + b)
        try:
            return b, oracle.tube_solve(N, R, v, times[b], rad1, tol=1e-10, max_iter=100)
        except RuntimeError:  # -22: breakdown away from the optimum, no solution
            return b, {"status": -22}

    with _pool() as ex:
        refs = dict(ex.map(ref, range(B)))
    ost = np.array([refs[b]["status"] for b in range(B)])
    print("config 3 oracle status histogram", dict(zip(*np.unique(ost, return_counts=True))))
    # The GPU fails (no usable point) no more often than the oracle, and at
    # most 0.25 % of the problems (the complementarity floor of the IPM,
    # mtg_tube_device.h ipm(); 0 of 2,400 oracle breakdowns).
    o_usable = (ost == 0) | (ost == 3)
    assert (~usable).sum() <= (~o_usable).sum(), ((~usable).sum(), (~o_usable).sum())
    assert (~usable).sum() <= 0.0025 * B and (~o_usable).sum() <= 0.0025 * B
    # Round 6 (regularised retry of a failed KKT factorisation):
    # every config-3 problem has a usable solution on the GPU (round 5: two
    # near-optimal stops), and both implementations converge together.
    assert usable.all(), hist
    print("config 3 converged on both", int((conv & (ost == 0)).sum()), "of", B)
    assert (conv & (ost == 0)).sum() >= 0.999 * B
    both = np.nonzero(conv & (ost == 0))[0]
    for b in both[::max(1, len(both) // 32)][:33]:
        r = refs[b]
        assert rel_err_coeffs(x[b], r["x"]) <= 1e-6, b
        assert rel_err_coeffs(coeffs[b], r["coeffs"]) <= 1e-6, b
        assert rel_err(cost[b], r["cost"]) <= 1e-6, b


def test_config5_time_allocation_at_size(ctx, dev, oracle):
    """BASELINE config 5: 4096 trajectories x 50 objective evaluations.
    Bounds [0.1, 2 T0], at most 50 evaluations, monotone objective, the
    reported cost equals the objective at the returned times; 16 strided
    trajectories take the same steps as the oracle port of the optimiser."""
    import mav_tube_trajectory_generation_amd as mtg
    S, B, E = 10, 4096, 50
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=105)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    c0 = plan.time_cost(fd, td)["cost"].cpu().numpy()
    out = plan.time_optimize(fd, td, max_evals=E)
    Tt = out["times"].cpu().numpy()
    c1 = out["cost"].cpu().numpy()
    ev = out["evals"].cpu().numpy()
    sv = out["solves"].cpu().numpy()
    assert (out["status"].cpu().numpy() == 0).all()
    assert np.all((ev >= 1) & (ev <= E))
    # base point + 2S gradient points per accepted step + one solve per trial
    assert np.all(sv >= ev + 2 * S) and np.all((sv - ev) % (2 * S) == 0)
    assert np.all(Tt >= 0.1 - 1e-15) and np.all(Tt <= 2 * times + 1e-12)
    assert np.all(c1 <= c0)
    chk = plan.time_cost(fd, out["times"])["cost"].cpu().numpy()
    assert np.allclose(chk, c1, rtol=1e-12)
    picks = list(range(0, B, B // 16))

    def ref(b):
        return b, oracle.time_optimize(N, R, standard_vertices(N, S, D, 105 + b), times[b], E)

    agree = 0
    with _pool() as ex:
        for b, (Tc, fc, ec) in ex.map(ref, picks):
            if ec == ev[b] and np.max(np.abs(Tt[b] - Tc) / Tc) <= 1e-6:
                assert rel_err(c1[b], fc) <= 1e-6, b
                agree += 1
    # Accept/reject compares objectives that differ by rounding only when a
    # trial lands on a near-tie; allow one divergent path in sixteen.
    assert agree >= len(picks) - 1, agree


@pytest.mark.parametrize("kernel", ["standard", "generic"])
def test_time_optimize_kernels_agree_at_size(ctx, dev, kernel):
    """The standard-pattern and generic time kernels on the same 512
    trajectories.  They sum J in different orders (time-scaled H(1) vs the
    reference's A^-T Q A^-1), ~1e-12 apart, which the central-difference
    gradient amplifies by J / (2 increment); an accept/reject on a near-tie
    can then take another path.  So: >= 95 % of the trajectories take the
    same path (same evaluation count, times within 1e-4), the final
    objectives agree to 1e-6 on >= 90 % and to 1e-3 on >= 98 % (measured on
    MI355X: 50 % / 90 % / 99 % quantiles 2e-11 / 2e-8 / 4e-4).  Step-by-step parity of both
    kernels with the oracle port is test_time_gpu.py's."""
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 10, 512
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=4000)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    pa = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    pb = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel("standard")
    assert pa.kernel == kernel
    a, b = pa.time_optimize(fd, td, 50), pb.time_optimize(fd, td, 50)
    ea, eb = a["evals"].cpu().numpy(), b["evals"].cpu().numpy()
    ta, tb = a["times"].cpu().numpy(), b["times"].cpu().numpy()
    ca, cb = a["cost"].cpu().numpy(), b["cost"].cpu().numpy()
    dt = np.max(np.abs(ta - tb) / tb, axis=1)
    dc = np.abs(ca - cb) / cb
    print(f"{kernel} vs standard: same evals {np.mean(ea == eb):.3f}, time diff quantiles "
          f"{np.quantile(dt, [0.5, 0.9, 0.99])}, cost diff quantiles "
          f"{np.quantile(dc, [0.5, 0.9, 0.99])}")
    assert np.mean(ea == eb) >= 0.95
    assert np.mean(dt <= 1e-4) >= 0.95
    assert np.mean(dc <= 1e-6) >= 0.9
    assert np.mean(dc <= 1e-3) >= 0.98


def test_time_optimize_n8_generic_vs_oracle(ctx, dev, oracle):
    """N = 8 (the generic time kernel; the standard one is N = 10 only)
    against the oracle port of the optimiser."""
    import mav_tube_trajectory_generation_amd as mtg
    n8, r8, S, B, E = 8, 3, 6, 8, 20
    mask, fixed, times, _ = mtg.generate_random_problems(n8, D, S, B, seed0=700)
    plan = mtg.LinearPlan(ctx, n8, D, r8, S, mask)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    out = plan.time_optimize(fd, td, max_evals=E)
    Tt = out["times"].cpu().numpy()
    c1 = out["cost"].cpu().numpy()
    ev = out["evals"].cpu().numpy()
    for b in range(B):
        v = oracle.random_vertices(n8 // 2 - 1, S, D, -10.0, 10.0, 700 + b)
        Tr, fr, er = optimize_reference(oracle, n8, r8, v, times[b], E)
        assert ev[b] == er, b
        assert np.max(np.abs(Tt[b] - Tr) / Tr) <= 1e-6, b
        assert rel_err(c1[b], fr) <= 1e-6, b
