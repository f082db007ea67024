"""The reference's default time optimiser on the device: LN_SBPLX
(nlopt::LN_SBPLX, polynomial_optimization_nonlinear.h:61; optimizeTime,
impl/polynomial_optimization_nonlinear_impl.h:332-397, on
objectiveFunctionTime, :877-945) restated in mtg_sbplx_device.h, against the
oracle's CPU restatement (oracle/orc_sbplx.cpp, itself pinned evaluation for
evaluation to an independent Python restatement in tests/test_sbplx.py).

NLopt is absent, so parity with NLopt itself is unpinned.  Subplex compares
objective values that the device (block LDL^T) and the oracle (QR) compute
~1e-12 apart; a comparison that lands on a near-tie can send a trajectory
down another path, so agreement is required on all but one of every 16.
"""
import concurrent.futures as cf

import numpy as np
import pytest

from helpers import rel_err, standard_vertices

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N, D, R = 10, 3, 4


def _run(ctx, dev, S, B, E, kernel="auto", seed0=105, d=D, r=R, times_fn=None, **kw):
    import mav_tube_trajectory_generation_amd as mtg
    mask, fixed, times, _ = mtg.generate_random_problems(N, d, S, B, seed0=seed0)
    if times_fn is not None:
        times_fn(times)
    plan = mtg.LinearPlan(ctx, N, d, r, S, mask).set_kernel(kernel)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    out = plan.time_optimize(fd, td, max_evals=E, optimizer="sbplx", **kw)
    torch.cuda.synchronize()
    return plan, fd, td, times, {k: v.cpu().numpy() for k, v in out.items()}


def _agree(oracle, out, times, S, E, picks, seed0=105, d=D, r=R, **kw):
    def ref(b):
        return b, oracle.time_optimize_sbplx(N, r, standard_vertices(N, S, d, seed0 + b),
                                             times[b], E, **kw)
    agree, n = 0, 0
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        for b, (Tc, fc, ec, rc, _) in ex.map(ref, picks):
            n += 1
            if (ec == out["evals"][b] and rc == out["result"][b]
                    and np.max(np.abs(out["times"][b] - Tc) / Tc) <= 1e-6):
                assert rel_err(out["cost"][b], fc) <= 1e-6, b
                agree += 1
    return agree, n


def test_config5_sbplx_matches_oracle(ctx, dev, oracle):
    """Config 5 (4096 x 50 evaluations) in the reference's algorithm: 16
    strided trajectories take the oracle's path (evaluation count, stopping
    code, final point, cost); every trajectory keeps the bounds and the
    budget and never ends above its start."""
    S, B, E = 10, 4096, 50
    plan, fd, td, times, out = _run(ctx, dev, S, B, E)
    assert (out["status"] == 0).all()
    assert np.all((out["evals"] >= 1) & (out["evals"] <= E))
    assert np.array_equal(out["solves"], out["evals"])  # gradient-free
    assert set(np.unique(out["result"])) <= {3, 4, 5}
    Tt = out["times"]
    assert np.all(Tt >= 0.1 - 1e-15) and np.all(Tt <= 2 * times + 1e-12)
    c0 = plan.time_cost(fd, td)["cost"].cpu().numpy()
    assert np.all(out["cost"] <= c0)
    chk = plan.time_cost(fd, torch.from_numpy(Tt).to(dev))["cost"].cpu().numpy()
    assert np.allclose(chk, out["cost"], rtol=1e-12)
    agree, n = _agree(oracle, out, times, S, E, list(range(0, B, B // 16)))
    assert agree >= n - 1, (agree, n)


@pytest.mark.parametrize("S", [2, 3, 5, 7, 12, 16])
def test_sbplx_segment_counts(ctx, dev, oracle, S):
    """Subspace partitions of every shape (n < nsmin, n = nsmin + 1, n > 2
    nsmax, the largest n), budgets that stop by maxeval and by ftol."""
    B = 24
    for E, f_rel in ((40, 0.05), (120, 1e-6)):
        _, _, _, times, out = _run(ctx, dev, S, B, E, f_rel=f_rel)
        assert (out["status"] == 0).all()
        agree, n = _agree(oracle, out, times, S, E, list(range(0, B, 3)), f_rel=f_rel)
        assert agree >= n - 1, (S, E, agree, n)


def test_sbplx_generic_kernel(ctx, dev, oracle):
    """The generic-pattern kernel runs the same machine."""
    S, B, E = 6, 32, 60
    _, _, _, times, out = _run(ctx, dev, S, B, E, kernel="generic")
    agree, n = _agree(oracle, out, times, S, E, list(range(0, B, 4)))
    assert agree >= n - 1, (agree, n)


@pytest.mark.parametrize("d,r,S", [(2, 4, 6), (3, 3, 6), (1, 2, 5), (3, 4, 20)],
                         ids=["D2", "r3", "D1r2", "S20"])
def test_sbplx_runtime_s_kernel(ctx, dev, oracle, d, r, S):
    """The runtime-S standard kernel (time_optimize_std_kernel: r = 2/3,
    D < 3, or S beyond the compile-time-S kernels' 16) runs the same machine,
    its state sized by S in LDS after the solver's (more than 16 segments,
    the default kOptimizeTime path of the C++ shim for long trajectories)."""
    B, E = 24, 60
    _, _, _, times, out = _run(ctx, dev, S, B, E, d=d, r=r)
    assert (out["status"] == 0).all()
    agree, n = _agree(oracle, out, times, S, E, list(range(0, B, 3)), d=d, r=r)
    assert agree >= n - 1, (d, r, S, agree, n)


@pytest.mark.parametrize("kernel", ["auto", "generic"])
def test_sbplx_start_out_of_bounds(ctx, dev, oracle, kernel):
    """A segment time below kOptimizationTimeLowerBound (0.1) is NLopt's
    invalid start (nlopt_optimize returns NLOPT_INVALID_ARGS before any
    evaluation; optimizeTime returns nlopt::FAILURE, nonlinear_impl:389-394):
    result -1, no evaluation, times unchanged, cost NaN, as the oracle."""
    S, B, E = 5, 4, 30

    def shorten(t):
        t[1, 2] = 0.08
        t[3, 0] = 0.04  # lb > ub as well

    _, _, _, times, out = _run(ctx, dev, S, B, E, kernel=kernel, times_fn=shorten)
    for b in (1, 3):
        assert out["result"][b] == -1 and out["evals"][b] == 0, (b, out["result"][b])
        assert np.array_equal(out["times"][b], times[b]) and np.isnan(out["cost"][b])
        Tc, fc, ec, rc, _ = oracle.time_optimize_sbplx(
            N, R, standard_vertices(N, S, D, 105 + b), times[b], E)
        assert rc == -1 and ec == 0 and np.array_equal(Tc, times[b])
    for b in (0, 2):
        assert out["result"][b] in (3, 4, 5) and out["evals"][b] >= 1


def test_sbplx_soft_constraints(ctx, dev, oracle):
    """Soft magnitude constraints enter the objective (use_soft_constraints,
    nonlinear_impl:907-913, evaluateMaximumMagnitudeAsSoftConstraint
    :2735-2766)."""
    S, B, E = 10, 32, 50
    soft = [(1, 3.0), (2, 5.0)]
    _, _, _, times, out = _run(ctx, dev, S, B, E, soft=soft)
    agree, n = _agree(oracle, out, times, S, E, list(range(0, B, 4)), soft=soft)
    assert agree >= n - 1, (agree, n)


def test_sbplx_rejects_hard_constraints(ctx, dev):
    import mav_tube_trajectory_generation_amd as mtg
    with pytest.raises(mtg.MTGError):
        _run(ctx, dev, 10, 4, 20, soft=[(1, 3.0)], hard=True)


def test_sbplx_graph_capture(ctx, dev):
    import mav_tube_trajectory_generation_amd as mtg
    S, B, E = 10, 256, 50
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=105)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    eager = {k: v.clone() for k, v in
             plan.time_optimize(fd, td, max_evals=E, optimizer="sbplx").items()}
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        got = plan.time_optimize(fd, td, max_evals=E, optimizer="sbplx")
    g.replay()
    torch.cuda.synchronize()
    for k in eager:
        assert torch.equal(got[k], eager[k]), k
