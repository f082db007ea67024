"""The reference's actual kOptimizeTime path: LN_SBPLX (the default,
polynomial_optimization_nonlinear.h:61) over the fork's objectiveFunctionTime,
which re-solves the tube QCQP at every evaluation
(impl/polynomial_optimization_nonlinear_impl.h:332-397, 877-945; solveQCQP at
:892).  The device runs Subplex (mtg_sbplx_device.h) one evaluation per round
over batched tube solves (mtg_tube_time_optimize_ex, optimizer 1); the oracle
runs its Subplex restatement (orc_sbplx.cpp) on its own interior-point QCQP
(orc_tube_time_optimize_sbplx).

NLopt and MOSEK are absent, so this is parity against the oracle's
restatements.  The two QCQP solvers agree to ~1e-9 relative;
Subplex compares objective values, so a comparison that lands on a near-tie
can send one trajectory down another path: agreement is required on all but
one of every 16 (evaluation count, stopping code, final point within 1e-6,
cost within 1e-6)."""
import concurrent.futures as cf

import numpy as np
import pytest

from helpers import rel_err
from test_tube_gpu import tube_inputs

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N, R = 10, 4
M = N // 2
RADIUS = 0.15


def _T(dev, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _problems(oracle, S, seeds):
    vs = [oracle.random_vertices(M - 1, S, 3, -10.0, 10.0, s) for s in seeds]
    times = np.stack([oracle.estimate_segment_times(v, 3.0, 5.0) for v in vs])
    return vs, times


def _run(ctx, dev, vs, times, E, **kw):
    import mav_tube_trajectory_generation_amd as mtg
    B, S = times.shape
    pos = _T(dev, np.stack([tube_inputs(v)[0] for v in vs]))
    fv = _T(dev, np.stack([tube_inputs(v)[1] for v in vs]))
    radii = _T(dev, np.full((B, S, 2), RADIUS))
    out = mtg.tube_time_optimize(ctx, N, R, pos, fv, radii, _T(dev, times), max_evals=E,
                                 optimizer="sbplx", **kw)
    torch.cuda.synchronize()
    return (pos, fv, radii), {k: v.cpu().numpy() for k, v in out.items()}


def _agree(oracle, vs, times, out, E, picks, **kw):
    S = times.shape[1]

    def ref(b):
        return b, oracle.tube_time_optimize_sbplx(N, R, vs[b], times[b], np.full((S, 2), RADIUS),
                                                  E, **kw)
    agree, n = 0, 0
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        for b, r in ex.map(ref, picks):
            n += 1
            if (r["evals"] == out["evals"][b] and r["result"] == out["result"][b]
                    and np.max(np.abs(out["times"][b] - r["times"]) / r["times"]) <= 1e-6):
                assert rel_err(out["cost"][b], r["cost"]) <= 1e-6, (b, out["cost"][b], r["cost"])
                agree += 1
    return agree, n


def test_tube_sbplx_matches_oracle(ctx, dev, oracle):
    """S = 10, 50 evaluations (config 5's budget in the fork's QCQP form):
    16 strided trajectories of a 256 batch take the oracle's path; every
    trajectory keeps the bounds and the budget, never ends above J(T0), and
    its reported cost is the objective at the returned times."""
    import mav_tube_trajectory_generation_amd as mtg
    S, B, E = 10, 256, 50
    vs, times = _problems(oracle, S, range(700, 700 + B))
    geo, out = _run(ctx, dev, vs, times, E)
    assert (out["status"] == 0).all()
    assert np.all((out["evals"] >= 1) & (out["evals"] <= E))
    assert set(np.unique(out["result"])) <= {3, 4, 5}
    Tt = out["times"]
    assert np.all(Tt >= 0.1 - 1e-15) and np.all(Tt <= 2 * times + 1e-12)
    pos, fv, radii = geo
    t0 = _T(dev, times)
    c0 = mtg.tube_time_cost(ctx, N, R, pos, fv, t0, t0, radii)["cost"].cpu().numpy()
    assert np.all(out["cost"] <= c0)
    chk = mtg.tube_time_cost(ctx, N, R, pos, fv, t0, _T(dev, Tt), radii)["cost"].cpu().numpy()
    assert np.allclose(chk, out["cost"], rtol=1e-12)
    agree, n = _agree(oracle, vs, times, out, E, list(range(0, B, B // 16)))
    assert agree >= n - 1, (agree, n)


@pytest.mark.parametrize("S", [2, 3, 7])
def test_tube_sbplx_segment_counts(ctx, dev, oracle, S):
    """Subspace partitions of other shapes (n = nsmin, n = nsmin + 1, n >
    nsmax), budgets that stop by maxeval and by ftol."""
    B = 16
    vs, times = _problems(oracle, S, range(800, 800 + B))
    for E, f_rel in ((30, 0.05), (80, 1e-6)):
        _, out = _run(ctx, dev, vs, times, E, f_rel=f_rel)
        assert (out["status"] == 0).all()
        agree, n = _agree(oracle, vs, times, out, E, list(range(0, B, 2)), f_rel=f_rel)
        assert agree >= n - 1, (S, E, agree, n)


def test_tube_sbplx_soft_constraints(ctx, dev, oracle):
    """Soft magnitude constraints enter the objective after each QCQP
    (use_soft_constraints, nonlinear_impl:907-913)."""
    S, B, E = 5, 16, 30
    vs, times = _problems(oracle, S, range(900, 900 + B))
    soft = [(1, 3.0), (2, 5.0)]
    _, out = _run(ctx, dev, vs, times, E, soft=soft)
    agree, n = _agree(oracle, vs, times, out, E, list(range(0, B, 2)), soft=soft)
    assert agree >= n - 1, (agree, n)


def test_tube_sbplx_start_out_of_bounds(ctx, dev, oracle):
    """A segment time below kOptimizationTimeLowerBound (0.1) is NLopt's
    invalid start (nlopt_optimize: NLOPT_INVALID_ARGS, turned into
    nlopt::FAILURE by optimizeTime, nonlinear_impl:389-394): result -1, no
    evaluation, times unchanged, on the device and in the oracle.  The other
    trajectories of the batch run normally."""
    S, B, E = 4, 4, 20
    vs, times = _problems(oracle, S, range(950, 950 + B))
    times[1, 2] = 0.08   # below the lower bound
    times[3, 0] = 0.04   # lb > ub = 2 T0
    _, out = _run(ctx, dev, vs, times, E)
    for b in (1, 3):
        assert out["result"][b] == -1 and out["evals"][b] == 0, b
        assert np.array_equal(out["times"][b], times[b])
        assert np.isnan(out["cost"][b])
        r = oracle.tube_time_optimize_sbplx(N, R, vs[b], times[b], np.full((S, 2), RADIUS), E)
        assert r["result"] == -1 and r["evals"] == 0 and np.array_equal(r["times"], times[b])
    for b in (0, 2):
        assert out["result"][b] in (3, 4, 5) and out["evals"][b] >= 1


def test_tube_sbplx_poisoned_workspace_and_graph(ctx, dev, oracle):
    """Every scratch word (the machine states included) is written before it
    is read: a 0xFF-filled workspace gives bit-identical results; and the
    whole call captures in a HIP graph whose replay gives the eager result."""
    import mav_tube_trajectory_generation_amd as mtg
    from mav_tube_trajectory_generation_amd._abi import make_time_params
    S, B, E = 6, 8, 25
    vs, times = _problems(oracle, S, range(980, 980 + B))
    pos = _T(dev, np.stack([tube_inputs(v)[0] for v in vs]))
    fv = _T(dev, np.stack([tube_inputs(v)[1] for v in vs]))
    radii = _T(dev, np.full((B, S, 2), RADIUS))
    t0 = _T(dev, times)
    p = make_time_params(grad_mode=2, optimizer="sbplx")
    nb = mtg.tube_time_workspace_bytes(N, S, B, p, True)
    # the LN_SBPLX workspace is the one-point layout plus the machine states
    assert nb < mtg.tube_time_workspace_bytes(N, S, B, make_time_params(grad_mode=2), True)
    outs = []
    for fill in (0x00, 0xFF):
        ws = torch.full((nb,), fill, dtype=torch.uint8, device=dev)
        outs.append(mtg.tube_time_optimize(ctx, N, R, pos, fv, radii, t0, max_evals=E,
                                           optimizer="sbplx", workspace=ws))
    for k in ("times", "cost", "evals", "result", "status"):
        assert torch.equal(outs[0][k], outs[1][k]), k
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        tin = t0.clone()
        with torch.cuda.graph(g, stream=side):
            got = mtg.tube_time_optimize(ctx, N, R, pos, fv, radii, tin, max_evals=E,
                                         optimizer="sbplx", workspace=ws)
    g.replay()
    torch.cuda.synchronize()
    for k in ("times", "cost", "evals", "result", "status"):
        assert torch.equal(got[k], outs[0][k]), k
