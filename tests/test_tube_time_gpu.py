"""GPU parity of the segment-time objective with the QCQP inner solve (the
fork's objectiveFunctionTime, nonlinear_impl:877-945, solveQCQP at :892;
mtg_tube_time_cost) and of its optimiser (mtg_tube_time_optimize) against
the oracle (orc_tube_time_cost / orc_tube_time_optimize).

The QCQP values agree to the interior-point tolerance (test_tube_gpu.py:
1e-6 relative), so J is compared at 1e-6 of the QCQP cost; the time
penalty (sum T)^2 is exact arithmetic on both sides.  The gradient is a
difference of two such values over 2h, compared at the same absolute error
divided by h.  MOSEK is absent: the QCQP itself is parity-unpinned against
the reference and pinned against SciPy in test_tube_oracle.py."""
import numpy as np
import pytest

from test_tube_gpu import main_cpp_vertices, tube_inputs

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N, R = 10, 4
M = N // 2
H = 0.1


def _T(dev, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _batch(oracle, S, seeds):
    items = []
    for s in seeds:
        v = oracle.random_vertices(M - 1, S, 3, -10.0, 10.0, s)
        items.append((v, oracle.estimate_segment_times(v, 3.0, 5.0)))
    return items


def _geometry(dev, items, radius=0.15):
    S = items[0][0].S
    pos = np.stack([tube_inputs(v)[0] for v, _ in items])
    fv = np.stack([tube_inputs(v)[1] for v, _ in items])
    radii = np.full((len(items), S, 2), radius)
    return _T(dev, pos), _T(dev, fv), _T(dev, radii)


@pytest.mark.parametrize("soft", [False, True], ids=["nosoft", "soft"])
def test_tube_time_cost_vs_oracle(ctx, dev, oracle, soft):
    import mav_tube_trajectory_generation_amd as mtg
    S = 6
    items = _batch(oracle, S, range(300, 306))
    rng = np.random.default_rng(4)
    t0 = np.stack([t for _, t in items])
    t = t0 * rng.uniform(0.85, 1.15, size=t0.shape)  # stale control-point maps
    pos, fv, radii = _geometry(dev, items)
    # soft limits near the QCQP trajectories' own maxima (exponential regime)
    spec = None
    if soft:
        ref0 = oracle.tube_solve(N, R, items[0][0], t[0], np.full((S, 2), 0.15), times_cp=t0[0])
        spec = [(k, 1.03 * oracle.max_magnitude(N, ref0["coeffs"], t[0], k)["value"])
                for k in (1, 2)]
    out = mtg.tube_time_cost(ctx, N, R, pos, fv, _T(dev, t0), _T(dev, t), radii, grad=True,
                             soft=spec)
    J = out["cost"].cpu().numpy()
    g = out["grad"].cpu().numpy()
    st = out["status"].cpu().numpy()
    for b, (v, _) in enumerate(items):
        Jr, gr = oracle.tube_time_cost(N, R, v, t[b], np.full((S, 2), 0.15), times_cp=t0[b],
                                       grad_mode=2, soft=spec)
        qc = oracle.tube_solve(N, R, v, t[b], np.full((S, 2), 0.15), times_cp=t0[b])["cost"]
        assert st[b] == 0, b
        tolJ = 1e-6 * abs(qc) + 1e-9 * abs(Jr)
        if soft:
            tolJ += 1e-4 * abs(Jr - qc - 500.0 * t[b].sum() ** 2)  # soft term amplifies by 100
        assert abs(J[b] - Jr) <= tolJ, (b, J[b], Jr)
        assert np.max(np.abs(g[b] - gr)) <= 2 * tolJ / (2 * H) + 1e-9 * np.max(np.abs(gr)), b
    # grad=False gives the same J
    out0 = mtg.tube_time_cost(ctx, N, R, pos, fv, _T(dev, t0), _T(dev, t), radii, soft=spec)
    assert out0["grad"] is None
    assert np.array_equal(out0["cost"].cpu().numpy(), J)


def test_tube_time_cost_main_cpp(ctx, dev, oracle):
    """The 4-segment main.cpp geometry (src/main.cpp:26-74) at its own times:
    J = QCQP cost + 500 (sum T)^2."""
    import mav_tube_trajectory_generation_amd as mtg
    v = main_cpp_vertices(oracle)
    t = oracle.estimate_segment_times(v, 2.0, 2.0)
    pos, fv, radii = _geometry(dev, [(v, t)])
    out = mtg.tube_time_cost(ctx, N, R, pos, fv, _T(dev, t[None]), _T(dev, t[None]), radii)
    ref = oracle.tube_solve(N, R, v, t, np.full((4, 2), 0.15))
    J = float(out["cost"][0])
    assert abs(J - (ref["cost"] + 500.0 * t.sum() ** 2)) <= 1e-6 * ref["cost"]


def test_tube_time_cost_repeated_calls(ctx, dev, oracle):
    """Back-to-back calls alternating grad on/off, each with fresh output
    buffers, return the same J every time.  Regression for a stale cost read
    when the call's scratch came from the stream-ordered pool (the C++
    shim's TimeCostWithQCQPInnerSolve failed one run in three)."""
    import mav_tube_trajectory_generation_amd as mtg
    v = main_cpp_vertices(oracle)
    t = oracle.estimate_segment_times(v, 2.0, 2.0)
    pos, fv, radii = _geometry(dev, [(v, t)])
    Jr, _ = oracle.tube_time_cost(N, R, v, t, np.full((4, 2), 0.15))
    for i in range(24):
        out = mtg.tube_time_cost(ctx, N, R, pos, fv, _T(dev, t[None]), _T(dev, t[None]), radii,
                                 grad=bool(i & 1))
        J = float(out["cost"][0])
        assert abs(J - Jr) <= 1e-6 * abs(Jr), (i, J, Jr)


def test_tube_time_optimize_vs_oracle(ctx, dev, oracle):
    """Same steps as the oracle's driver: accepted points, evaluation counts
    and the final J on all but one of 24 problems (a trial landing on a
    near-tie of two J values that agree only to the QCQP tolerance may take
    another path).  Round 5 allowed a third to part: a QCQP breakdown at an
    explored point (1-2 % of random tube solves then, in either
    implementation) ended a path; with the round-6 IPM (tube-axis start,
    regularised retry) there is none, and 24 of 24 agree on
    MI355X.  Every path is also checked: descent from J(T0), bounds, and the
    cost equal to the oracle's at the returned times."""
    import mav_tube_trajectory_generation_amd as mtg
    S, E = 4, 10
    items = _batch(oracle, S, range(400, 424))
    t0 = np.stack([t for _, t in items])
    pos, fv, radii = _geometry(dev, items)
    out = mtg.tube_time_optimize(ctx, N, R, pos, fv, radii, _T(dev, t0), max_evals=E)
    T = out["times"].cpu().numpy()
    J = out["cost"].cpu().numpy()
    ev = out["evals"].cpu().numpy()
    assert np.all(out["status"].cpu().numpy() == 0)
    assert np.all(T >= 0.1) and np.all(T <= 2 * t0 + 1e-12)
    agree = breakdowns = 0
    for b, (v, _) in enumerate(items):
        J0, _ = oracle.tube_time_cost(N, R, v, t0[b], np.full((S, 2), 0.15))
        assert J[b] <= J0 * (1 + 1e-9), b
        assert 1 <= ev[b] <= E
        # the reported cost is the objective at the returned times
        Jc, _ = oracle.tube_time_cost(N, R, v, T[b], np.full((S, 2), 0.15), times_cp=t0[b])
        if np.isfinite(Jc):
            assert abs(J[b] - Jc) <= 1e-6 * abs(Jc), b
        else:
            # the oracle IPM breaks down at this point (IPM
            # robustness: a few random tube problems fail in one of the two)
            breakdowns += 1
        tr, fr, er = oracle.tube_time_optimize(N, R, v, t0[b], np.full((S, 2), 0.15),
                                               max_evals=E)
        if er == ev[b] and np.max(np.abs(T[b] - tr)) <= 1e-6 * np.max(tr):
            agree += 1
    print(f"tube FD descent: {agree} of {len(items)} paths agree, {breakdowns} breakdowns")
    assert agree >= len(items) - 1 and breakdowns == 0, (agree, breakdowns)


def test_tube_time_rejects_bad_arguments(ctx, dev, oracle):
    import mav_tube_trajectory_generation_amd as mtg
    from mav_tube_trajectory_generation_amd._abi import MTGError, lib, make_time_params
    import ctypes
    items = _batch(oracle, 4, [5])
    t = _T(dev, items[0][1][None])
    pos, fv, radii = _geometry(dev, items)
    with pytest.raises(MTGError):
        mtg.tube_time_optimize(ctx, N, R, pos, fv, radii, t, max_evals=0)
    p = make_time_params(grad_mode=1)
    c = torch.empty(1, dtype=torch.float64, device=dev)
    g = torch.empty((1, 4), dtype=torch.float64, device=dev)
    vp = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    rc = lib().mtg_tube_time_cost(ctx.handle, N, R, 4, 1, vp(pos), vp(fv), vp(t), vp(t),
                                  vp(radii), 1e-10, 100, ctypes.byref(p), vp(c), vp(g), None,
                                  vp(ws), ws.numel(), None)
    assert rc == -4  # MTG_ERR_UNSUPPORTED: grad_mode 1 needs d held fixed
    # a workspace below mtg_tube_time_workspace_bytes is refused, as is none
    p2 = make_time_params(grad_mode=2)
    need = mtg.tube_time_workspace_bytes(N, 4, 1, p2, False)
    for wp, nb in ((vp(ws), need - 1), (None, need)):
        rc = lib().mtg_tube_time_cost(ctx.handle, N, R, 4, 1, vp(pos), vp(fv), vp(t), vp(t),
                                      vp(radii), 1e-10, 100, ctypes.byref(p2), vp(c), vp(g),
                                      None, wp, nb, None)
        assert rc == -1
    # grids beyond one launch (2^26 problems) are refused by the size query
    assert lib().mtg_tube_time_workspace_bytes(N, 10, 1 << 22, ctypes.byref(p2), 0) == -1


def test_tube_time_poisoned_workspace(ctx, dev, oracle):
    """Every scratch word the objective reads is written first in the same
    call: with the caller's workspace filled with 0xFF bytes (NaN doubles,
    int32 -1) the results are bit-identical to a zeroed workspace, for the
    cost (grad on and off) and for the optimiser.  This is the check for the
    round-1 stale-J report."""
    import mav_tube_trajectory_generation_amd as mtg
    from mav_tube_trajectory_generation_amd._abi import make_time_params
    S = 4
    items = _batch(oracle, S, range(500, 504))
    t0 = _T(dev, np.stack([t for _, t in items]))
    t = t0 * 1.05
    pos, fv, radii = _geometry(dev, items)
    for grad in (False, True):
        p = make_time_params(grad_mode=2 if grad else 0)
        nb = mtg.tube_time_workspace_bytes(N, S, len(items), p, False)
        outs = []
        for fill in (0x00, 0xFF):
            ws = torch.full((nb,), fill, dtype=torch.uint8, device=dev)
            outs.append(mtg.tube_time_cost(ctx, N, R, pos, fv, t0, t, radii, grad=grad,
                                           workspace=ws))
        for k in ("cost", "status") + (("grad",) if grad else ()):
            assert torch.equal(outs[0][k], outs[1][k]), (grad, k)
        assert torch.isfinite(outs[1]["cost"]).all()
    p = make_time_params(grad_mode=2)
    nb = mtg.tube_time_workspace_bytes(N, S, len(items), p, True)
    outs = []
    for fill in (0x00, 0xFF):
        ws = torch.full((nb,), fill, dtype=torch.uint8, device=dev)
        outs.append(mtg.tube_time_optimize(ctx, N, R, pos, fv, radii, t0, max_evals=6,
                                           workspace=ws))
    for k in ("times", "cost", "evals", "status"):
        assert torch.equal(outs[0][k], outs[1][k]), k


def test_tube_time_optimize_graph_capture(ctx, dev, oracle):
    """The optimiser never allocates or synchronises, so a whole call can be
    captured in a HIP graph; the replay gives the eager result."""
    import mav_tube_trajectory_generation_amd as mtg
    from mav_tube_trajectory_generation_amd._abi import make_time_params
    S = 4
    items = _batch(oracle, S, range(510, 513))
    t0 = _T(dev, np.stack([t for _, t in items]))
    pos, fv, radii = _geometry(dev, items)
    eager = mtg.tube_time_optimize(ctx, N, R, pos, fv, radii, t0, max_evals=5)
    p = make_time_params(grad_mode=2)
    ws = torch.empty(mtg.tube_time_workspace_bytes(N, S, len(items), p, True), dtype=torch.uint8,
                     device=dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        tin = t0.clone()
        with torch.cuda.graph(g, stream=side):
            out = mtg.tube_time_optimize(ctx, N, R, pos, fv, radii, tin, max_evals=5,
                                         workspace=ws)
    g.replay()
    torch.cuda.synchronize()
    for k in ("times", "cost", "evals", "status"):
        assert torch.equal(out[k], eager[k]), k
