"""The lane linear kernels (mtg_linear_lane.hip, LANE: one (trajectory,
dimension) per lane; mtg_linear_lane2.hip, LANE_PAIR: two lanes per
(trajectory, dimension), twisted elimination) against the wavefront standard-pattern kernel and the
oracle, and AUTO's choice by batch size."""
import numpy as np
import pytest

from helpers import REL_TOL, rel_err, rel_err_coeffs, standard_vertices

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N, D, R = 10, 3, 4


def _solve(ctx, dev, mask, fixed, times, kernel):
    import mav_tube_trajectory_generation_amd as mtg
    S = times.shape[1]
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    out = plan.solve(torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev), free=True)
    torch.cuda.synchronize()
    return plan, {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("kernel", ["lane", "lane_pair"])
@pytest.mark.parametrize("S", list(range(2, 13)))
def test_lane_kernels_match_wavefront_kernel(ctx, dev, oracle, kernel, S):
    """Same inputs as the wavefront kernel, a batch that is not a multiple of
    the trajectories per wavefront (21): coefficients, d_p and cost to
    1e-9 (different elimination order: block Thomas vs twisted), oracle spot
    checks at the 1e-6 parity bar."""
    import mav_tube_trajectory_generation_amd as mtg
    B = 203
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=2000 + S)
    plan, out = _solve(ctx, dev, mask, fixed, times, kernel)
    assert plan.kernel == kernel
    _, ref = _solve(ctx, dev, mask, fixed, times, "standard")
    assert (out["status"] == 0).all()
    for b in range(B):
        assert rel_err_coeffs(out["coeffs"][b], ref["coeffs"][b]) <= 1e-9, b
        assert rel_err_coeffs(out["free"][b], ref["free"][b]) <= 1e-9, b
        assert rel_err(out["cost"][b], ref["cost"][b]) <= 1e-8, b
    for b in (0, 101, B - 1):
        o = oracle.linear_solve(N, R, standard_vertices(N, S, D, 2000 + S + b), times[b])
        assert rel_err_coeffs(out["coeffs"][b], o["coeffs"]) <= REL_TOL, b
        assert rel_err(out["cost"][b], o["cost"]) <= REL_TOL, b


@pytest.mark.parametrize("S", [2, 3, 7, 10, 12])
def test_lane_pair_staged_outputs(ctx, dev, S):
    """From 4096 trajectories the lane-pair kernel stages its coefficients in
    LDS and copies each workgroup's range out coalesced (kLane2StageMinBatch):
    a batch whose last workgroup is ragged (4096 + 5 = 195 x 21 + 2), one bad
    time, against the wavefront kernel on every trajectory."""
    import mav_tube_trajectory_generation_amd as mtg
    B = 4096 + 5
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=7000 + S)
    times[4095, 0] = 0.0
    plan, out = _solve(ctx, dev, mask, fixed, times, "lane_pair")
    assert plan.kernel == "lane_pair"
    _, ref = _solve(ctx, dev, mask, fixed, times, "standard")
    np.testing.assert_array_equal(out["status"], ref["status"])
    assert out["status"][4095] == 1 and np.isnan(out["coeffs"][4095]).all()
    ok = out["status"] == 0
    assert ok.sum() == B - 1
    c, r = out["coeffs"][ok], ref["coeffs"][ok]
    # rel_err_coeffs over the whole batch: per (trajectory, segment, dim)
    err = np.linalg.norm(c - r, axis=-1) / np.maximum(np.linalg.norm(r, axis=-1), 1e-12)
    assert err.max() <= 1e-9, float(err.max())
    np.testing.assert_allclose(out["cost"][ok], ref["cost"][ok], rtol=1e-8)


@pytest.mark.parametrize("kernel", ["lane", "lane_pair", "standard", "generic"])
def test_lane_kernels_bad_time(ctx, dev, kernel):
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 5, 70
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=31)
    times[3, 1] = 0.0
    times[64, 4] = -2.0
    times[65, 0] = np.inf
    _, out = _solve(ctx, dev, mask, fixed, times, kernel)
    bad = {3, 64, 65}
    for b in range(B):
        if b in bad:
            assert out["status"][b] == 1 and np.isnan(out["cost"][b])
            assert np.isnan(out["coeffs"][b]).all()
            # every kernel reports a bad time's free values as NaN (the same
            # answer whatever kernel AUTO picks for the batch size)
            assert np.isnan(out["free"][b]).all()
        else:
            assert out["status"][b] == 0 and np.isfinite(out["cost"][b])
            assert np.isfinite(out["free"][b]).all()


def test_auto_selection_by_batch(ctx):
    import mav_tube_trajectory_generation_amd as mtg
    S = 10
    mask, _, _, _ = mtg.generate_random_problems(N, D, S, 1, seed0=1)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    assert plan.kernel == "standard"
    assert plan.kernel_for_batch(1024) == "standard"
    assert plan.kernel_for_batch(2048) == "standard"
    assert plan.kernel_for_batch(2049) == "lane_pair"
    assert plan.kernel_for_batch(4096) == "lane_pair"
    assert plan.kernel_for_batch(65536) == "lane_pair"
    assert plan.set_kernel("standard").kernel_for_batch(65536) == "standard"
    # outside the lane kernels' instantiations: the wavefront kernel
    p2 = mtg.LinearPlan(ctx, N, 2, R, S, mask)
    assert p2.kernel_for_batch(65536) == "standard"
    with pytest.raises(mtg.MTGError):
        p2.set_kernel("lane")
    with pytest.raises(mtg.MTGError):
        p2.set_kernel("lane_pair")
    m20, _, _, _ = mtg.generate_random_problems(N, D, 20, 1, seed0=1)
    p3 = mtg.LinearPlan(ctx, N, D, R, 20, m20)
    assert p3.kernel_for_batch(65536) == "standard"
