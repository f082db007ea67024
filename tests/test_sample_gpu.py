"""GPU trajectory sampling (mtg_sample_trajectories) against the oracle's
statement-by-statement restatement of Trajectory::evaluateRange
(src/trajectory.cpp:74-134).

The sample count and sample times must agree exactly.  Values use Horner's
rule in both; the GPU contracts to FMA and computes k*dt where the reference
accumulates dt, so the tolerance is 1e-9 relative to the channel scale.
"""
import numpy as np
import pytest

from helpers import standard_vertices

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _solve(ctx, dev, oracle, N, D, S, seeds, r=None):
    import mav_tube_trajectory_generation_amd as mtg
    r = N // 2 - 1 if r is None else r
    vs = [standard_vertices(N, S, D, s) for s in seeds]
    times = np.stack([oracle.estimate_segment_times(v, 3.0, 5.0) for v in vs])
    coeffs = np.stack([oracle.linear_solve(N, r, v, t)["coeffs"] for v, t in zip(vs, times)])
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    return T(coeffs), T(times), coeffs, times


@pytest.mark.parametrize("N,D,S", [(10, 3, 10), (10, 1, 3), (6, 2, 5), (12, 3, 4)])
def test_sampling_matches_evaluate_range(ctx, dev, oracle, N, D, S):
    import mav_tube_trajectory_generation_amd as mtg
    seeds = list(range(200, 206))
    cd, td, coeffs, times = _solve(ctx, dev, oracle, N, D, S, seeds)
    K = min(4, N - 1)
    dt = 0.01
    smp, st, cnt = mtg.sample_trajectories(cd, td, dt, max_derivative=K)
    torch.cuda.synchronize()
    smp, st, cnt = smp.cpu().numpy(), st.cpu().numpy(), cnt.cpu().numpy()
    for b in range(len(seeds)):
        total = float(times[b].sum())
        for k in range(K + 1):
            ref, rt, n = oracle.evaluate_range(N, coeffs[b], times[b], 0.0, total, dt, k)
            assert cnt[b] == n, (b, k, cnt[b], n)
            got = smp[b, k * D:(k + 1) * D, :n].T
            scale = max(1.0, np.abs(ref).max())
            assert np.max(np.abs(got - ref)) <= 1e-9 * scale, (b, k)
            assert np.max(np.abs(st[b, :n] - rt)) <= 1e-9 * total


def test_sampling_window_and_start_offset(ctx, dev, oracle):
    """t_start inside a segment (the first sample keeps the segment's
    accumulated time, trajectory.cpp:104-106) and t_end before the end."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S = 10, 3, 6
    cd, td, coeffs, times = _solve(ctx, dev, oracle, N, D, S, [301, 302])
    for b in range(2):
        t0 = float(times[b, :2].sum()) + 0.37
        t1 = float(times[b].sum()) - 1.3
        smp, st, cnt = mtg.sample_trajectories(cd[b:b + 1], td[b:b + 1], 0.05, t_start=t0,
                                               t_end=t1, max_derivative=2)
        torch.cuda.synchronize()
        for k in range(3):
            ref, rt, n = oracle.evaluate_range(N, coeffs[b], times[b], t0, t1, 0.05, k)
            assert int(cnt[0]) == n
            got = smp[0, k * D:(k + 1) * D, :n].cpu().numpy().T
            assert np.max(np.abs(got - ref)) <= 1e-9 * max(1.0, np.abs(ref).max())
            assert np.allclose(st[0, :n].cpu().numpy(), rt, rtol=0, atol=1e-9)


def test_sampling_properties_full_batch(ctx, dev):
    """Config-2-sized batch straight from the solver: positions at the
    segment starts equal the vertices, samples are continuous across
    vertices, and counts are ceil(total / dt)."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S, B = 10, 3, 10, 1024
    mask, fixed, times, pos = mtg.generate_random_problems(N, D, S, B, seed0=105)
    plan = mtg.LinearPlan(ctx, N, D, 4, S, mask)
    td = torch.from_numpy(times).to(dev)
    out = plan.solve(torch.from_numpy(fixed).to(dev), td)
    dt = 0.02
    smp, st, cnt = mtg.sample_trajectories(out["coeffs"], td, dt, max_derivative=1)
    torch.cuda.synchronize()
    cnt = cnt.cpu().numpy()
    total = times.sum(axis=1)
    expect = np.ceil(total / dt).astype(int)
    assert np.all(np.abs(cnt - expect) <= 1)
    smp = smp.cpu().numpy()
    # first sample = start vertex position
    assert np.allclose(smp[:, 0:D, 0], pos[:, 0, :], atol=1e-9)
    # velocity samples bounded and finite
    assert np.isfinite(smp[:, D:2 * D, :cnt.min()]).all()


def test_sampling_rejects_bad_arguments(ctx, dev):
    import mav_tube_trajectory_generation_amd as mtg
    from mav_tube_trajectory_generation_amd._abi import MTGError
    c = torch.zeros((1, 3, 3, 10), dtype=torch.float64, device=dev)
    t = torch.ones((1, 3), dtype=torch.float64, device=dev)
    with pytest.raises(MTGError):
        mtg.sample_trajectories(c, t, 0.0)
    with pytest.raises(MTGError):
        mtg.sample_trajectories(c, t, 0.1, max_derivative=10)


@pytest.mark.parametrize("n_max", [1001, 1000, 64])
def test_sampling_row_lengths(ctx, dev, oracle, n_max):
    """An odd n_max takes the 8-byte store path, an even one the paired
    16-byte path; both give the padded run's values, times and counts (a
    row shorter than the trajectory ends the count at n_max)."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S = 10, 3, 10
    cd, td, _, _ = _solve(ctx, dev, oracle, N, D, S, [211, 212, 213])
    ref_s, ref_t, ref_c = mtg.sample_trajectories(cd, td, 0.01, max_derivative=3)
    smp, st, cnt = mtg.sample_trajectories(cd, td, 0.01, max_derivative=3, n_max=n_max)
    torch.cuda.synchronize()
    ref_c, cnt = ref_c.cpu().numpy(), cnt.cpu().numpy()
    assert np.array_equal(cnt, np.minimum(ref_c, n_max))
    for b in range(3):
        n = int(cnt[b])
        assert torch.equal(smp[b, :, :n], ref_s[b, :, :n])
        assert torch.equal(st[b, :n], ref_t[b, :n])
