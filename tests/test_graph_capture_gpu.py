"""Every bench workload's step captured in a HIP graph, replayed once and
compared bit for bit with the same step run eagerly (the timed region of
bench.py is a graph replay, so a step that does not capture, or captures
something else, must fail here rather than in the bench).

Also: a stale error left in the HIP runtime's per-thread last-error slot by
an unrelated failed call must not be reported as the next entry point's
MTG_ERR_HIP (the cause of round 4's failed captures), and the
selection pipeline (shard.SelectionPipeline: each launch reduces the
previous step's costs, a bucket of steps closes with one selection) must
give every step's winner inside a graph.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N, D, R = 10, 3, 4


def _capture(fn, reps=3):
    """Run fn eagerly once (warm-up), capture reps calls, replay once."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            res = fn()
    g.replay()
    torch.cuda.synchronize()
    return res


def _problems(S, B, seed0=105):
    import mav_tube_trajectory_generation_amd as mtg
    mask, fixed, times, pos = mtg.generate_random_problems(N, D, S, B, seed0=seed0)
    return mask, fixed, times, pos


@pytest.mark.parametrize("B,kernel", [(1024, "auto"), (8192, "auto"), (64, "generic")])
def test_linear_step_captures(ctx, dev, B, kernel):
    import mav_tube_trajectory_generation_amd as mtg
    S = 10
    mask, fixed, times, _ = _problems(S, B)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    eager = {k: v.clone() for k, v in plan.solve(fd, td).items()}
    torch.cuda.synchronize()
    out = plan.solve(fd, td)
    for v in out.values():
        v.fill_(0)
    got = _capture(lambda: plan.solve(fd, td, out=out))
    for k in eager:
        assert torch.equal(got[k], eager[k]), k


def test_time_step_captures(ctx, dev):
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 10, 256
    mask, fixed, times, _ = _problems(S, B)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    eager = plan.time_optimize(fd, td, max_evals=20)
    eager = {k: v.clone() for k, v in eager.items()}
    torch.cuda.synchronize()
    got = _capture(lambda: plan.time_optimize(fd, td, max_evals=20), reps=1)
    for k in eager:
        assert torch.equal(got[k], eager[k]), k


def test_tube_step_captures(ctx, dev):
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 10, 64
    _, _, times, pos = _problems(S, B)
    M = N // 2
    pos = np.asarray(pos)[:, :, :3] if np.asarray(pos).ndim == 3 else np.asarray(pos)
    # the bench's tube inputs: vertex positions, start / end fixed at rest
    fv = np.zeros((B, 3, N))
    fv[:, :, 0] = pos[:, 0, :]
    fv[:, :, M] = pos[:, S, :]
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    args = (T(pos), T(fv), T(times), T(times), T(np.full((B, S, 2), 0.15)))
    eager = {k: v.clone() for k, v in mtg.tube_solve(ctx, N, R, *args).items()}
    torch.cuda.synchronize()
    got = _capture(lambda: mtg.tube_solve(ctx, N, R, *args), reps=1)
    for k in eager:
        assert torch.equal(got[k], eager[k]), k


@pytest.mark.parametrize("B,kernel", [(1024, "auto"), (8192, "auto"), (300, "generic"),
                                      (2000, "lane")])
def test_selection_pipeline_in_graph(ctx, dev, B, kernel):
    """shard.SelectionPipeline: each launch reduces the previous step's costs
    in an extra workgroup (or a launch of its own for the other kernels),
    buckets of steps close with one selection; every step's winner is the
    argmin of its costs (select_local's rule), eagerly and replayed from a
    graph, across bucket boundaries."""
    import mav_tube_trajectory_generation_amd as mtg
    from mav_tube_trajectory_generation_amd.shard import SelectionPipeline
    S, start = 10, 4096
    mask, fixed, times, _ = _problems(S, B)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask).set_kernel(kernel)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    base = plan.solve(fd, td)["cost"].cpu().numpy()
    j = int(np.argmin(base))
    want = torch.tensor([base[j], start + j, 1.0], dtype=torch.float64)
    outs = [plan.solve(fd, td), plan.solve(fd, td)]
    for o in outs:
        o["cost"].fill_(float("nan"))
    pipe = SelectionPipeline(plan, fd, td, outs, 2 * B, start, 1, dev, use_dist=False, bucket=3)
    for _ in range(5):  # a bucket of 3, then 2 closed by drain()
        pipe.step()
    eager = pipe.drain().clone()
    torch.cuda.synchronize()
    assert eager.shape == (2, 3)
    for r in eager.cpu():
        assert torch.equal(r, want)

    def steps():
        for _ in range(3):
            pipe.step()
        return pipe.drain()
    got = _capture(steps, reps=1)
    assert got.shape == (3, 3)
    for r in got.cpu():
        assert torch.equal(r, want)


def _hip_runtime():
    """The HIP runtime this process already loaded (the one torch and
    libmtg_hip.so use), found by path in /proc/self/maps."""
    with open("/proc/self/maps") as f:
        for line in f:
            path = line.split()[-1]
            if "libamdhip64.so" in path:
                return ctypes.CDLL(path)
    pytest.skip("HIP runtime not mapped")


def test_stale_error_not_reported(ctx, dev):
    import mav_tube_trajectory_generation_amd as mtg
    S, B = 10, 64
    mask, fixed, times, _ = _problems(S, B)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    hip = _hip_runtime()
    # a failed call of "another library": an invalid device ordinal
    assert hip.hipSetDevice(ctypes.c_int(1 << 20)) != 0
    out = plan.solve(fd, td)  # raises MTGError if the stale error leaked
    torch.cuda.synchronize()
    assert (out["status"].cpu().numpy() == 0).all()


def test_bench_timing_events(ctx, dev):
    """bench.py's timing events: device scope (hipEventDisableSystemFence,
    recorded through the HIP runtime torch mapped) and torch's system-scope
    events both time a replayed graph of solves."""
    import importlib.util
    import os
    import mav_tube_trajectory_generation_amd as mtg
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
    spec = importlib.util.spec_from_file_location("bench_mod", path)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    S, B = 10, 1024
    mask, fixed, times, _ = _problems(S, B)
    plan = mtg.LinearPlan(ctx, N, D, R, S, mask)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    out = plan.solve(fd, td)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            plan.solve(fd, td, out=out)
    g.replay()
    torch.cuda.synchronize()
    for scope in ("device", "system"):
        ev = bench.TimingEvents(scope)
        ev.record(0, stream)
        g.replay()
        ev.record(1, stream)
        torch.cuda.synchronize()
        ms = ev.elapsed_ms()
        assert 0.0 < ms < 50.0, (scope, ms)
