"""GPU selection kernels of the multi-GPU path (mtg_select_local /
mtg_select_global) against the selection rule written in
numpy, and the whole select_best_device step on a one-rank RCCL group."""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _ref_local(c, start, rank):
    if len(c) == 0:
        return (math.inf, -1.0, float(rank))
    k = np.where(np.isnan(c), np.inf, c)
    i = int(np.argmin(k))  # first minimum
    return (float(k[i]), float(i + start), float(rank))


def _ref_global(t):
    keys = np.where((t[:, 1] < 0) | np.isnan(t[:, 0]), np.inf, t[:, 0])
    return tuple(t[int(np.argmin(keys))])


def _call_local(dev, c, start, rank):
    from mav_tube_trajectory_generation_amd._abi import check, lib
    from mav_tube_trajectory_generation_amd.batch import _ptr, _stream
    ct = torch.from_numpy(np.ascontiguousarray(c, dtype=np.float64)).to(dev)
    out = torch.empty(3, dtype=torch.float64, device=dev)
    check(lib().mtg_select_local(_ptr(ct) if len(c) else None, len(c), start, rank, _ptr(out),
                                 _stream(dev)), "mtg_select_local")
    return tuple(out.cpu().numpy())


def _same(a, b):
    return all((x == y) or (math.isinf(x) and math.isinf(y)) for x, y in zip(a, b))


@pytest.mark.parametrize("case", ["random", "nan", "ties", "all_nan", "all_inf", "empty",
                                  "single", "large"])
def test_select_local_matches_rule(ctx, dev, case):
    rng = np.random.default_rng(abs(hash(case)) % 1000)
    n = {"empty": 0, "single": 1, "large": 65536}.get(case, 3000)
    c = rng.uniform(1.0, 2.0, n)
    if case == "nan":
        c[rng.integers(0, n, 50)] = np.nan
        c[17] = np.nan
    if case == "ties":
        c[:] = np.round(c, 1)
        c[[5, 900, 2999]] = 0.5
    if case == "all_nan":
        c[:] = np.nan
    if case == "all_inf":
        c[:] = np.inf
    if case == "large":
        c[40000] = 0.1
        c[60000] = 0.1
    got = _call_local(dev, c, 12345, 3)
    assert _same(got, _ref_local(c, 12345, 3)), (got, _ref_local(c, 12345, 3))


def test_select_global_matches_rule(ctx, dev):
    from mav_tube_trajectory_generation_amd._abi import check, lib
    from mav_tube_trajectory_generation_amd.batch import _ptr, _stream
    rng = np.random.default_rng(5)
    cases = []
    for world in (1, 2, 3, 8):
        t = np.stack([rng.uniform(1, 2, world), np.arange(world) * 100.0, np.arange(world) * 1.0], 1)
        cases.append(t)
        t2 = t.copy(); t2[:, 0] = 1.5; cases.append(t2)                  # ties: first rank
        t3 = t.copy(); t3[0, 1] = -1; t3[0, 0] = np.inf; cases.append(t3)  # empty shard
        t4 = t.copy(); t4[:, 0] = np.nan; cases.append(t4)                # nothing finite
        t5 = t.copy(); t5[-1, 0] = 0.0; t5[0, 0] = np.nan; cases.append(t5)
    for t in cases:
        tt = torch.from_numpy(np.ascontiguousarray(t.reshape(-1))).to(dev)
        out = torch.empty(3, dtype=torch.float64, device=dev)
        check(lib().mtg_select_global(_ptr(tt), t.shape[0], _ptr(out), _stream(dev)),
              "mtg_select_global")
        got = tuple(out.cpu().numpy())
        ref = _ref_global(t)
        assert all((x == y) or (np.isnan(x) and np.isnan(y)) or (math.isinf(x) and math.isinf(y))
                   for x, y in zip(got, ref)), (t, got, ref)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_select_global_steps_matches_rule(ctx, dev, world):
    """mtg_select_global_steps, the per-step winners of a bucket at world > 1
    (shard.select_steps after the RCCL all-gather), on synthetic [world, G,
    3] rings: NaN costs, empty shards (index -1, cost inf), ties across ranks
    and buckets with n < G.  Each row g < n must be the select_global rule
    over the ranks' row g; rows >= n are left untouched."""
    from mav_tube_trajectory_generation_amd._abi import check, lib
    from mav_tube_trajectory_generation_amd.batch import _ptr, _stream
    G = 16
    rng = np.random.default_rng(world)
    ring = np.empty((world, G, 3))
    ring[..., 0] = rng.uniform(1.0, 2.0, (world, G))
    ring[..., 1] = rng.integers(0, 65536, (world, G)).astype(np.float64)
    ring[..., 2] = np.arange(world)[:, None]
    ring[:, 1, 0] = np.nan                      # no finite cost anywhere
    ring[0, 2, 0] = np.nan                      # NaN on one rank only
    ring[:, 3, 0] = 1.25                        # a tie on every rank: the first rank
    ring[-1, 4, :2] = (np.inf, -1.0)            # an empty shard
    ring[:, 5, :2] = (np.inf, -1.0)             # every shard empty
    ring[1, 6, 0] = 0.0                         # the winner on rank 1
    ring[-1, 7, :2] = (0.5, -1.0)               # a finite cost with index -1 never wins
    flat = torch.from_numpy(np.ascontiguousarray(ring.reshape(-1))).to(dev)
    for n in (G, 9, 1):
        out = torch.full((G, 3), 7.0, dtype=torch.float64, device=dev)
        check(lib().mtg_select_global_steps(_ptr(flat), world, G, n, _ptr(out), _stream(dev)),
              "mtg_select_global_steps")
        got = out.cpu().numpy()
        for g in range(n):
            ref = _ref_global(ring[:, g])
            assert all((x == y) or (np.isnan(x) and np.isnan(y)) or
                       (math.isinf(x) and math.isinf(y)) for x, y in zip(got[g], ref)), \
                (world, n, g, got[g], ref)
        assert (got[n:] == 7.0).all(), (world, n)


def test_select_best_device_one_rank_rccl(ctx, dev):
    """The whole device selection step (local kernel, RCCL all-gather, global
    kernel) on a one-rank process group, inside a captured HIP graph."""
    import torch.distributed as dist

    from mav_tube_trajectory_generation_amd.shard import select_best, select_best_device
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29650 + os.getpid() % 200))
    created = not dist.is_initialized()
    if created:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        c = torch.rand(4096, dtype=torch.float64, device=dev) + 1.0
        c[1234] = 0.25
        c[17] = float("nan")
        assert select_best(c, 4096) == (1234, 0.25, 0)
        res = torch.empty(3, dtype=torch.float64, device=dev)
        select_best_device(c, 4096)  # warm-up outside the capture
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            res.copy_(select_best_device(c, 4096))
        c[1234] = 3.0
        c[99] = 0.125
        g.replay()
        torch.cuda.synchronize(dev)
        assert tuple(res.cpu().numpy()) == (0.125, 99.0, 0.0)
    finally:
        if created:
            dist.destroy_process_group()


@pytest.mark.parametrize("kernel", ["standard", "lane", "lane_pair", "generic"])
def test_solve_select_fused(ctx, dev, kernel):
    """mtg_linear_solve_select: the shard's triple (lane kernels: per-
    workgroup partials from the solve's epilogue, then one reduction launch)
    equals the selection rule on the costs the same solve wrote, with NaN
    costs (bad times), ties (duplicated trajectories) and repeated launches on
    one uninitialised workspace; inside a captured graph as well."""
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S, B = 10, 3, 10, 3000
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=400)
    plan = mtg.LinearPlan(ctx, N, D, 4, S, mask).set_kernel(kernel)
    ref = plan.solve(torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev))
    c0 = ref["cost"].cpu().numpy()
    best = int(np.argmin(c0))
    # Ties: copies of the best trajectory after it and before it.
    for j in (best + 7) % B, (best + 1500) % B:
        fixed[j] = fixed[best]
        times[j] = times[best]
    times[5, 2] = -1.0  # a bad time: NaN cost, never selected
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    ws = plan.select_workspace(B, dev)
    ws.fill_(0xFF)  # no initialisation needed
    for rep in range(3):
        out = plan.solve_select(fd, td, 1000, 2, ws)
        torch.cuda.synchronize(dev)
        c = out["cost"].cpu().numpy()
        assert np.isnan(c[5])
        got = tuple(out["triple"].cpu().numpy())
        assert _same(got, _ref_local(c, 1000, 2)), (rep, got, _ref_local(c, 1000, 2))
        assert got[1] - 1000 == min(best, (best + 7) % B, (best + 1500) % B)
    # Captured graph: new costs after a change of the inputs.
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = plan.solve_select(fd, td, 0, 0, ws, out=out)
    td[best, :] *= 3.0
    td[(best + 7) % B, :] *= 3.0
    td[(best + 1500) % B, :] *= 3.0
    g.replay()
    torch.cuda.synchronize(dev)
    c = out["cost"].cpu().numpy()
    assert _same(tuple(out["triple"].cpu().numpy()), _ref_local(c, 0, 0))


def test_solve_select_all_bad_and_empty(ctx, dev):
    import mav_tube_trajectory_generation_amd as mtg
    N, D, S, B = 10, 3, 4, 70
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=9)
    plan = mtg.LinearPlan(ctx, N, D, 4, S, mask)
    times[:] = -1.0
    ws = plan.select_workspace(B, dev)
    out = plan.solve_select(torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev),
                            50, 1, ws)
    # every cost NaN: the shard's first index, cost +inf
    assert tuple(out["triple"].cpu().numpy()) == (math.inf, 50.0, 1.0)
