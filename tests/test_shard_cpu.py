"""Multi-process (gloo, world_size 2 and 3) tests of the sharded selection
path: each rank solves its contiguous shard (here with the oracle on CPU,
standing in for the per-GPU kernel), costs are all-gathered, the global
argmin and the winner's coefficients agree with a single-process solve."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _solve_shard(seeds, N=10, S=6, D=3):
    sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
    import pyoracle
    costs, coeffs = [], []
    for sd in seeds:
        v = pyoracle.random_vertices(N // 2 - 1, S, D, -10.0, 10.0, int(sd))
        t = pyoracle.estimate_segment_times(v, 3.0, 5.0)
        sol = pyoracle.linear_solve(N, 4, v, t)
        costs.append(sol["cost"])
        coeffs.append(sol["coeffs"])
    return np.array(costs), np.array(coeffs)


def _worker(rank, world, port, global_batch, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, REPO)
    import torch.distributed as dist
    from mav_tube_trajectory_generation_amd.shard import (broadcast_best, select_best,
                                                          select_best_device, shard_range)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, count = shard_range(global_batch, world, rank)
    costs, coeffs = _solve_shard(range(105 + start, 105 + start + count))
    idx, cost, owner = select_best(torch.from_numpy(costs), global_batch)
    best = broadcast_best(torch.from_numpy(coeffs), idx, owner, global_batch)
    # Device-side path (no host sync): the same triple as a tensor.
    dev_triple = select_best_device(torch.from_numpy(costs), global_batch).tolist()
    # NaN never wins, ties go to the lowest global index, an all-NaN batch
    # selects index 0 (single-process argmin semantics).
    nan_costs = costs.copy()
    nan_costs[:] = np.nan
    all_nan = select_best_device(torch.from_numpy(nan_costs), global_batch).tolist()
    tie = np.full_like(costs, 7.0)
    if rank == world - 1:
        tie[-1] = np.nan
    ties = select_best_device(torch.from_numpy(tie), global_batch).tolist()
    # An empty shard (global batch smaller than the world) never wins.
    tiny = select_best_device(torch.tensor([3.0] if rank == 0 else []), 1).tolist()
    # A cost tensor that is not this rank's shard is refused before any launch.
    try:
        select_best_device(torch.from_numpy(costs[:-1]), global_batch)
        short_refused = False
    except ValueError:
        short_refused = True
    assert short_refused
    result_q.put((rank, idx, cost, owner, best.numpy(), dev_triple, all_nan, ties, tiny))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,global_batch", [(2, 10), (3, 11)])
def test_sharded_selection_matches_single_process(world, global_batch):
    from mav_tube_trajectory_generation_amd.shard import shard_range
    # Shards cover the batch exactly once.
    covered = []
    for r in range(world):
        s, c = shard_range(global_batch, world, r)
        covered += list(range(s, s + c))
    assert covered == list(range(global_batch))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, global_batch, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    costs, coeffs = _solve_shard(range(105, 105 + global_batch))
    want = int(np.argmin(costs))
    for rank, idx, cost, owner, best, dev_triple, all_nan, ties, tiny in results:
        assert idx == want
        assert cost == costs[want]
        assert np.array_equal(best, coeffs[want])
        assert dev_triple == [costs[want], float(want), float(owner)]
        assert all_nan[1:] == [0.0, 0.0]
        assert ties == [7.0, 0.0, 0.0]
        assert tiny == [3.0, 0.0, 0.0]


def _steps_worker(rank, world, port, G, n, result_q):
    """select_steps over gloo: each rank's ring of per-step triples, one
    all-gather per bucket, every step's winner by the select_global rule."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, REPO)
    import torch.distributed as dist
    from mav_tube_trajectory_generation_amd.shard import select_steps
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(7)  # the same on every rank: all rings known
    rings = rng.uniform(1.0, 2.0, (world, G, 3))
    rings[:, :, 1] = np.arange(world)[:, None] * 100 + np.arange(G)[None, :]
    rings[:, :, 2] = np.arange(world)[:, None]
    rings[:, 1, 0] = 1.5              # step 1: a tie across every rank
    rings[world - 1, 2, 0] = np.nan   # NaN never wins
    rings[0, 3, 1] = -1.0             # an empty shard never wins
    out = select_steps(torch.from_numpy(rings[rank].copy()), n)
    result_q.put((rank, out[:n].numpy(), rings))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_select_steps_bucket_gloo(world):
    G, n = 6, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_steps_worker, args=(r, world, port, G, n, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rings = res[0][2]
    for g in range(n):
        keys = [np.inf if (rings[w, g, 1] < 0 or np.isnan(rings[w, g, 0])) else rings[w, g, 0]
                for w in range(world)]
        w = int(np.argmin(keys))
        for rank, got, _ in res:
            assert np.array_equal(got[g], rings[w, g]), (rank, g)
