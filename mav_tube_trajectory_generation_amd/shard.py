"""Data-parallel sharding of a trajectory batch over GPUs.

Trajectories are independent, so a global batch is split into contiguous
shards, one per rank (one process per GPU), with no exchange during the
solve.  The only collective is the all-gather of per-trajectory costs for
selection (RCCL over xGMI when the process group is "nccl"; gloo on CPU in
the tests), followed by a broadcast of the winning trajectory's
coefficients from its owner.
"""
import torch
import torch.distributed as dist


def shard_range(global_batch, world, rank):
    """Contiguous shard [start, start+count) of rank in a batch of
    global_batch: the first global_batch % world ranks get one extra."""
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def gather_costs(local_costs, global_batch, group=None):
    """All-gather the per-trajectory costs of every shard -> [global_batch].

    Shards may differ by one trajectory; they are padded to the largest
    shard with +inf so a single fixed-size all_gather suffices."""
    world = dist.get_world_size(group)
    biggest = shard_range(global_batch, world, 0)[1]
    buf = torch.full((biggest,), float("inf"), dtype=local_costs.dtype,
                     device=local_costs.device)
    buf[:local_costs.numel()] = local_costs
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = []
    for r in range(world):
        out.append(parts[r][:shard_range(global_batch, world, r)[1]])
    return torch.cat(out)


def select_best(local_costs, global_batch, group=None):
    """Global argmin over all shards (NaN costs never win).  Returns
    (global index, cost, owner rank); identical on every rank."""
    allc = gather_costs(local_costs, global_batch, group)
    allc = torch.where(torch.isnan(allc), torch.full_like(allc, float("inf")), allc)
    idx = int(torch.argmin(allc).item())
    world = dist.get_world_size(group)
    owner = next(r for r in range(world)
                 if shard_range(global_batch, world, r)[0] <= idx <
                 sum(shard_range(global_batch, world, r)))
    return idx, float(allc[idx].item()), owner


def broadcast_best(local_coeffs, global_index, owner, global_batch, group=None):
    """Broadcast the winner's coefficients [S, D, N] from its owner rank."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    shape = tuple(local_coeffs.shape[1:])
    buf = torch.empty(shape, dtype=local_coeffs.dtype, device=local_coeffs.device)
    if rank == owner:
        start = shard_range(global_batch, world, rank)[0]
        buf.copy_(local_coeffs[global_index - start])
    dist.broadcast(buf, src=owner, group=group)
    return buf
