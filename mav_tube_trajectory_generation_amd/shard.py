"""Data-parallel sharding of a trajectory batch over GPUs.

Trajectories are independent, so a global batch is split into contiguous
shards, one per rank (one process per GPU), with no exchange during the
solve.  The only collective is the all-gather for selection (RCCL over xGMI
when the process group is "nccl"; gloo on CPU in the tests), followed by a
broadcast of the winning trajectory's coefficients from its owner.

Two selection paths:
  select_best_device  each rank reduces its shard to one (cost, global index,
                      rank) triple on the device (fused into the solve launch
                      by LinearPlan.solve_select, or one extra launch), the
                      triples are all-gathered
                      (24 B per rank) and reduced again on the device: on GPU
                      tensors one HIP launch each (mtg_select_local /
                      mtg_select_global) around the RCCL all-gather; on CPU
                      tensors (gloo) the same rule with torch ops.  No host
                      synchronisation, so it can sit inside a timed loop or a
                      captured graph.
  select_best         the same, returned as Python numbers (one sync).
  gather_costs        every per-trajectory cost on every rank (the SURVEY's
                      512 KiB all-gather at config 4), for callers that need
                      the whole cost vector.
"""
import torch
import torch.distributed as dist


def _hip():
    """The HIP selection kernels (device tensors only; no CPU fallback)."""
    from ._abi import check, lib
    from .batch import _ptr, _stream
    return lib(), check, _ptr, _stream


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


def local_best(local_costs, global_batch, group=None):
    """This rank's (cost, global index, rank) triple as a float64 device
    tensor [3]: the shard's smallest cost (NaN never wins; the first index on
    ties).  An empty shard reports (+inf, -1, rank)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    start, count = shard_range(global_batch, world, rank)
    if local_costs.numel() != count:
        raise ValueError(f"rank {rank}: {local_costs.numel()} local costs, but the shard of "
                         f"{global_batch} over {world} ranks holds {count}")
    if local_costs.is_cuda:  # one HIP launch (mtg_select_local)
        lib, check, ptr, stream = _hip()
        c = local_costs
        if c.dtype != torch.float64 or not c.is_contiguous():
            c = c.to(torch.float64).contiguous()
        out = torch.empty(3, dtype=torch.float64, device=c.device)
        check(lib.mtg_select_local(ptr(c), count, start, rank, ptr(out), stream(c.device)),
              "mtg_select_local")
        return out
    # CPU tensors (gloo): the same rule with torch ops.
    out = torch.full((3,), float(rank), dtype=torch.float64, device=local_costs.device)
    if count == 0:
        out[0] = float("inf")
        out[1] = -1.0
        return out
    c = local_costs[:count].to(torch.float64)
    c = torch.where(torch.isnan(c), torch.full_like(c, float("inf")), c)
    i = torch.argmin(c)
    out[0] = c[i]
    out[1] = i.to(torch.float64) + float(start)
    return out


def select_best_device(local_costs, global_batch, group=None, local_triple=None):
    """Global argmin over all shards without a host sync.  Returns a float64
    device tensor [3] = (cost, global index, owner rank), identical on every
    rank.  Ties go to the lowest global index (shards are contiguous and in
    rank order, so the first rank holding the minimum); if every cost is NaN
    or +inf the winner is global index 0, as a single-process argmin.
    local_triple: this rank's triple already reduced (the fused
    LinearPlan.solve_select); local_costs is then not read."""
    world = dist.get_world_size(group)
    mine = local_triple if local_triple is not None else \
        local_best(local_costs, global_batch, group)
    flat = torch.empty(world * 3, dtype=torch.float64, device=mine.device)
    dist.all_gather_into_tensor(flat, mine, group=group)
    if flat.is_cuda:  # one HIP launch (mtg_select_global)
        lib, check, ptr, stream = _hip()
        out = torch.empty(3, dtype=torch.float64, device=flat.device)
        check(lib.mtg_select_global(ptr(flat), world, ptr(out), stream(flat.device)),
              "mtg_select_global")
        return out
    allv = flat.view(world, 3)
    # Empty shards (index -1) only win when every shard is empty.
    key = torch.where(allv[:, 1] < 0, torch.full_like(allv[:, 0], float("nan")), allv[:, 0])
    key = torch.where(torch.isnan(key), torch.full_like(key, float("inf")), key)
    w = torch.argmin(key)
    return allv[w]


def select_steps(ring, n, group=None, out=None, use_dist=True):
    """Per-step global winners of a bucket of n steps: ring [G, 3] holds this
    rank's triple of each step (rows >= n unused).  The ranks all-gather
    their whole rings (world x G x 3 doubles, one collective per bucket) and
    step g's winner is the select_global rule over the ranks' row g.
    Returns out [G, 3] (rows < n set).  use_dist=False (one process): the
    rank's own triples are the winners."""
    G = ring.shape[0]
    if out is None:
        out = torch.full_like(ring, float("nan"))
    if n == 0:
        return out
    if not use_dist:
        out[:n].copy_(ring[:n])
        return out
    world = dist.get_world_size(group)
    flat = torch.empty(world * G * 3, dtype=torch.float64, device=ring.device)
    dist.all_gather_into_tensor(flat, ring.reshape(-1), group=group)
    if flat.is_cuda:  # one HIP launch (mtg_select_global_steps)
        lib, check, ptr, stream = _hip()
        check(lib.mtg_select_global_steps(ptr(flat), world, G, n, ptr(out),
                                          stream(flat.device)), "mtg_select_global_steps")
        return out
    allv = flat.view(world, G, 3)[:, :n]
    key = torch.where(allv[..., 1] < 0, torch.full_like(allv[..., 0], float("nan")),
                      allv[..., 0])
    key = torch.where(torch.isnan(key), torch.full_like(key, float("inf")), key)
    w = torch.argmin(key, dim=0)  # the first rank holding the minimum
    out[:n] = allv[w, torch.arange(n)]
    return out


class SelectionPipeline:
    """The multi-GPU step with the selection off the solve's critical path.

    Step k solves into output set k % 2 and, in the SAME launch, reduces
    step k - 1's costs (the other set) to the shard's triple
    (mtg_linear_solve_select_prev: one extra workgroup of the wave /
    lane-pair kernels, running beside the solves).  The triples of a bucket
    of up to `bucket` steps collect in a device ring; at the end of the
    bucket (or drain()) the last step's costs are reduced, the ranks
    all-gather their rings in ONE collective (RCCL over xGMI) and every
    step's global winner is taken at once (mtg_select_global_steps).  So a
    step costs the solve launch alone, and the collective's fixed latency
    is paid once per bucket, not per step.  Everything is stream-ordered on
    the current stream, so a captured graph holds it without cross-stream
    edges (a side-stream fork and join per step measured 6.4 us of graph
    overhead per step).  The selection never feeds a later solve.

    best [bucket, 3]: the winners (cost, global index, owner rank) of the
    last closed bucket, rows < n_done valid.  use_dist=False (one process,
    no process group): the shard's triples are the winners."""

    def __init__(self, plan, fixed_vals, times, outs, global_batch, start, rank, device,
                 use_dist=True, bucket=32, group=None):
        self.plan = plan
        self.fixed_vals = fixed_vals
        self.times = times
        self.outs = list(outs)
        if len(self.outs) != 2:
            raise ValueError("two output sets alternate")
        self.global_batch = int(global_batch)
        self.start = int(start)
        self.rank = int(rank)
        self.use_dist = use_dist
        self.group = group
        self.bucket = int(bucket)
        self.ring = torch.full((self.bucket, 3), float("nan"), dtype=torch.float64,
                               device=device)
        self.best = torch.full((self.bucket, 3), float("nan"), dtype=torch.float64,
                               device=device)
        self.k = 0
        self.n = 0          # steps in the open bucket
        self.n_done = 0     # steps of the last closed bucket
        self.last = None    # output set of the last solve (costs not yet reduced)

    def step(self):
        if self.n == self.bucket:
            self._flush()
        i = self.k % 2
        o = self.outs[i]
        if self.last is None:
            self.plan.solve_select_prev(self.fixed_vals, self.times, o)
        else:
            self.plan.solve_select_prev(self.fixed_vals, self.times, o,
                                        prev_cost=self.outs[self.last]["cost"],
                                        prev_start=self.start, rank=self.rank,
                                        prev_triple=self.ring[self.n - 1])
        self.last = i
        self.n += 1
        self.k += 1
        return self.best

    def _flush(self):
        if self.n == 0:
            return
        lib, check, ptr, stream = _hip()
        c = self.outs[self.last]["cost"]
        t = self.ring[self.n - 1]
        check(lib.mtg_select_local(ptr(c), c.numel(), self.start, self.rank, ptr(t),
                                   stream(c.device)), "mtg_select_local")
        select_steps(self.ring, self.n, self.group, out=self.best, use_dist=self.use_dist)
        self.last = None
        self.n_done = self.n
        self.n = 0

    def drain(self):
        """Close the open bucket (end of a captured sequence or of an eager
        batch of steps); returns the winners of its steps [n_done, 3]."""
        self._flush()
        return self.best[:self.n_done]


def select_best(local_costs, global_batch, group=None):
    """Global argmin over all shards (NaN costs never win).  Returns
    (global index, cost, owner rank) as Python numbers; identical on every
    rank (one host synchronisation)."""
    cost, idx, owner = select_best_device(local_costs, global_batch, group).tolist()
    return int(idx), float(cost), int(owner)


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
