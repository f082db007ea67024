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


class SelectionPipeline:
    """The multi-GPU step with the selection off the solve's critical path.

    Step k solves into output set k % depth on the current stream; a side
    stream then reduces that set's costs to the shard's triple
    (mtg_select_local), all-gathers the triples (RCCL) and takes the global
    argmin (mtg_select_global), while the current stream already runs step
    k + 1's solve.  The selection never feeds a later solve; the only
    ordering is that solve k + depth, which overwrites output set k % depth,
    waits for selection k to have read it.  Every call sequence ends with
    drain() (the side stream joins the current one), so a captured graph or
    an eager batch of steps is closed and `best` is final after it.

    solve_into(out): enqueue one solve writing out["cost"] (and the rest of
    the output set) on the current stream.  use_dist=False (one process, no
    process group): the all-gather and the global argmin of one triple are
    the identity, so the shard's triple is the winner."""

    def __init__(self, solve_into, outs, global_batch, start, rank, device, use_dist=True,
                 group=None):
        self.solve_into = solve_into
        self.outs = list(outs)
        self.global_batch = int(global_batch)
        self.start = int(start)
        self.rank = int(rank)
        self.use_dist = use_dist
        self.group = group
        self.side = torch.cuda.Stream(device)
        self.triples = [torch.empty(3, dtype=torch.float64, device=device) for _ in self.outs]
        self.best = torch.empty(3, dtype=torch.float64, device=device)
        self.k = 0
        self._read = [None] * len(self.outs)  # event: selection done reading set i
        self._pending = False  # side stream forked from the current one since drain()

    def step(self):
        lib, check, ptr, stream = _hip()
        main = torch.cuda.current_stream()
        i = self.k % len(self.outs)
        if self._read[i] is not None:
            main.wait_event(self._read[i])
        o = self.outs[i]
        self.solve_into(o)
        solved = torch.cuda.Event()
        solved.record(main)
        self.side.wait_event(solved)
        with torch.cuda.stream(self.side):
            cost = o["cost"]
            t = self.triples[i]
            check(lib.mtg_select_local(ptr(cost), cost.numel(), self.start, self.rank, ptr(t),
                                       stream(cost.device)), "mtg_select_local")
            if self.use_dist:
                self.best = select_best_device(None, self.global_batch, self.group,
                                               local_triple=t)
            else:
                self.best = t
            done = torch.cuda.Event()
            done.record(self.side)
        self._read[i] = done
        self._pending = True
        self.k += 1
        return self.best

    def drain(self):
        """Join the side stream into the current one (end of a captured
        sequence or of an eager batch of steps)."""
        if self._pending:
            torch.cuda.current_stream().wait_stream(self.side)
        self._pending = False
        self._read = [None] * len(self.outs)
        return self.best


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
