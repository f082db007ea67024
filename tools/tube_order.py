"""Config 3 (4096 x 10-segment tube QCQP) launched in different problem
orders: does the order the workgroups are dispatched in change the launch
time, and by how much?

* as generated (the bench's order);
* longest first (by the measured IPM iteration counts: LPT order);
* shortest first;
* "xcd": the longest eighth of the problems on indices = 0 mod 8 (if the
  dispatcher deals workgroups to the eight XCDs round-robin, one XCD then
  gets all the long problems).

Writes gpurun_out/tube_order.json (iteration counts and per-order times) and
prints a summary.  Run on the GPU box: python tools/tube_order.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mav_tube_trajectory_generation_amd as mtg  # noqa: E402


def main():
    N, D, r, S, B = 10, 3, 4, 10, 4096
    dev = torch.device("cuda:0")
    mask, fixed, times, pos = mtg.generate_random_problems(N, D, S, B, seed0=105)
    ctx = mtg.Context(0)
    M = N // 2
    tf = np.zeros((B, 3, N))
    tf[:, :, 0] = pos[:, 0, :]
    tf[:, :, M] = pos[:, S, :]

    def inputs(perm):
        p = torch.from_numpy(pos[perm]).to(dev)
        t = torch.from_numpy(times[perm]).to(dev)
        f = torch.from_numpy(tf[perm]).to(dev)
        rad = torch.full((B, S, 2), 0.15, dtype=torch.float64, device=dev)
        return p, f, t, rad

    def timed(perm, reps=5):
        p, f, t, rad = inputs(perm)
        out = mtg.tube_solve(ctx, N, r, p, f, t, t, rad)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ms = []
        for _ in range(reps):
            e0.record()
            mtg.tube_solve(ctx, N, r, p, f, t, t, rad)
            e1.record()
            torch.cuda.synchronize(dev)
            ms.append(e0.elapsed_time(e1))
        return float(np.median(ms)), out

    ident = np.arange(B)
    t_id, out = timed(ident)
    iters = out["iters"].cpu().numpy().astype(int)
    lpt = np.argsort(-iters, kind="stable")
    spt = np.argsort(iters, kind="stable")
    # The longest B/8 problems at indices 0, 8, 16, ...; the rest elsewhere.
    xcd = np.empty(B, dtype=int)
    slots0 = np.arange(0, B, 8)
    others = np.setdiff1d(ident, slots0)
    xcd[slots0] = lpt[: B // 8]
    xcd[others] = lpt[B // 8:]
    res = {"iters_mean": float(iters.mean()), "iters_max": int(iters.max()),
           "iters_min": int(iters.min()), "iters": iters.tolist(), "ms": {"generated": t_id}}
    for name, perm in (("longest_first", lpt), ("shortest_first", spt), ("xcd_skew", xcd)):
        res["ms"][name] = timed(perm)[0]
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/tube_order.json", "w") as f:
        json.dump(res, f)
    print("iters mean %.2f min %d max %d" % (iters.mean(), iters.min(), iters.max()))
    for k, v in res["ms"].items():
        print("%-15s %.3f ms" % (k, v))


if __name__ == "__main__":
    main()
