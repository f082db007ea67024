"""Kernel-time sweep over batch sizes (HIP events on the launch stream).

python tools/sweep.py [--workload linear|time|tube] [--batches 1024,8192,...]
Prints one JSON line per batch size: kernel ms, trajectories/s, algorithmic
GB/s of the dominant kernel.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="linear")
    p.add_argument("--batches", default="1024,4096,16384,65536,262144")
    p.add_argument("--segments", type=int, default=10)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--evals", type=int, default=50)
    a = p.parse_args()
    import numpy as np
    import torch
    import mav_tube_trajectory_generation_amd as mtg
    dev = torch.device("cuda", 0)
    N, D, r, S = 10, 3, 4, a.segments
    ctx = mtg.Context(0)
    for B in map(int, a.batches.split(",")):
        mask, fixed, times, pos = mtg.generate_random_problems(N, D, S, B, seed0=105)
        plan = mtg.LinearPlan(ctx, N, D, r, S, mask)
        fd = torch.from_numpy(fixed).to(dev)
        td = torch.from_numpy(times).to(dev)
        nf = plan.n_fixed
        if a.workload == "linear":
            out = plan.solve(fd, td)
            fn = lambda: plan.solve(fd, td, out=out)  # noqa: E731
            bytes_per = (D * nf + S) * 8 + (S * D * N + 1) * 8 + 4
        elif a.workload == "time":
            fn = lambda: plan.time_optimize(fd, td, max_evals=a.evals)  # noqa: E731
            bytes_per = (D * nf + S) * 8 + (S + 2) * 8
        else:
            radii = torch.full((B, S, 2), 0.15, dtype=torch.float64, device=dev)
            pd = torch.from_numpy(pos).to(dev)
            tf = np.zeros((B, 3, N))
            tf[:, :, 0] = pos[:, 0, :]
            tf[:, :, N // 2] = pos[:, S, :]
            tfd = torch.from_numpy(tf).to(dev)
            fn = lambda: mtg.tube_solve(ctx, N, r, pd, tfd, td, td, radii)  # noqa: E731
            bytes_per = ((S + 1) * 3 + 3 * N + 4 * S) * 8 + (S * 3 * N + 1) * 8
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        ms = []
        for _ in range(a.reps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        k = float(np.median(ms))
        print(json.dumps({"workload": a.workload, "B": B, "S": S, "kernel_ms": k,
                          "traj_per_s": B / (k * 1e-3),
                          "alg_GBps": bytes_per * B / (k * 1e-3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
