"""Diagnostic (GPU): IPM iteration counts of the tube solves along LN_SBPLX
paths (the oracle's evaluation histories of 16 C3 problems, 50 evaluations
each, control-point maps at T0) against the C3 problems at T0 themselves."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import mav_tube_trajectory_generation_amd as mtg  # noqa: E402
import pyoracle as oracle  # noqa: E402
from test_tube_gpu import tube_inputs  # noqa: E402

N, R, M, S = 10, 4, 5, 10
dev = torch.device("cuda", 0)
ctx = mtg.Context(0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
pts, t0s, pos, fv = [], [], [], []
for b in range(0, 256, 16):
    v = oracle.random_vertices(M - 1, S, 3, -10.0, 10.0, 700 + b)
    t = oracle.estimate_segment_times(v, 3.0, 5.0)
    h = oracle.tube_time_optimize_sbplx(N, R, v, t, np.full((S, 2), 0.15), 50)["history"]
    p0, f0 = tube_inputs(v)
    for x in h:
        pts.append(x)
        t0s.append(t)
        pos.append(p0)
        fv.append(f0)
K = len(pts)
out = mtg.tube_solve(ctx, N, R, T(np.stack(pos)), T(np.stack(fv)), T(np.stack(t0s)),
                     T(np.stack(pts)), T(np.full((K, S, 2), 0.15)))
it = out["iters"].cpu().numpy()
st = out["status"].cpu().numpy()
base = mtg.tube_solve(ctx, N, R, T(np.stack(pos)), T(np.stack(fv)), T(np.stack(t0s)),
                      T(np.stack(t0s)), T(np.full((K, S, 2), 0.15)))
ib = base["iters"].cpu().numpy()
print(f"SBPLX points: {K}, mean iterations {it.mean():.1f}, median {np.median(it):.0f}, "
      f"p90 {np.percentile(it, 90):.0f}, at cap {(it >= 100).mean():.3f}; "
      f"statuses {dict(zip(*np.unique(st, return_counts=True)))}")
print(f"same problems at T0: mean iterations {ib.mean():.1f}")
hist = np.bincount(np.minimum(it, 100) // 10, minlength=11)
print("iterations histogram (bins of 10):", hist.tolist())
