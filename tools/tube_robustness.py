"""Status histogram of the GPU tube IPM vs the oracle over random problems.

python tools/tube_robustness.py [B] [S] [radius]
"""
import os
import sys
from collections import Counter

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..'),
                os.path.join(os.path.dirname(__file__), '..', 'oracle'),
                os.path.join(os.path.dirname(__file__), '..', 'tests')]
import numpy as np  # noqa: E402
import pyoracle as o  # noqa: E402
import torch  # noqa: E402

import mav_tube_trajectory_generation_amd as mtg  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
S = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rad = float(sys.argv[3]) if len(sys.argv) > 3 else 0.15
N, R, M = 10, 4, 5
dev = torch.device('cuda', 0)
ctx = mtg.Context(0)
_, _, times, pos = mtg.generate_random_problems(N, 3, S, B, seed0=105)
fv = np.zeros((B, 3, N))
fv[:, :, 0] = pos[:, 0, :]
fv[:, :, M] = pos[:, S, :]
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
out = mtg.tube_solve(ctx, N, R, T(pos), T(fv), T(times), T(times), T(np.full((B, S, 2), rad)))
st = out["status"].cpu().numpy()
it = out["iters"].cpu().numpy()
x = out["x"].cpu().numpy()
ost, errs = [], []
for b in range(B):
    mask = np.zeros((S + 1, M), np.uint8)
    mask[:, 0] = 1
    mask[0, :] = 1
    mask[S, :] = 1
    vals = np.zeros((S + 1, M, 3))
    vals[:, 0, :] = pos[b]
    v = o.Vertices(mask, vals)
    try:
        r = o.tube_solve(N, R, v, times[b], np.full((S, 2), rad))
        ost.append(r["status"])
        if st[b] == 0 and r["status"] == 0:
            errs.append(np.linalg.norm(x[b] - r["x"]) / np.linalg.norm(r["x"]))
    except RuntimeError:
        ost.append(2)
print("gpu status", dict(Counter(st.tolist())), "oracle status", dict(Counter(ost)))
both = sum(1 for b in range(B) if st[b] == 0 and ost[b] == 0)
print("both converged", both, "of", B, " max rel err x", max(errs) if errs else None,
      " mean iters", it.mean())
print("gpu!=0 seeds", [105 + b for b in range(B) if st[b] != 0][:20])
print("oracle!=0 seeds", [105 + b for b in range(B) if ost[b] != 0][:20])
