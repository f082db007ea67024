"""Per-iteration comparison of the GPU tube IPM with the oracle on one case.

python tools/debug_tube.py [random SEED S | stale]
"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..'),
                os.path.join(os.path.dirname(__file__), '..', 'oracle'),
                os.path.join(os.path.dirname(__file__), '..', 'tests')]
import numpy as np  # noqa: E402
import pyoracle as o  # noqa: E402
import torch  # noqa: E402

import mav_tube_trajectory_generation_amd as mtg  # noqa: E402
from test_tube_gpu import tube_inputs  # noqa: E402

N, R, M = 10, 4, 5
ctx = mtg.Context(0)
dev = torch.device('cuda', 0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
mode = sys.argv[1] if len(sys.argv) > 1 else "random"
if mode == "stale":
    S = 6
    v = o.random_vertices(M - 1, S, 3, -10., 10., 77)
    tcp = o.estimate_segment_times(v, 3., 5.)
    t = tcp * 0.9
else:
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 108
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    v = o.random_vertices(M - 1, S, 3, -10., 10., seed)
    t = o.estimate_segment_times(v, 3., 5.)
    tcp = t
radii = np.full((S, 2), 0.15)
pos, fv = tube_inputs(v)
for it in range(1, 45, 2):
    out = mtg.tube_solve(ctx, N, R, T(pos[None]), T(fv[None]), T(tcp[None]), T(t[None]),
                         T(radii[None]), tol=1e-10, max_iter=it)
    try:
        ro = o.tube_solve(N, R, v, t, radii, times_cp=tcp, tol=1e-10, max_iter=it)
        rc, rx, rs = ro['cost'], ro['x'], ro['status']
    except RuntimeError as e:
        rc, rx, rs = float('nan'), None, str(e)[-3:]
    x = out['x'].cpu().numpy()[0]
    dx = np.linalg.norm(x - rx) / np.linalg.norm(rx) if rx is not None else float('nan')
    print(it, int(out['status'][0]), int(out['iters'][0]), float(out['cost'][0]), rc, rs, dx)
