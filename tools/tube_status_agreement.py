"""Status agreement of the GPU tube QCQP with the oracle on 400 random
10-segment problems (histogram of (gpu, oracle) statuses, -22 = oracle
breakdown).  MTG_LIB_PATH=<lib> python tools/tube_status_agreement.py [label]
"""
import sys
sys.path[:0] = ['.', 'oracle', 'tests']
import numpy as np, torch
import pyoracle as oracle
import mav_tube_trajectory_generation_amd as mtg
dev = torch.device('cuda', 0)
ctx = mtg.Context(0)
N, R, S, B = 10, 4, 10, 400
M = N // 2
items = []
for b in range(B):
    v = oracle.random_vertices(M - 1, S, 3, -10.0, 10.0, 105 + b)
    items.append((v, oracle.estimate_segment_times(v, 3.0, 5.0)))
pos = np.stack([v.vals[:, 0, :] for v, _ in items])
fv = np.zeros((B, 3, N))
for b, (v, _) in enumerate(items):
    fv[b, :, :M] = v.vals[0, :M, :].T
    fv[b, :, M:] = v.vals[S, :M, :].T
times = np.stack([t for _, t in items])
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
out = mtg.tube_solve(ctx, N, R, T(pos), T(fv), T(times), T(times), T(np.full((B, S, 2), 0.15)), tol=1e-10, max_iter=100)
o = {k: v.cpu().numpy() for k, v in out.items()}
agree = 0; both0 = 0; g0 = 0; r0 = 0; maxerr = 0
hist = {}
for b, (v, t) in enumerate(items):
    try:
        ref = oracle.tube_solve(N, R, v, t, np.full((S, 2), 0.15), tol=1e-10, max_iter=100)
        rs = int(ref['status'])
    except RuntimeError:
        rs = -22
    key = (int(o['status'][b]), rs)
    hist[key] = hist.get(key, 0) + 1
    if key == (0, 0):
        maxerr = max(maxerr, abs(o['cost'][b] - ref['cost']) / abs(ref['cost']))
print(sys.argv[1] if len(sys.argv) > 1 else '', 'status (gpu, oracle) histogram', sorted(hist.items()), 'max rel cost err', maxerr, 'mean iters', o['iters'].mean())
