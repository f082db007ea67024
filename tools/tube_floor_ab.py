"""Config-3 status histogram and mean IPM iterations of the loaded library
(MTG_LIB_PATH=<variant> python tools/tube_floor_ab.py <label>): 4096
10-segment tube QCQPs of test_config3_tube_at_size's seeds."""
import sys
sys.path[:0] = ['.', 'tests']
import numpy as np
import torch
import mav_tube_trajectory_generation_amd as mtg
N, S, B, M, D = 10, 10, 4096, 5, 3
dev = torch.device('cuda', 0)
ctx = mtg.Context(0)
mask, fixed, times, pos = mtg.generate_random_problems(N, D, S, B, seed0=105)
tf = np.zeros((B, 3, N))
tf[:, :, 0] = pos[:, 0, :]
tf[:, :, M] = pos[:, S, :]
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
out = mtg.tube_solve(ctx, N, 4, T(pos), T(tf), T(times), T(times), T(np.full((B, S, 2), 0.15)))
st = out['status'].cpu().numpy()
it = out['iters'].cpu().numpy()
u, n = np.unique(st, return_counts=True)
print(sys.argv[1] if len(sys.argv) > 1 else '', 'status', dict(zip(u.tolist(), n.tolist())),
      'mean iters %.2f max %d' % (it.mean(), it.max()), 'non-zero', np.nonzero(st)[0].tolist())
