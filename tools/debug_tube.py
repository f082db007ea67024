import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..'), os.path.join(os.path.dirname(__file__), '..', 'oracle'), os.path.join(os.path.dirname(__file__), '..', 'tests')]
import numpy as np, torch, pyoracle as o
import mav_tube_trajectory_generation_amd as mtg
from test_tube_gpu import tube_inputs
N, R, M, S = 10, 4, 5, 10
ctx = mtg.Context(0); dev = torch.device('cuda', 0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
for b in [3]:
    v = o.random_vertices(M-1, S, 3, -10., 10., 105+b); t = o.estimate_segment_times(v, 3., 5.)
    ref = o.tube_solve(N, R, v, t, np.full((S,2),0.15), tol=1e-10, max_iter=100)
    print('oracle iters', ref['iters'], ref['status'], ref['cost'])
    pos, fv = tube_inputs(v)
    for it in list(range(1, 40, 2)):
        out = mtg.tube_solve(ctx, N, R, T(pos[None]), T(fv[None]), T(t[None]), T(t[None]), T(np.full((1,S,2),0.15)), tol=1e-10, max_iter=it)
        ro = o.tube_solve(N, R, v, t, np.full((S,2),0.15), tol=1e-10, max_iter=it)
        x = out['x'].cpu().numpy()[0]
        print(it, int(out['status'][0]), int(out['iters'][0]), float(out['cost'][0]), ro['cost'], np.linalg.norm(x-ro['x'])/np.linalg.norm(ro['x']))
