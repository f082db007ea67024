"""Per-lane work of the soft-constraint extremum searches inside the time
optimiser (diagnostic build, make STAMPS=1): nodes visited and Laguerre
iterations per lane of workgroup 0, summed over one 50-evaluation
optimisation, for a few trajectories of the bench's C5 problem set.

MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so \
    python tools/soft_search_stats.py [n_traj]
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch
    import mav_tube_trajectory_generation_amd as mtg
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    N, D, r, S = 10, 3, 4, 10
    dev = torch.device("cuda", 0)
    ctx = mtg.Context(0)
    L = mtg.lib()
    L.mtg_debug_stamps_time.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]

    def read():
        st = (ctypes.c_ulonglong * 512)()
        L.mtg_debug_stamps_time(st, 512)
        return np.array(st[:], dtype=np.int64)

    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, n, seed0=105)
    plan = mtg.LinearPlan(ctx, N, D, r, S, mask)
    tot_nodes = np.zeros(64, np.int64)
    for b in range(n):
        fd = torch.from_numpy(fixed[b:b + 1]).to(dev)
        td = torch.from_numpy(times[b:b + 1]).to(dev)
        before = read()
        out = plan.time_optimize(fd, td, max_evals=50, soft=[(1, 3.0), (2, 5.0)])
        torch.cuda.synchronize()
        after = read()
        nodes = (after - before)[320:384]
        iters = (after - before)[384:448]
        act = nodes[:60]
        tot_nodes += nodes
        print(f"traj {b}: solves {int(out['solves'][0])}  nodes/lane mean {act.mean():.0f} "
              f"max {act.max()} (lane {act.argmax()})  min {act.min()}  "
              f"laguerre/lane mean {iters[:60].mean():.0f} max {iters[:60].max()}")
        d = after - before
        tot = after[461] - after[460]
        print(f"   cycles: kernel loop {tot}  solve+coeffs {d[450]}  search K=1 {d[451]}  "
              f"search K=2 {d[452]}  per solve: {d[450] / int(out['solves'][0]):.0f} / "
              f"{d[451] / int(out['solves'][0]):.0f} / {d[452] / int(out['solves'][0]):.0f}")
        ns = 2 * int(out['solves'][0])
        print(f"   search phases per call (lane 0): bound {d[470] / ns:.0f}  setup "
              f"{d[471] / ns:.0f}  tree walk {d[472] / ns:.0f}  reductions {d[473] / ns:.0f}")
        print(f"   node {d[474] / (ns / 2):.0f}  lane-0 refine {d[475] / (ns / 2):.0f}  "
              f"refine+value {d[476] / (ns / 2):.0f} (per evaluation)")
        print("   nodes per lane:", " ".join(str(x) for x in act))
        print("   iters per lane:", " ".join(str(x) for x in iters[:60]))
        print("   max iters in one call per lane:", " ".join(str(x) for x in after[256:316]))


if __name__ == "__main__":
    main()
