"""Phase timing of workgroup 0 from the diagnostic build (make STAMPS=1).

MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so \
    python tools/stamps.py [B]
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N, D, r, S = 10, 3, 4, 10
    dev = torch.device("cuda", 0)
    ctx = mtg.Context(0)
    mask, fixed, times, _ = mtg.generate_random_problems(N, D, S, B, seed0=105)
    plan = mtg.LinearPlan(ctx, N, D, r, S, mask)
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    out = plan.solve(fd, td)
    L = mtg.lib()
    L.mtg_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    runs = []
    for _ in range(5):
        plan.solve(fd, td, out=out)
        torch.cuda.synchronize()
        st = (ctypes.c_ulonglong * 512)()
        L.mtg_debug_stamps(st, 512)
        runs.append(np.array(st[:], dtype=np.int64))
    st = np.median(np.array(runs), axis=0)
    t0 = st[0]
    names = {0: "start", 1: "loaded", 2: "powers", 3: "assembled", 4: "swept", 5: "backsub",
             6: "end"}
    print("phase cycles (workgroup 0, median of 5):")
    prev = t0
    for k in (1, 2, 3):
        print(f"  {names[k]:>10}: {st[k] - prev:8.0f}")
        prev = st[k]
    for v in range(S + 1):
        a, b = st[100 + 2 * v], st[101 + 2 * v]
        print(f"  vertex {v:2d}: schur {a - prev:6.0f}  factor+solve {b - a:6.0f}")
        prev = b
    for k in (4, 5, 6):
        print(f"  {names[k]:>10}: {st[k] - prev:8.0f}")
        prev = st[k]
    print(f"  total: {st[6] - t0:.0f} cycles")


if __name__ == "__main__":
    main()
