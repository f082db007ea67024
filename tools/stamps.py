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
        L.mtg_debug_stamps_clear() if hasattr(L, 'mtg_debug_stamps_clear') else None
    st = np.median(np.array(runs), axis=0)
    t0 = st[0]
    print("phase cycles (workgroup 0, median of 5):")
    print(f"  {'loaded':>22}: {st[1] - t0:8.0f}")
    print(f"  {'powers':>22}: {st[2] - st[1]:8.0f}")
    print(f"  {'assembled':>22}: {st[3] - st[2]:8.0f}")
    prev = st[3]
    k = 0
    while st[100 + 2 * k] > 0 and 100 + 2 * k < 500:  # sweep steps (both ends at once)
        a, b = st[100 + 2 * k], st[101 + 2 * k]
        print(f"  {'sweep step ' + str(k):>22}: {b - prev:8.0f}")
        prev = b
        k += 1
    print(f"  {'middle vertex':>22}: {st[4] - prev:8.0f}")
    print(f"  {'back substitution':>22}: {st[5] - st[4]:8.0f}")
    print(f"  {'coeffs+cost+store':>22}: {st[6] - st[5]:8.0f}")
    print(f"  total: {st[6] - t0:.0f} cycles")


if __name__ == "__main__":
    main()
