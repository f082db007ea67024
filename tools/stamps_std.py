"""Phase timing of workgroup 0 of the standard-pattern linear kernel from the
diagnostic build (make STAMPS=1 STAMPS_OUT=...):

MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so \
    python tools/stamps_std.py [B]
Slots (mtg_linear_std.hip, mtg_std_device.h): 0 start, 7 times + powers,
1 fixed values, 2 assembly, 100+2k sweep step k start, 3 sweep end,
4 middle-vertex loads, 8 middle-vertex LDL^T, 9 back-substitution steps,
5 back substitution end (any/barrier), 6 coefficients/cost/stores.
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
    assert plan.kernel == "standard"
    fd, td = torch.from_numpy(fixed).to(dev), torch.from_numpy(times).to(dev)
    out = plan.solve(fd, td)
    L = mtg.lib()
    # STAMPS_SYM=wave: the compile-time-S kernel (mtg_linear_wave.hip)
    fn = getattr(L, "mtg_debug_stamps_" + os.environ.get("STAMPS_SYM", "std"))
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    runs = []
    for _ in range(7):
        plan.solve(fd, td, out=out)
        torch.cuda.synchronize()
        st = (ctypes.c_ulonglong * 512)()
        fn(st, 512)
        runs.append(np.array(st[:], dtype=np.int64))
    st = np.median(np.array(runs), axis=0)
    order = [(0, "start"), (7, "times arrived, powers"), (1, "fixed stored"),
             (12, "assembly stores"), (2, "assembly")]
    k = 0
    while st[100 + 2 * k] > 0:
        order.append((100 + 2 * k, f"(sweep step {k} start)"))
        k += 1
    order += [(3, "sweep end"), (4, "middle vertex loads")]
    if st[8] > 0:  # finer slots of the middle vertex / back substitution
        order += [(8, "middle vertex LDL^T")]
        if st[10] > 0:
            order += [(10, "back-sub loads"), (11, "back-sub chain")]
        order += [(9, "back substitution steps")]
    order += [(5, "back substitution end"), (6, "coeffs + cost + stores")]
    print(f"phase cycles (workgroup 0, median of 7, B={B}):")
    prev = st[0]
    for slot, name in order[1:]:
        if st[slot] == 0:  # slot not stamped by this kernel
            continue
        print(f"  {name:>24}: {st[slot] - prev:8.0f}")
        prev = st[slot]
    print(f"  total: {st[6] - st[0]:.0f} cycles")



if __name__ == "__main__":
    main()
