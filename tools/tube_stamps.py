"""Phase cycle totals of the tube IPM (workgroup 0) from the diagnostic
build (make STAMPS=1 STAMPS_OUT=../libmtg_hip_stamps.so):

MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so \\
    python tools/tube_stamps.py [B]
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

NAMES = {200: "residuals+rd", 201: "assemble G", 202: "factor", 203: "direction 1",
         204: "step/sigma", 205: "direction 2", 206: "update", 210: "  (solves in dirs)",
         220: "  (factor: init cols)", 221: "  (factor: G terms)", 222: "  (factor: Schur)",
         223: "  (factor: eliminate)", 224: "  (factor: store)"}


def main():
    import numpy as np
    import torch
    import mav_tube_trajectory_generation_amd as mtg
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N, R, S = 10, 4, 10
    dev = torch.device("cuda", 0)
    ctx = mtg.Context(0)
    _, _, times, pos = mtg.generate_random_problems(N, 3, S, B, seed0=105)
    M = N // 2
    fv = np.zeros((B, 3, N))
    fv[:, :, 0] = pos[:, 0, :]
    fv[:, :, M] = pos[:, S, :]
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    args = (ctx, N, R, T(pos), T(fv), T(times), T(times), T(np.full((B, S, 2), 0.15)))
    L = mtg.lib()
    L.mtg_debug_tube_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]

    def read():
        st = (ctypes.c_ulonglong * 512)()
        L.mtg_debug_tube_stamps(st, 512)
        return np.array(st[:], dtype=np.int64)

    mtg.tube_solve(*args)
    torch.cuda.synchronize()
    s0 = read()
    out = mtg.tube_solve(*args)
    torch.cuda.synchronize()
    d = read() - s0
    it = int(out["iters"][0])
    print(f"workgroup 0: {it} iterations; cycles per iteration:")
    tot = 0
    for k, name in NAMES.items():
        v = d[k] / max(it, 1)
        if k < 210:  # top-level phases; the rest are breakdowns
            tot += v
        print(f"  {name:>20}: {v:10.0f}")
    print(f"  {'total':>20}: {tot:10.0f}")


if __name__ == "__main__":
    main()
