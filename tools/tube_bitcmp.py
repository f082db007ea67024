"""Config 3 tube solve outputs of this build written to an .npz (run twice,
with MTG_LIB_PATH pointing at two builds, then compare): a bit-identity check
for changes that must not alter the arithmetic.

    python tools/tube_bitcmp.py out.npz
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mav_tube_trajectory_generation_amd as mtg  # noqa: E402


def main():
    N, D, r, S, B = 10, 3, 4, 10, 4096
    dev = torch.device("cuda:0")
    _, _, times, pos = mtg.generate_random_problems(N, D, S, B, seed0=105)
    M = N // 2
    tf = np.zeros((B, 3, N))
    tf[:, :, 0] = pos[:, 0, :]
    tf[:, :, M] = pos[:, S, :]
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    out = mtg.tube_solve(mtg.Context(0), N, r, T(pos), T(tf), T(times), T(times),
                         torch.full((B, S, 2), 0.15, dtype=torch.float64, device=dev))
    torch.cuda.synchronize()
    np.savez(sys.argv[1], **{k: v.cpu().numpy() for k, v in out.items()})


if __name__ == "__main__":
    main()
