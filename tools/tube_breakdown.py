"""Residuals recorded at an IPM breakdown of workgroup 0 (diagnostic build).

MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so python tools/tube_breakdown.py
"""
import ctypes
import os
import struct
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..'),
                os.path.join(os.path.dirname(__file__), '..', 'oracle'),
                os.path.join(os.path.dirname(__file__), '..', 'tests')]
import numpy as np  # noqa: E402
import pyoracle as o  # noqa: E402
import torch  # noqa: E402

import mav_tube_trajectory_generation_amd as mtg  # noqa: E402
from test_tube_gpu import tube_inputs  # noqa: E402

N, R, M, S = 10, 4, 5, 6
ctx = mtg.Context(0)
dev = torch.device('cuda', 0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
v = o.random_vertices(M - 1, S, 3, -10., 10., 77)
tcp = o.estimate_segment_times(v, 3., 5.)
t = tcp * 0.9
pos, fv = tube_inputs(v)
out = mtg.tube_solve(ctx, N, R, T(pos[None]), T(fv[None]), T(tcp[None]), T(t[None]),
                     T(np.full((1, S, 2), 0.15)), tol=1e-10, max_iter=100)
torch.cuda.synchronize()
L = mtg.lib()
L.mtg_debug_tube_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
st = (ctypes.c_ulonglong * 512)()
L.mtg_debug_tube_stamps(st, 512)
f = lambda k: struct.unpack('d', struct.pack('Q', st[k]))[0]  # noqa: E731
print("status", int(out["status"][0]), "iters", int(out["iters"][0]), "cause", st[303])
print("rdn", f(300), "rpn", f(301), "mu", f(302), "x304", f(304), "dxn", f(305), "sigma", f(306))
