"""GPU debug: objectiveFunctionTime with the QCQP inner solve on the main.cpp
geometry, at the control-point times and off them, grad on/off; the oracle
value beside it (test infrastructure, not the product path)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
import pyoracle as orc
import mav_tube_trajectory_generation_amd as mtg
from test_tube_gpu import main_cpp_vertices, tube_inputs

orc.lib()
ctx = mtg.Context(0)
dev = torch.device("cuda", 0)
v = main_cpp_vertices(orc)
S = v.S
t0 = orc.estimate_segment_times(v, 2.0, 2.0)
pos, fv = tube_inputs(v)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
radii = np.full((1, S, 2), 0.15)
for scale in (1.0, 1.05):
    t = t0 * scale
    for grad in (False, True):
        out = mtg.tube_time_cost(ctx, 10, 4, T(pos[None]), T(fv[None]), T(t0[None]), T(t[None]),
                                 T(radii), grad=grad)
        Jr, gr = orc.tube_time_cost(10, 4, v, t, radii[0], times_cp=t0, grad_mode=2)
        print("scale", scale, "grad", grad, "J", out["cost"].item(), "oracle", Jr,
              "status", out["status"].item(), "sumT", t.sum(), flush=True)
