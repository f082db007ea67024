"""Diagnostic (GPU): where the device LN_SBPLX-over-QCQP path and the oracle's
part.  For each picked trajectory: device (evals, result, cost) vs oracle, and
the objective of both implementations at every point of the oracle's
evaluation history (first point where they differ by more than 1e-8
relative, or where exactly one is NaN), plus the QCQP statuses there."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import mav_tube_trajectory_generation_amd as mtg  # noqa: E402
import pyoracle as oracle  # noqa: E402
from test_tube_gpu import tube_inputs  # noqa: E402

N, R, M = 10, 4, 5
S, B, E = int(sys.argv[1]) if len(sys.argv) > 1 else 10, 256, 50
dev = torch.device("cuda", 0)
ctx = mtg.Context(0)
vs = [oracle.random_vertices(M - 1, S, 3, -10.0, 10.0, s) for s in range(700, 700 + B)]
times = np.stack([oracle.estimate_segment_times(v, 3.0, 5.0) for v in vs])
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
pos = T(np.stack([tube_inputs(v)[0] for v in vs]))
fv = T(np.stack([tube_inputs(v)[1] for v in vs]))
radii = T(np.full((B, S, 2), 0.15))
out = mtg.tube_time_optimize(ctx, N, R, pos, fv, radii, T(times), max_evals=E, optimizer="sbplx")
out = {k: v.cpu().numpy() for k, v in out.items()}
for b in range(0, B, B // 16):
    r = oracle.tube_time_optimize_sbplx(N, R, vs[b], times[b], np.full((S, 2), 0.15), E)
    h = r["history"]
    k = len(h)
    Jg = mtg.tube_time_cost(ctx, N, R, pos[b:b + 1].repeat(k, 1, 1), fv[b:b + 1].repeat(k, 1, 1),
                            T(np.repeat(times[b:b + 1], k, 0)), T(h),
                            radii[b:b + 1].repeat(k, 1, 1))
    jg = Jg["cost"].cpu().numpy()
    sg = Jg["status"].cpu().numpy()
    jo = np.array([oracle.tube_time_cost(N, R, vs[b], h[i], np.full((S, 2), 0.15),
                                         times_cp=times[b])[0] for i in range(k)])
    rel = np.abs(jg - jo) / np.abs(jo)
    nanmis = np.isnan(jg) != np.isnan(jo)
    bad = np.where(nanmis | (rel > 1e-8))[0]
    first = int(bad[0]) if len(bad) else -1
    print(f"b={b:3d} dev(evals={out['evals'][b]}, res={out['result'][b]}, cost={out['cost'][b]:.12g})"
          f" orc(evals={r['evals']}, res={r['result']}, cost={r['cost']:.12g})"
          f" maxrel={np.nanmax(rel):.2e} nan_dev={int(np.isnan(jg).sum())}"
          f" nan_orc={int(np.isnan(jo).sum())} first_diff={first}"
          f" dev_status_hist={dict(zip(*np.unique(sg, return_counts=True)))}", flush=True)
