"""Regenerate tests/golden/linear_golden.json from the oracle.

The fixtures freeze the oracle's outputs (coefficients, cost) for small
problems: the reference's TwoVerticesSetup case, BASELINE config 1 (3-segment
3-D snap, seed 105), reference-fixture seeds, another polynomial order and an
irregular constraint pattern.  Inputs come from createRandomVertices /
estimateSegmentTimes (bit-exact to the reference generator).
Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pyoracle  # noqa: E402


def case(name, N, r, v, t):
    sol = pyoracle.linear_solve(N, r, v, t)
    return dict(name=name, N=N, r=r, mask=v.mask.tolist(), vals=v.vals.tolist(),
                times=list(map(float, t)), coeffs=sol["coeffs"].tolist(), cost=sol["cost"],
                nf=sol["nf"], np=sol["np"])


def main():
    cases = []
    mask = np.ones((2, 5), np.uint8)
    vals = np.zeros((2, 5, 1))
    vals[1, 0, 0] = 5.0
    cases.append(case("two_vertices_setup", 10, 4, pyoracle.Vertices(mask, vals), [5.0]))
    for name, N, r, S, D, seed, vm, am in [
            ("config1_3seg_3d_seed105", 10, 4, 3, 3, 105, 3.0, 5.0),
            ("segment_10_dim_3_seed105", 10, 4, 10, 3, 105, 3.0, 5.0),
            ("segment_10_dim_1_seed102", 10, 4, 10, 1, 102, 3.0, 5.0),
            ("deriv_jerk_seed110", 10, 3, 5, 3, 110, 1.0, 2.0),
            ("deriv_accel_seed109", 10, 2, 5, 3, 109, 1.0, 2.0),
            ("n8_snap_minus_one", 8, 3, 6, 3, 77, 3.0, 5.0)]:
        v = pyoracle.random_vertices(N // 2 - 1, S, D, -10.0, 10.0, seed)
        t = pyoracle.estimate_segment_times(v, vm, am)
        cases.append(case(name, N, r, v, t))
    v = pyoracle.random_vertices(4, 7, 2, -10.0, 10.0, 302)
    v.mask[0, 3:] = 0
    v.mask[3, 0] = 0
    v.mask[5, :] = 1
    v.vals[5, 1:, :] = np.random.default_rng(7).normal(size=(4, 2))
    cases.append(case("irregular_pattern_2d", 10, 4, v, np.linspace(0.8, 5.0, 7)))
    with open(os.path.join(HERE, "linear_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": cases}, f)
    print(f"wrote {len(cases)} cases")


if __name__ == "__main__":
    main()
