"""Exact (rational-arithmetic) solutions of small linear problems.

The reference algorithm in FP64 is only as accurate as cond(R_pp) * eps: for
N = 12 and low derivative orders the cost matrix Q(1) is Hilbert-like and the
reference-faithful oracle drifts up to ~4e-4 from the true minimiser.  These
fixtures hold the exact solution (fractions.Fraction end to end, rounded once
to FP64) so tests can state both parity with the oracle where the oracle is
accurate, and accuracy against the truth everywhere.
Run: python tests/golden/make_exact.py   (a few minutes)
"""
import json
import os
import sys
from fractions import Fraction as F

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "..", "oracle"), os.path.join(HERE, "..")]
import helpers  # noqa: E402
import pyoracle  # noqa: E402


def falling(n, i):
    if i < n:
        return 0
    p = 1
    for m in range(n):
        p *= (i - m)
    return p


def gauss_jordan(A, m, ncols):
    for k in range(m):
        p = next(i for i in range(k, m) if A[i][k] != 0)
        A[k], A[p] = A[p], A[k]
        pv = A[k][k]
        A[k] = [x / pv for x in A[k]]
        for i in range(m):
            if i != k and A[i][k] != 0:
                f = A[i][k]
                A[i] = [a - f * b for a, b in zip(A[i], A[k])]
    return A


def exact_solve(N, r, mask, vals, times):
    M = N // 2
    S = len(times)
    D = vals.shape[2]
    T = [F(float(t)) for t in times]
    n = (S + 1) * M
    R = [[F(0)] * n for _ in range(n)]
    Ais = []
    for s in range(S):
        A = [[F(0)] * N for _ in range(N)]
        for l in range(M):
            A[l][l] = F(falling(l, l))
            for j in range(l, N):
                A[M + l][j] = F(falling(l, j)) * T[s] ** (j - l)
        aug = gauss_jordan([row[:] + [F(int(i == j)) for j in range(N)]
                            for i, row in enumerate(A)], N, 2 * N)
        Ai = [row[N:] for row in aug]
        Ais.append(Ai)
        Q = [[F(0)] * N for _ in range(N)]
        for j in range(r, N):
            for k in range(r, N):
                e = j + k - 2 * r + 1
                Q[j][k] = F(2 * falling(r, j) * falling(r, k)) * T[s] ** e / e
        QA = [[sum(Q[i][k] * Ai[k][j] for k in range(N)) for j in range(N)] for i in range(N)]
        H = [[sum(Ai[k][i] * QA[k][j] for k in range(N)) for j in range(N)] for i in range(N)]
        for a in range(N):
            for b in range(N):
                R[s * M + a][s * M + b] += H[a][b]
    fixed = mask.reshape(-1).astype(bool)
    fr = [i for i in range(n) if not fixed[i]]
    fx = [i for i in range(n) if fixed[i]]
    out = np.zeros((S, D, N))
    for d in range(D):
        x = [F(0)] * n
        for i in fx:
            x[i] = F(float(vals[i // M, i % M, d]))
        A = [[R[i][j] for j in fr] + [-sum(R[i][j] * x[j] for j in fx)] for i in fr]
        A = gauss_jordan(A, len(fr), len(fr) + 1)
        for t, i in enumerate(fr):
            x[i] = A[t][len(fr)]
        for s in range(S):
            e = x[s * M:(s + 2) * M]
            for k in range(N):
                out[s, d, k] = float(sum(Ais[s][k][j] * e[j] for j in range(N)))
    return out


def main():
    cases = []
    S, D = 6, 1
    for N in (4, 6, 8, 10, 12):
        v3 = helpers.standard_vertices(N, S, 3, 200 + N)
        v = pyoracle.Vertices(v3.mask, v3.vals[:, :, :1])
        t = pyoracle.estimate_segment_times(v, 3.0, 5.0)
        for r in range(N // 2):
            ex = exact_solve(N, r, v.mask, v.vals, t)
            orc = pyoracle.linear_solve(N, r, v, t)
            err = helpers.rel_err_coeffs(orc["coeffs"], ex)
            cases.append(dict(N=N, r=r, mask=v.mask.tolist(), vals=v.vals.tolist(),
                              times=list(map(float, t)), exact=ex.tolist(), oracle_err=err))
            print(N, r, err, flush=True)
    with open(os.path.join(HERE, "exact_linear.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_exact.py", "cases": cases}, f)


if __name__ == "__main__":
    main()
