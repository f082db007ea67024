"""Independent NumPy restatement of the linear path, used only to cross-check
the C++ oracle (tests/test_oracle.py).  Written from the math, not from the
oracle: dense A(T), Q(T) by definition, and the constrained minimiser from the
full KKT system of  min 0.5 sum c^T Q c  s.t.  A_s c_s = endpoint derivatives
with shared (continuity) and fixed values.
"""
import numpy as np


def falling(n, i):
    if i < n:
        return 0.0
    p = 1.0
    for m in range(n):
        p *= (i - m)
    return p


def mapping_matrix(N, T):
    M = N // 2
    A = np.zeros((N, N))
    for l in range(M):
        A[l, l] = falling(l, l)
        for j in range(l, N):
            A[M + l, j] = falling(l, j) * T ** (j - l)
    return A


def cost_matrix(N, r, T):
    Q = np.zeros((N, N))
    for j in range(r, N):
        for k in range(r, N):
            e = j + k - 2 * r + 1
            Q[j, k] = 2.0 * falling(r, j) * falling(r, k) * T ** e / e
    return Q


def solve_linear(N, r, mask, vals, times):
    """mask [(S+1), M] fixed flags, vals [(S+1), M, D]; returns coeffs [S, D, N]
    and cost.  Unknowns: all vertex derivatives x (S+1)*M per dimension;
    coefficients c_s = A_s^-1 [x_s; x_{s+1}]; minimise sum x^T H x over the
    free entries with an equality-constrained dense solve."""
    M = N // 2
    S = len(times)
    D = vals.shape[2]
    n = (S + 1) * M
    R = np.zeros((n, n))
    Ainvs = []
    for s in range(S):
        Ai = np.linalg.inv(mapping_matrix(N, times[s]))
        Ainvs.append(Ai)
        H = Ai.T @ cost_matrix(N, r, times[s]) @ Ai
        idx = np.r_[s * M:(s + 1) * M, (s + 1) * M:(s + 2) * M]
        R[np.ix_(idx, idx)] += H
    fixed = mask.reshape(-1).astype(bool)
    free = ~fixed
    coeffs = np.zeros((S, D, N))
    cost = 0.0
    for d in range(D):
        x = np.zeros(n)
        x[fixed] = vals.reshape(n, D)[fixed, d]
        if free.any():
            x[free] = np.linalg.solve(R[np.ix_(free, free)], -R[np.ix_(free, fixed)] @ x[fixed])
        for s in range(S):
            e = x[s * M:(s + 2) * M]
            coeffs[s, d] = Ainvs[s] @ e
            cost += 0.5 * coeffs[s, d] @ cost_matrix(N, r, times[s]) @ coeffs[s, d]
    return coeffs, cost


# -- std::mt19937 + std::uniform_real_distribution<double> (libstdc++) ------
class MT19937:
    def __init__(self, seed):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            self.mt[i] = (1812433253 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.i = 624

    def __call__(self):
        if self.i >= 624:
            for k in range(624):
                y = (self.mt[k] & 0x80000000) | (self.mt[(k + 1) % 624] & 0x7FFFFFFF)
                self.mt[k] = self.mt[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            self.i = 0
        y = self.mt[self.i]
        self.i += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF


def uniform_real(gen, a, b):
    """generate_canonical<double, 53> with a 32-bit engine: two draws."""
    lo = float(gen())
    hi = float(gen())
    s = lo + hi * 4294967296.0
    x = s / 18446744073709551616.0
    if x >= 1.0:
        x = np.nextafter(1.0, 0.0)
    return x * (b - a) + a


def random_positions(S, D, lo, hi, seed):
    """Vertex positions of createRandomVertices (vertex.cpp:27-82)."""
    g = MT19937(seed)
    last = np.array([uniform_real(g, lo, hi) for _ in range(D)])
    out = [last]
    for _ in range(S):
        while True:
            p = np.array([uniform_real(g, lo, hi) for _ in range(D)])
            if np.linalg.norm(p - last) > 0.2:
                break
        out.append(p)
        last = p
    return np.array(out)
