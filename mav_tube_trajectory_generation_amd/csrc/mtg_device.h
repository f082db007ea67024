// mtg_device.h — per-trajectory FP64 solver run by one 64-lane wavefront
// (one workgroup) on gfx950.  Shared by the linear-solve, time-cost and
// time-optimisation kernels (mtg_kernels.hip).
//
// Math (restated from the reference):
//   per segment s: H_s = A_s^-T Q_s A_s^-1            (linear_impl:318)
//   R = M^T blkdiag(H_s) M,  R_pp d_p = -R_pf d_f      (linear_impl:306-375)
//   c_s = A_s^-1 [d(vertex s); d(vertex s+1)]          (linear_impl:254-275)
//   J = 0.5 sum_s sum_dim c^T Q_s c                    (linear_impl:113-130)
// MI355X formulation:
//   * H_s(T) = T^(1-2r) S_T H(1) S_T and A_s^-1(T) = D_T^-1 A(1)^-1 S_T with
//     S_T = diag(T^(j mod M)), D_T = diag(T^k): an exact identity of the
//     time-scaling t = T tau, so the per-segment inversion and the two 10x10
//     GEMMs of constructR become one table lookup times a power of T per
//     entry (tables H(1), A(1)^-1 are built once per (N, r) on the host in
//     long double, mtg_host.cpp).
//   * R in vertex order is block tridiagonal with M x M blocks
//     (M = N/2 derivatives per vertex).  Fixed derivatives are "pinned"
//     (identity row/column, value on the right-hand side), which leaves the
//     free-free system R_pp d_p = -R_pf d_f unchanged while giving every
//     trajectory the same uniform block structure.  It is solved by a block
//     Cholesky sweep over the S+1 vertices: lanes build the Schur complement
//     and right-hand side in parallel, then lane c factors the M x M block in
//     registers and triangular-solves column c (M columns of the coupling
//     block + D right-hand sides), so one barrier pair per vertex.
// LDS holds everything a trajectory touches (about 9 KB at S=10, N=10, D=3);
// HBM sees only the compact inputs (times, d_f) and the outputs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtg_internal.h"

namespace mtg {

constexpr int kWave = 64;

// LDS carve-up (in doubles, then ints), identical for every kernel.
struct Layout {
  int tabH, tabA;  // H(1), A(1)^-1: N*N each
  int pw;          // S * (2N-1): T_s^e for e in [-(N-1), N-1]
  int T;           // S segment times
  int dv;          // (S+1)*M*D vertex derivatives (fixed values, then x)
  int L;           // (S+1)*M*M Cholesky factors
  int W;           // S*M*M     L_v^-1 * O_v
  int Y;           // (S+1)*M*D forward solutions
  int Sv, Ov, Rv;  // per-step workspace
  int red;         // 64 reduction scratch
  int aux;         // 4*S extra (optimiser state)
  int ndouble;
  int slot;        // (S+1)*M int slots (after the doubles)
  int nint;
  size_t bytes() const { return sizeof(double) * ndouble + sizeof(int) * nint; }
};

__host__ __device__ inline Layout make_layout(int N, int S, int D) {
  const int M = N / 2;
  Layout l;
  int o = 0;
  l.tabH = o; o += N * N;
  l.tabA = o; o += N * N;
  l.pw = o;   o += S * (2 * N - 1);
  l.T = o;    o += S;
  l.dv = o;   o += (S + 1) * M * D;
  l.L = o;    o += (S + 1) * M * M;
  l.W = o;    o += S * M * M;
  l.Y = o;    o += (S + 1) * M * D;
  l.Sv = o;   o += M * M;
  l.Ov = o;   o += M * M;
  l.Rv = o;   o += M * kMaxD;
  l.red = o;  o += kWave;
  l.aux = o;  o += 4 * S + 8;
  l.ndouble = o;
  l.slot = 0;
  l.nint = (S + 1) * M + 4;
  return l;
}

// Per-trajectory solver state living in LDS.  Every method is called by all
// 64 lanes of the (single-wave) workgroup.
template <int N>
struct Traj {
  static constexpr int M = N / 2;
  static constexpr int PWN = 2 * N - 1;
  int S, D, r;
  const Layout* lay;
  double* sm;   // double region
  int* si;      // int region
  int lane;

  __device__ double* tabH() const { return sm + lay->tabH; }
  __device__ double* tabA() const { return sm + lay->tabA; }
  __device__ double* pw() const { return sm + lay->pw; }
  __device__ double* T() const { return sm + lay->T; }
  __device__ double* dv() const { return sm + lay->dv; }
  __device__ double* Lf() const { return sm + lay->L; }
  __device__ double* W() const { return sm + lay->W; }
  __device__ double* Y() const { return sm + lay->Y; }
  __device__ int* slot() const { return si + lay->slot; }
  __device__ int* flag() const { return si + (S + 1) * M; }

  // T_s^e, e in [-(N-1), N-1].
  __device__ double pwr(int s, int e) const { return pw()[s * PWN + e + (N - 1)]; }
  __device__ bool fixed_at(int v, int k) const { return slot()[v * M + k] >= 0; }

  // H_s block entry: row (a_blk, j), column (b_blk, k); a_blk 0 = start
  // vertex s, 1 = end vertex s+1.
  __device__ double H(int s, int ab, int bb, int j, int k) const {
    return tabH()[(ab * M + j) * N + bb * M + k] * pwr(s, 1 - 2 * r + j + k);
  }

  // Load the constant tables and the slot map (global -> LDS).
  __device__ void load_static(const double* __restrict__ tab,
                              const int* __restrict__ slots) {
    for (int i = lane; i < 2 * N * N; i += kWave) sm[lay->tabH + i] = tab[i];
    for (int i = lane; i < (S + 1) * M; i += kWave) slot()[i] = slots[i];
    if (lane == 0) flag()[0] = 0;
  }

  // Powers T_s^e by repeated multiplication (exact integer exponents).
  // Returns via flag()[0] |= 1 if any time is not > 0.
  __device__ void compute_powers() {
    for (int i = lane; i < S * PWN; i += kWave) {
      const int s = i / PWN;
      const int e = i % PWN - (N - 1);
      const double t = T()[s];
      if (!(t > 0.0) || !(t < 1e300)) atomicOr(&flag()[0], 1);
      const double base = e < 0 ? 1.0 / t : t;
      const int n = e < 0 ? -e : e;
      double p = 1.0;
      for (int q = 0; q < n; ++q) p *= base;
      pw()[i] = p;
    }
  }

  // Scatter compact fixed values d_f (D x nf, global) into dv; free entries 0.
  __device__ void load_fixed(const double* __restrict__ df, int nf) {
    for (int i = lane; i < (S + 1) * M * D; i += kWave) {
      const int v = i / (M * D);
      const int rem = i % (M * D);
      const int k = rem / D;
      const int d = rem % D;
      const int sl = slot()[v * M + k];
      dv()[i] = sl >= 0 ? df[d * nf + sl] : 0.0;
    }
  }

  // Re-zero the free entries of dv (before a re-solve that reuses dv).
  __device__ void clear_free() {
    for (int i = lane; i < (S + 1) * M * D; i += kWave) {
      const int v = i / (M * D);
      const int k = (i % (M * D)) / D;
      if (slot()[v * M + k] < 0) dv()[i] = 0.0;
    }
  }

  __device__ double dval(int v, int k, int d) const {
    return dv()[(v * M + k) * D + d];
  }

  // Block-tridiagonal Cholesky forward sweep + back substitution.  On exit
  // dv holds every vertex derivative (fixed values untouched bit-for-bit).
  // Sets flag()[0] |= 2 on a non-positive pivot.
  __device__ void solve() {
    double* Sv = sm + lay->Sv;
    double* Ov = sm + lay->Ov;
    double* Rv = sm + lay->Rv;
    for (int v = 0; v <= S; ++v) {
      const double* Wp = W() + (v - 1) * M * M;  // valid for v > 0
      const double* Yp = Y() + (v - 1) * M * D;
      if (lane < M * M) {
        const int j = lane / M, k = lane % M;
        const bool fj = fixed_at(v, j), fk = fixed_at(v, k);
        double sval;
        if (fj || fk) {
          sval = (j == k) ? 1.0 : 0.0;
        } else {
          sval = 0.0;
          if (v > 0) sval += H(v - 1, 1, 1, j, k);
          if (v < S) sval += H(v, 0, 0, j, k);
          if (v > 0) {
#pragma unroll
            for (int m = 0; m < M; ++m) sval -= Wp[m * M + j] * Wp[m * M + k];
          }
        }
        Sv[j * M + k] = sval;
        if (v < S) {
          const bool pin = fj || fixed_at(v + 1, k);
          Ov[j * M + k] = pin ? 0.0 : H(v, 0, 1, j, k);
        }
      } else if (lane < M * M + M * D) {
        const int idx = lane - M * M;
        const int j = idx / D, d = idx % D;
        double rv;
        if (fixed_at(v, j)) {
          rv = dval(v, j, d);
        } else {
          double b = 0.0;
#pragma unroll
          for (int k = 0; k < M; ++k) {
            double dkk = 0.0;
            if (v > 0) dkk += H(v - 1, 1, 1, j, k);
            if (v < S) dkk += H(v, 0, 0, j, k);
            b += dkk * dval(v, k, d);
            if (v < S) b += H(v, 0, 1, j, k) * dval(v + 1, k, d);
            if (v > 0) b += H(v - 1, 1, 0, j, k) * dval(v - 1, k, d);
          }
          rv = -b;
          if (v > 0) {
#pragma unroll
            for (int m = 0; m < M; ++m) rv -= Wp[m * M + j] * Yp[m * D + d];
          }
        }
        Rv[j * D + d] = rv;
      }
      __syncthreads();
      // Lane -> column: 0..M-1 the coupling block W_v (absent at v = S),
      // then the D right-hand sides.
      int col;
      if (v < S)
        col = lane < M + D ? lane : -1;
      else
        col = lane < D ? M + lane : -1;
      if (col >= 0) {
        // Cholesky of Sv in registers (lower triangle).
        double Lr[M][M];
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
          for (int j = 0; j < M; ++j) Lr[i][j] = (j <= i) ? Sv[i * M + j] : 0.0;
        bool ok = true;
#pragma unroll
        for (int j = 0; j < M; ++j) {
          double dj = Lr[j][j];
#pragma unroll
          for (int k = 0; k < j; ++k) dj -= Lr[j][k] * Lr[j][k];
          ok = ok && (dj > 0.0);
          dj = sqrt(dj > 0.0 ? dj : 1.0);
          Lr[j][j] = dj;
          const double inv = 1.0 / dj;
#pragma unroll
          for (int i = j + 1; i < M; ++i) {
            double s = Lr[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) s -= Lr[i][k] * Lr[j][k];
            Lr[i][j] = s * inv;
          }
        }
        if (!ok) atomicOr(&flag()[0], 2);
        if (lane == 0) {
          double* Lv = Lf() + v * M * M;
#pragma unroll
          for (int i = 0; i < M; ++i)
#pragma unroll
            for (int j = 0; j < M; ++j) Lv[i * M + j] = Lr[i][j];
        }
        // Forward substitution on one column.
        double x[M];
        const bool isW = col < M;
#pragma unroll
        for (int i = 0; i < M; ++i)
          x[i] = isW ? Ov[i * M + col] : Rv[i * D + (col - M)];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          double s = x[i];
#pragma unroll
          for (int k = 0; k < i; ++k) s -= Lr[i][k] * x[k];
          x[i] = s / Lr[i][i];
        }
        if (isW) {
          double* Wv = W() + v * M * M;
#pragma unroll
          for (int i = 0; i < M; ++i) Wv[i * M + col] = x[i];
        } else {
          double* Yv = Y() + v * M * D;
#pragma unroll
          for (int i = 0; i < M; ++i) Yv[i * D + (col - M)] = x[i];
        }
      }
      __syncthreads();
    }
    // Back substitution: x_v = L_v^-T (y_v - W_v x_{v+1}), one lane per dim.
    if (lane < D) {
      const int d = lane;
      double xn[M];
#pragma unroll
      for (int i = 0; i < M; ++i) xn[i] = 0.0;
      for (int v = S; v >= 0; --v) {
        const double* Lv = Lf() + v * M * M;
        const double* Wv = W() + v * M * M;
        const double* Yv = Y() + v * M * D;
        double t[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          double s = Yv[i * D + d];
          if (v < S) {
#pragma unroll
            for (int k = 0; k < M; ++k) s -= Wv[i * M + k] * xn[k];
          }
          t[i] = s;
        }
#pragma unroll
        for (int i = M - 1; i >= 0; --i) {
          double s = t[i];
#pragma unroll
          for (int k = i + 1; k < M; ++k) s -= Lv[k * M + i] * t[k];
          t[i] = s / Lv[i * M + i];
        }
#pragma unroll
        for (int i = 0; i < M; ++i) {
          xn[i] = t[i];
          // Fixed entries come back as their pinned value exactly; keep the
          // original bits anyway (no-op in exact arithmetic).
          if (!fixed_at(v, i)) dv()[(v * M + i) * D + d] = t[i];
        }
      }
    }
    __syncthreads();
  }

  // c_s[d][k] = sum_j A(1)^-1[k][j] T_s^(j mod M - k) e_j, e = [x_s; x_{s+1}].
  __device__ double coeff(int s, int d, int k) const {
    double c = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int l = j % M;
      const int v = s + j / M;
      c += tabA()[k * N + j] * pwr(s, l - k) * dval(v, l, d);
    }
    return c;
  }

  // Write B x S x D x N coefficients for this trajectory (coalesced).
  __device__ void write_coeffs(double* __restrict__ out) const {
    const int n = S * D * N;
    for (int i = lane; i < n; i += kWave) {
      const int s = i / (D * N);
      const int rem = i % (D * N);
      const int d = rem / N;
      const int k = rem % N;
      out[i] = coeff(s, d, k);
    }
  }

  // Wave-wide sum (all 64 lanes receive it).
  __device__ static double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
    return x;
  }

  // Quadratic form of segment s for dimension d: e^T H_s e.
  __device__ double seg_quad(int s, int d, int a) const {
    // Row a of H_s times e, times e_a.
    const int la = a % M, va = s + a / M;
    double h = 0.0;
#pragma unroll
    for (int b = 0; b < N; ++b) {
      const int lb = b % M, vb = s + b / M;
      h += tabH()[a * N + b] * pwr(s, 1 - 2 * r + la + lb) * dval(vb, lb, d);
    }
    return h * dval(va, la, d);
  }

  // computeCost() = 0.5 * sum_s sum_d e^T H_s e  (== 0.5 sum c^T Q c).
  __device__ double cost() const {
    double acc = 0.0;
    const int n = S * D * N;
    for (int i = lane; i < n; i += kWave) {
      const int s = i / (D * N);
      const int rem = i % (D * N);
      acc += seg_quad(s, rem / N, rem % N);
    }
    return 0.5 * wave_sum(acc);
  }

  // sum_d e_s^T H_s(tau) e_s for segment s at time tau (fixed e): the part of
  // getCostAndGradientDerivative's J_d that depends on T_s.
  __device__ double seg_energy_at(int s, double tau) const {
    double acc = 0.0;
    // tau powers computed on the fly (per lane, small loops).
    const double inv = 1.0 / tau;
    for (int i = lane; i < D * N * N; i += kWave) {
      const int d = i / (N * N);
      const int a = (i / N) % N;
      const int b = i % N;
      const int la = a % M, lb = b % M;
      const int e = 1 - 2 * r + la + lb;
      const double base = e < 0 ? inv : tau;
      const int ne = e < 0 ? -e : e;
      double p = 1.0;
      for (int q = 0; q < ne; ++q) p *= base;
      acc += tabH()[a * N + b] * p * dval(s + a / M, la, d) * dval(s + b / M, lb, d);
    }
    return wave_sum(acc);
  }
};

}  // namespace mtg
