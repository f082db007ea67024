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
  int Dt;          // (S+1)*M*M pinned diagonal blocks -> Schur complements
  int Ot;          // S*M*M     pinned coupling blocks -> W_v = L_v^-1 O_v
  int Bt;          // (S+1)*M*D right-hand sides -> y_v = L_v^-1 r_v
  int Lu;          // (S+1)*M*M unit-lower LDL^T factors
  int dinv;        // (S+1)*M   inverse pivots
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
  l.Dt = o;   o += (S + 1) * M * M;
  l.Ot = o;   o += S * M * M;
  l.Bt = o;   o += (S + 1) * M * D;
  l.Lu = o;   o += (S + 1) * M * M;
  l.dinv = o; o += (S + 1) * M;
  l.aux = o;  o += 4 * S + 8;
  l.ndouble = o;
  l.slot = 0;
  l.nint = (S + 1) * M + 4;
  return l;
}

// 1/d to full FP64 accuracy: v_rcp_f64 seed + two Newton steps (no IEEE
// division sequence on the serial chain).
__device__ inline double rcp64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
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
  // Sets flag()[0] |= 1 if any time is not > 0.
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

  // Phase C (parallel over all vertices): pinned diagonal blocks, pinned
  // coupling blocks and right-hand sides b = -R_pf d_f, so the serial sweep
  // below only does Schur updates and factorisations.
  __device__ void assemble() {
    double* Dt = sm + lay->Dt;
    double* Ot = sm + lay->Ot;
    double* Bt = sm + lay->Bt;
    for (int i = lane; i < (S + 1) * M * M; i += kWave) {
      const int v = i / (M * M);
      const int j = (i / M) % M, k = i % M;
      double val;
      if (fixed_at(v, j) || fixed_at(v, k)) {
        val = (j == k) ? 1.0 : 0.0;
      } else {
        val = 0.0;
        if (v > 0) val += H(v - 1, 1, 1, j, k);
        if (v < S) val += H(v, 0, 0, j, k);
      }
      Dt[i] = val;
    }
    for (int i = lane; i < S * M * M; i += kWave) {
      const int v = i / (M * M);
      const int j = (i / M) % M, k = i % M;
      Ot[i] = (fixed_at(v, j) || fixed_at(v + 1, k)) ? 0.0 : H(v, 0, 1, j, k);
    }
    for (int i = lane; i < (S + 1) * M * D; i += kWave) {
      const int v = i / (M * D);
      const int j = (i / D) % M, d = i % D;
      double val;
      if (fixed_at(v, j)) {
        val = dval(v, j, d);
      } else {
        // dv is zero at free entries, so these sums run over fixed columns.
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
        val = -b;
      }
      Bt[i] = val;
    }
  }

  // Block LDL^T forward sweep over the S+1 vertices, then back substitution.
  // On exit dv holds every vertex derivative (fixed values untouched).
  // Sets flag()[0] |= 2 on a non-positive pivot.
  __device__ void solve() {
    double* Dt = sm + lay->Dt;
    double* Ot = sm + lay->Ot;
    double* Bt = sm + lay->Bt;
    double* Lu = sm + lay->Lu;
    double* dinv = sm + lay->dinv;
    assemble();
    __syncthreads();
    for (int v = 0; v <= S; ++v) {
      double* Sv = Dt + v * M * M;
      double* Rv = Bt + v * M * D;
      if (v > 0) {
        // Schur update with the previous vertex:
        //   S_v = Dt_v - W^T diag(dinv) W,  r_v = b_v - W^T diag(dinv) y.
        const double* Wp = Ot + (v - 1) * M * M;
        const double* Yp = Bt + (v - 1) * M * D;
        const double* dp = dinv + (v - 1) * M;
        if (lane < M * M) {
          const int j = lane / M, k = lane % M;
          double s = Sv[lane];
#pragma unroll
          for (int m = 0; m < M; ++m) s -= Wp[m * M + j] * dp[m] * Wp[m * M + k];
          Sv[lane] = s;
        } else if (lane < M * M + M * D) {
          const int idx = lane - M * M;
          const int j = idx / D, d = idx % D;
          double s = Rv[idx];
#pragma unroll
          for (int m = 0; m < M; ++m) s -= Wp[m * M + j] * dp[m] * Yp[m * D + d];
          Rv[idx] = s;
        }
        __syncthreads();
      }
      // Lane -> column: 0..M-1 the coupling block (absent at v = S), then
      // the D right-hand sides.  Each active lane factors S_v = L Delta L^T
      // in registers (redundantly) and forward-substitutes its column.
      int col;
      if (v < S)
        col = lane < M + D ? lane : -1;
      else
        col = lane < D ? M + lane : -1;
      if (col >= 0) {
        double Lr[M][M];
        double inv[M];
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
          for (int j = 0; j <= i; ++j) Lr[i][j] = Sv[i * M + j];
        bool ok = true;
#pragma unroll
        for (int j = 0; j < M; ++j) {
          // Lr[i][k] for k < j holds L[i][k] * delta_k (scaled column).
          double dj = Lr[j][j];
#pragma unroll
          for (int k = 0; k < j; ++k) dj -= Lr[j][k] * (Lr[j][k] * inv[k]);
          ok = ok && (dj > 0.0);
          inv[j] = rcp64(dj > 0.0 ? dj : 1.0);
#pragma unroll
          for (int i = j + 1; i < M; ++i) {
            double s = Lr[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) s -= Lr[i][k] * (Lr[j][k] * inv[k]);
            Lr[i][j] = s;  // = L[i][j] * delta_j
          }
        }
        if (!ok) atomicOr(&flag()[0], 2);
        // Unit-lower L[i][j] = Lr[i][j] * inv[j].
        double x[M];
        const bool isW = col < M;
#pragma unroll
        for (int i = 0; i < M; ++i) x[i] = isW ? Ot[v * M * M + i * M + col] : Rv[i * D + (col - M)];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          double s = x[i];
#pragma unroll
          for (int k = 0; k < i; ++k) s -= (Lr[i][k] * inv[k]) * x[k];
          x[i] = s;
        }
        if (isW) {
#pragma unroll
          for (int i = 0; i < M; ++i) Ot[v * M * M + i * M + col] = x[i];
        } else {
#pragma unroll
          for (int i = 0; i < M; ++i) Rv[i * D + (col - M)] = x[i];
        }
        if (lane == 0) {
#pragma unroll
          for (int i = 0; i < M; ++i) {
            dinv[v * M + i] = inv[i];
#pragma unroll
            for (int j = 0; j < i; ++j) Lu[v * M * M + i * M + j] = Lr[i][j] * inv[j];
          }
        }
      }
      __syncthreads();
    }
    // Back substitution x_v = L_v^-T diag(dinv_v) (y_v - W_v x_{v+1}), one
    // lane per dimension.
    if (lane < D) {
      const int d = lane;
      double xn[M];
#pragma unroll
      for (int i = 0; i < M; ++i) xn[i] = 0.0;
      for (int v = S; v >= 0; --v) {
        const double* L = Lu + v * M * M;
        const double* Wv = Ot + v * M * M;
        const double* Yv = Bt + v * M * D;
        const double* di = dinv + v * M;
        double t[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          double s = Yv[i * D + d];
          if (v < S) {
#pragma unroll
            for (int k = 0; k < M; ++k) s -= Wv[i * M + k] * xn[k];
          }
          t[i] = s * di[i];
        }
#pragma unroll
        for (int i = M - 1; i >= 0; --i) {
          double s = t[i];
#pragma unroll
          for (int k = i + 1; k < M; ++k) s -= L[k * M + i] * t[k];
          t[i] = s;
        }
#pragma unroll
        for (int i = 0; i < M; ++i) {
          xn[i] = t[i];
          // Pinned entries come back as their value; keep the input bits.
          if (!fixed_at(v, i)) dv()[(v * M + i) * D + d] = t[i];
        }
      }
    }
    __syncthreads();
  }

  // Wave-wide sum (all 64 lanes receive it).
  __device__ static double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
    return x;
  }

  // One pass over (segment, dimension, coefficient k) with e = [x_s; x_{s+1}]:
  //   c_s[d][k] = sum_j A(1)^-1[k][j] T_s^(j mod M - k) e_j   (coefficients,
  //               linear_impl:254-275; written to `out` when non-null)
  //   cost     += e_k (H_s e)_k                               (computeCost,
  //               linear_impl:113-130: 0.5 c^T Q c == 0.5 e^T H e)
  // Returns computeCost() on every lane.
  __device__ double coeffs_and_cost(double* __restrict__ out) const {
    double acc = 0.0;
    const int n = S * D * N;
    for (int i = lane; i < n; i += kWave) {
      const int s = i / (D * N);
      const int rem = i % (D * N);
      const int d = rem / N;
      const int k = rem % N;
      const int lk = k % M;
      double c = 0.0, h = 0.0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const int l = j % M;
        const double e = dval(s + j / M, l, d);
        c += tabA()[k * N + j] * pwr(s, l - k) * e;
        h += tabH()[k * N + j] * pwr(s, 1 - 2 * r + lk + l) * e;
      }
      if (out) out[i] = c;
      acc += h * dval(s + k / M, lk, d);
    }
    return 0.5 * wave_sum(acc);
  }

  __device__ double cost() const { return coeffs_and_cost(nullptr); }

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
