// mtg_linear_lane.hip — the batched linear solve for large batches of the
// standard vertex pattern: one (trajectory, dimension) per lane, SIMT over
// the batch (MTG_KERNEL_LANE).
//
// Same mathematics as linear_std_kernel (mtg_std_device.h: updateSegmentTimes
// + solveLinear + computeCost, linear_impl:277-379, 113-130, with the time
// scaling H_s(T) = T^(1-2r) S_T H(1) S_T and A_s^-1(T) = D_T^-1 A(1)^-1 S_T),
// organised for throughput instead of latency.  linear_std_kernel spreads one
// trajectory over a wavefront, so its block recurrences run on 14 to 36 of
// 64 lanes (43 % VALU lane utilisation measured, profiles/r02_sq_*.json);
// here every lane owns a whole problem and nearly every FP64 instruction does
// 63 lanes of useful work.  The price is latency: one lane walks the whole
// recurrence, so a launch takes one lane's instruction stream (~12 us)
// however small the batch.  AUTO picks this kernel from kLaneMinBatch
// trajectories (measured crossover).
//
// Per lane (S, N, D, r compile-time, so every array below lives in registers):
//   forward block elimination over the intermediate vertices v = 1 .. S-1
//   (block Thomas on the MF x MF blocks, MF = M-1 free derivatives per
//   vertex): assemble A_v, C_v, b_v from H(1) (exact compile-time constants,
//   tools/gen_tables.py) and the powers of the two adjacent segment times;
//   S_v = A_v - C_(v-1)^T Z_(v-1), r_v = b_v - C_(v-1)^T z_(v-1); LDL^T of
//   S_v; keep its factors and z_v = S_v^-1 r_v;
//   back substitution x_(S-1) = z_(S-1), x_v = z_v - S_v^-1 (C_v x_(v+1))
//   with C_v recomputed, fused with the coefficients and cost of segment v
//   (vertices v, v+1) as soon as both of its vertices are known
//   (computeCost's 0.5 c^T Q c in the Q-form of mtg_std_device.h, A(1)^-1
//   and the weights as instruction constants).
// ND = dimensions per lane.  The D lanes of a trajectory each repeat the
// shared factorisation and solve their own dimension (ND = 1): 418 registers
// at S = 10, no scratch, one wave per SIMD.  ND = D (one trajectory per lane)
// would do a third of the factorisation work but needs ~3x the per-vertex
// storage and spills to scratch (2.5 KB per lane at S = 10; measured 3.3x
// slower), so only ND = 1 is instantiated.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_select_device.h"
#include "mtg_std_device.h"

namespace mtg {
namespace lanek {

using stdp::AInvTab;
using stdp::CostW;
using stdp::rcp64_1;

template <int N, int R>
struct Pw {
  static constexpr int M = N / 2;
  static constexpr int EMIN = -(N - 1);
  static constexpr int EMAX = (M - 1) > (2 * M - 1 - 2 * R) ? (M - 1) : (2 * M - 1 - 2 * R);
  static constexpr int NE = EMAX - EMIN + 1;
  double p[NE];
  __device__ double operator[](int e) const { return p[e - EMIN]; }
  // Exact multiplication chains, as stdp::Solver::powers.
  __device__ void set(double t) {
    const double inv = rcp64(t);
    p[-EMIN] = 1.0;
    double up = 1.0, dn = 1.0;
#pragma unroll
    for (int e = 1; e <= (EMAX > -EMIN ? EMAX : -EMIN); ++e) {
      up *= t;
      dn *= inv;
      if (e <= EMAX) p[e - EMIN] = up;
      if (-e >= EMIN) p[-e - EMIN] = dn;
    }
  }
};

// LDL^T of a symmetric MF x MF block (lower triangle of A): unit-lower l,
// reciprocal pivots inv; pmin <- min(pmin, pivots).
template <int MF>
__device__ inline void ldlt(const double (&A)[MF][MF], double (&l)[MF][MF], double (&inv)[MF],
                            double& pmin) {
  double Lr[MF][MF];
#pragma unroll
  for (int j = 0; j < MF; ++j) {
    double dj = A[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) dj = fma(-Lr[j][k], l[j][k], dj);
    pmin = fmin(pmin, dj);
    inv[j] = rcp64_1(dj);
#pragma unroll
    for (int i = j + 1; i < MF; ++i) {
      double s = A[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) s = fma(-Lr[i][k], l[j][k], s);
      Lr[i][j] = s;
      l[i][j] = s * inv[j];
    }
  }
}

template <int MF>
__device__ inline void ldlt_apply(const double (&l)[MF][MF], const double (&inv)[MF],
                                  const double (&r)[MF], double (&x)[MF]) {
  double y[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    double s = r[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s = fma(-l[i][k], y[k], s);
    y[i] = s;
  }
#pragma unroll
  for (int i = MF - 1; i >= 0; --i) {
    double s = y[i] * inv[i];
#pragma unroll
    for (int k = i + 1; k < MF; ++k) s = fma(-l[k][i], x[k], s);
    x[i] = s;
  }
}

// H(1) as a local compile-time object (folds into instruction constants,
// which the compiler rematerialises instead of keeping them live).
template <int N, int R>
struct HTab {
  double v[N * N];
  constexpr HTab() : v() {
    for (int i = 0; i < N * N; ++i) v[i] = H1<N, R>::v[i];
  }
};

template <int N, int R, int D, int S, int ND>
struct LaneSolve {
  static constexpr int M = N / 2, MF = M - 1;
  static constexpr int NF = 2 * M + S - 1;  // fixed derivatives per dimension
  static constexpr int NL = MF * (MF - 1) / 2;

  __device__ static constexpr int ex(int a, int b) { return 1 - 2 * R + a % M + b % M; }

  // C_v = H_v(derivatives 1..M-1 of vertex v, of vertex v+1) at powers P of T_v.
  __device__ static void coupling(const Pw<N, R>& P, double (&C)[MF][MF]) {
    constexpr HTab<N, R> kH{};
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < MF; ++j) C[i][j] = kH.v[(i + 1) * N + M + j + 1] * P[ex(i + 1, j + 1)];
  }

  // Coefficients of segment s from its two vertices' derivatives e0, e1
  // (dimension-local) and the powers of T_s; returns 0.5 c^T Q c.
  __device__ static double segment(const double (&e0)[M], const double (&e1)[M],
                                   const Pw<N, R>& P, double* __restrict__ out) {
    constexpr AInvTab<N> kA{};
    double f[N], h[N];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      f[j] = e0[j] * P[j];
      f[M + j] = e1[j] * P[j];
    }
#pragma unroll
    for (int i = 0; i < M; ++i) h[i] = kA.v[i * N + i] * f[i];
#pragma unroll
    for (int i = M; i < N; ++i) {
      double t = 0.0;
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (kA.v[i * N + j] != 0.0) t = fma(kA.v[i * N + j], f[j], t);
      h[i] = t;
    }
    if (out) {
      double2* o2 = reinterpret_cast<double2*>(out);
#pragma unroll
      for (int i = 0; i < N / 2; ++i)
        o2[i] = make_double2(h[2 * i] * P[-2 * i], h[2 * i + 1] * P[-2 * i - 1]);
    }
    return stdp::Solver<N, R, D>::q_form(h) * P[1 - 2 * R];
  }

  // Returns 0 ok, 1 bad time, 2 not SPD; *cost_part = this lane's share.
  __device__ static int run(int64_t b, int d0, const double* __restrict__ fixed_vals,
                            const double* __restrict__ times, double* __restrict__ coeffs,
                            double* __restrict__ free_vals, double* cost_part) {
    constexpr HTab<N, R> kH{};
    double T[S];
    bool bad = false;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      T[s] = times[b * S + s];
      bad = bad || !(T[s] > 0.0) || !(T[s] < 1e300);
    }
    // Fixed values of this lane's dimensions (standard order of
    // linear_impl:171-252: vertex 0 derivatives, intermediate positions,
    // vertex S derivatives).
    double x0[ND][M], xS[ND][M], pos[ND][S + 1];
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) {
      const double* fb = fixed_vals + (b * D + d0 + dd) * NF;
#pragma unroll
      for (int k = 0; k < M; ++k) {
        x0[dd][k] = fb[k];
        xS[dd][k] = fb[M + S - 1 + k];
      }
      pos[dd][0] = x0[dd][0];
      pos[dd][S] = xS[dd][0];
#pragma unroll
      for (int v = 1; v < S; ++v) pos[dd][v] = fb[M + v - 1];
    }
    double* cb = coeffs + b * S * D * N;
    if (bad) {
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int dd = 0; dd < ND; ++dd)
#pragma unroll
          for (int i = 0; i < N; ++i) cb[(s * D + d0 + dd) * N + i] = NAN;
      if (free_vals) {
        constexpr int np = (S - 1) * MF;
#pragma unroll
        for (int dd = 0; dd < ND; ++dd)
#pragma unroll
          for (int i = 0; i < np; ++i) free_vals[(b * D + d0 + dd) * np + i] = NAN;
      }
      *cost_part = NAN;
      return 1;
    }

    // ---- forward elimination ------------------------------------------------
    // Kept for the back substitution, per vertex v = 1 .. S-1: the LDL^T
    // factors of S_v (unit-lower part, reciprocal pivots) and z_v; C_v is
    // recomputed from T_v there.
    double Lf[S - 1][NL > 0 ? NL : 1], If[S - 1][MF];
    double z[S - 1][ND][MF];
    double Zp[MF][MF], Cp[MF][MF];  // Z_(v-1) = S_(v-1)^-1 C_(v-1), C_(v-1)
    double pmin = 1.0;
    Pw<N, R> Pl, Pr;
    Pr.set(T[0]);
#pragma unroll
    for (int v = 1; v < S; ++v) {
      Pl = Pr;
      Pr.set(T[v]);
      double A[MF][MF], C[MF][MF], rr[ND][MF];
      coupling(Pr, C);
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const int k = i + 1;
#pragma unroll
        for (int j = 0; j <= i; ++j) {
          const int l = j + 1;
          A[i][j] = fma(kH.v[(M + k) * N + M + l], Pl[ex(k, l)], kH.v[k * N + l] * Pr[ex(k, l)]);
        }
        // b_v row i: -(R_pf d_f) restricted to the row (stdp::Solver::assemble_row).
        const double cprev = kH.v[(M + k) * N] * Pl[ex(k, 0)];
        const double cpos = fma(kH.v[(M + k) * N + M], Pl[ex(k, 0)], kH.v[k * N] * Pr[ex(k, 0)]);
        const double cnext = kH.v[k * N + M] * Pr[ex(k, 0)];
#pragma unroll
        for (int dd = 0; dd < ND; ++dd) {
          double s = cpos * pos[dd][v];
          s = fma(cprev, pos[dd][v - 1], s);
          s = fma(cnext, pos[dd][v + 1], s);
          if (v == 1) {
#pragma unroll
            for (int l = 1; l < M; ++l)
              s = fma(kH.v[(M + k) * N + l] * Pl[ex(k, l)], x0[dd][l], s);
          }
          if (v == S - 1) {
#pragma unroll
            for (int l = 1; l < M; ++l)
              s = fma(kH.v[k * N + M + l] * Pr[ex(k, l)], xS[dd][l], s);
          }
          rr[dd][i] = -s;
        }
      }
      if (v > 1) {
        // S_v = A_v - C_(v-1)^T Z_(v-1);  r_v = b_v - C_(v-1)^T z_(v-1)
#pragma unroll
        for (int i = 0; i < MF; ++i) {
#pragma unroll
          for (int j = 0; j <= i; ++j) {
            double s = A[i][j];
#pragma unroll
            for (int m = 0; m < MF; ++m) s = fma(-Cp[m][i], Zp[m][j], s);
            A[i][j] = s;
          }
#pragma unroll
          for (int dd = 0; dd < ND; ++dd) {
            double s = rr[dd][i];
#pragma unroll
            for (int m = 0; m < MF; ++m) s = fma(-Cp[m][i], z[v - 2][dd][m], s);
            rr[dd][i] = s;
          }
        }
      }
      double l[MF][MF];
      ldlt<MF>(A, l, If[v - 1], pmin);
      {
        int q = 0;
#pragma unroll
        for (int i = 1; i < MF; ++i)
#pragma unroll
          for (int j = 0; j < i; ++j) Lf[v - 1][q++] = l[i][j];
      }
#pragma unroll
      for (int dd = 0; dd < ND; ++dd) ldlt_apply<MF>(l, If[v - 1], rr[dd], z[v - 1][dd]);
      if (v < S - 1) {
#pragma unroll
        for (int c = 0; c < MF; ++c) {
          double col[MF], xc[MF];
#pragma unroll
          for (int i = 0; i < MF; ++i) col[i] = C[i][c];
          ldlt_apply<MF>(l, If[v - 1], col, xc);
#pragma unroll
          for (int i = 0; i < MF; ++i) Zp[i][c] = xc[i];
        }
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int j = 0; j < MF; ++j) Cp[i][j] = C[i][j];
      }
    }

    // ---- back substitution fused with coefficients and cost ----------------
    //   x_(S-1) = z_(S-1);  x_v = z_v - S_v^-1 (C_v x_(v+1));  then segment v
    //   (vertices v, v+1) as soon as both are known.
    double acc = 0.0;
    double xn[ND][MF];  // x_(v+1)
    const int np = (S - 1) * MF;
#pragma unroll
    for (int v = S - 1; v >= 0; --v) {
      // Recompute the powers (and C_v below) instead of keeping the forward
      // sweep's copies live: an empty asm hides that t is T[v], so the
      // compiler cannot merge the two computations (which would hold ~60
      // registers per segment through the whole sweep).
      double t = T[v];
      asm volatile("" : "+v"(t));
      Pw<N, R> P;
      P.set(t);
      double C[MF][MF], l[MF][MF];
      if (v >= 1 && v < S - 1) {
        coupling(P, C);
        int q = 0;
#pragma unroll
        for (int i = 1; i < MF; ++i)
#pragma unroll
          for (int j = 0; j < i; ++j) l[i][j] = Lf[v - 1][q++];
      }
#pragma unroll
      for (int dd = 0; dd < ND; ++dd) {
        double xv[MF];
        if (v >= 1) {
          if (v < S - 1) {
            double cx[MF], w[MF];
#pragma unroll
            for (int i = 0; i < MF; ++i) {
              double s = 0.0;
#pragma unroll
              for (int j = 0; j < MF; ++j) s = fma(C[i][j], xn[dd][j], s);
              cx[i] = s;
            }
            ldlt_apply<MF>(l, If[v - 1], cx, w);
#pragma unroll
            for (int i = 0; i < MF; ++i) xv[i] = z[v - 1][dd][i] - w[i];
          } else {
#pragma unroll
            for (int i = 0; i < MF; ++i) xv[i] = z[v - 1][dd][i];
          }
          if (free_vals) {
#pragma unroll
            for (int i = 0; i < MF; ++i)
              free_vals[(b * D + d0 + dd) * np + (v - 1) * MF + i] = xv[i];
          }
        }
        double e0[M], e1[M];
        e0[0] = pos[dd][v];
        e1[0] = pos[dd][v + 1];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          e0[i + 1] = v == 0 ? x0[dd][i + 1] : xv[i];
          e1[i + 1] = v == S - 1 ? xS[dd][i + 1] : xn[dd][i];
        }
        acc += segment(e0, e1, P, cb + (v * D + d0 + dd) * N);
        if (v >= 1) {
#pragma unroll
          for (int i = 0; i < MF; ++i) xn[dd][i] = xv[i];
        }
      }
    }
    *cost_part = acc;
    return pmin > 0.0 ? 0 : 2;
  }
};

}  // namespace lanek

template <int N, int R, int D, int S, int ND>
__global__ __launch_bounds__(kWave) void linear_lane_kernel(
    int64_t B, const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    const double* __restrict__ times, double* __restrict__ coeffs, double* __restrict__ cost,
    double* __restrict__ free_vals, int32_t* __restrict__ status, SelectArgs sel) {
  constexpr int LPT = D / ND;          // lanes per trajectory
  constexpr int TPW = kWave / LPT;     // trajectories per wavefront
  const int lane = threadIdx.x;
  const int tl = lane / LPT, part = lane - tl * LPT;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * TPW + tl;
  const bool act = tl < TPW && b < B;
  double cpart = 0.0;
  int st = 0;
  if (act)
    st = lanek::LaneSolve<N, R, D, S, ND>::run(b, part * ND, fixed_vals, times, coeffs,
                                               free_vals, &cpart);
  if constexpr (LPT > 1) {
    // Sum the per-dimension shares of the trajectory's lanes.
    double tot = 0.0;
#pragma unroll
    for (int p = 0; p < LPT; ++p) tot += __shfl(cpart, tl * LPT + p);
    cpart = tot;
  }
  if (act && part == 0) {
    if (cost) cost[b] = cpart;
    if (status) status[b] = st == 1 ? MTG_TRAJ_BAD_TIME : (st == 2 ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK);
  }
  // Fused selection: the wave's best trajectory is this workgroup's partial.
  if (sel.out)
    select_partial(sel, cpart, act && part == 0 ? b : -1, blockIdx.x);
}

namespace {

template <int N, int R, int D, int S, int ND>
hipError_t launch_lane(int64_t B, const double* tab, const double* df, const double* times,
                       double* coeffs, double* cost, double* free_vals, int32_t* status,
                       hipStream_t st, const SelectArgs& sel) {
  constexpr int TPW = kWave / (D / ND);
  const int64_t blocks = (B + TPW - 1) / TPW;
  hipLaunchKernelGGL((linear_lane_kernel<N, R, D, S, ND>), dim3(static_cast<unsigned>(blocks)),
                     dim3(kWave), 0, st, B, tab, df, times, coeffs, cost, free_vals, status, sel);
  return hipGetLastError();
}

template <int ND>
hipError_t launch_lane_s(int S, int64_t B, const double* tab, const double* df,
                         const double* times, double* coeffs, double* cost, double* free_vals,
                         int32_t* status, hipStream_t st, const SelectArgs& sel) {
  switch (S) {
#define MTG_LANE_S(SS) \
    case SS: return launch_lane<10, 4, 3, SS, ND>(B, tab, df, times, coeffs, cost, free_vals, status, st, sel);
    MTG_LANE_S(2) MTG_LANE_S(3) MTG_LANE_S(4) MTG_LANE_S(5) MTG_LANE_S(6) MTG_LANE_S(7)
    MTG_LANE_S(8) MTG_LANE_S(9) MTG_LANE_S(10) MTG_LANE_S(11) MTG_LANE_S(12)
#undef MTG_LANE_S
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool has_linear_lane(const PlanDev& pl) {
  return use_std_kernel(pl) && pl.N == 10 && pl.r == 4 && pl.D == 3 && pl.S >= 2 &&
         pl.S <= kMaxLaneS;
}

hipError_t launch_linear_solve_lane(const PlanDev& pl, int64_t B, const double* df,
                                    const double* times, double* coeffs, double* cost,
                                    double* free_vals, int32_t* status, hipStream_t st,
                                    const SelectArgs& sel) {
  if (!has_linear_lane(pl)) return hipErrorInvalidValue;
  return launch_lane_s<1>(pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st, sel);
}

int64_t lane_blocks(int64_t B) {
  constexpr int TPW = kWave / 3;  // N = 10, D = 3, one dimension per lane
  return (B + TPW - 1) / TPW;
}

}  // namespace mtg
