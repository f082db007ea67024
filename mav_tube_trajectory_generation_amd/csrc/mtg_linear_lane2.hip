// mtg_linear_lane2.hip — the batched linear solve of the standard vertex
// pattern with TWO lanes per (trajectory, dimension) (MTG_KERNEL_LANE_PAIR):
// a twisted block Thomas elimination.
//
// linear_lane_kernel (mtg_linear_lane.hip) gives every (trajectory,
// dimension) one lane, which walks the whole block recurrence over the S-1
// intermediate vertices: a launch lasts one lane's chain, and at one
// config-4 shard (B = 8192) the 8192 x 3 lanes fill only 384 of the 1024
// SIMDs.  Here a workgroup of two wavefronts covers 21 trajectories x 3
// dimensions twice: wave 0 eliminates each chain forward over
// v = 1 .. m-1, wave 1 backward over v = S-1 .. m+1 (the same recurrence on
// the reversed chain, whose couplings are the transposed blocks C_(v-1)^T),
// m = S/2.  The waves exchange their Schur terms at m through LDS (one
// barrier), both solve the middle block in the same operation order
// (bit-identical middle values), and each back-substitutes its half
// outward, fused with the coefficients and cost of its half's segments;
// wave 1 hands its cost shares to wave 0 (second barrier), which writes the
// per-trajectory cost, status and the selection partial.
//
// The direction is a template parameter of each wave's code path, so every
// index is compile-time and no lane selects between directions (a one-wave
// variant with the two directions in neighbouring lanes needed ~540 selects
// and 256 + AGPR registers per lane and was 14.3 vs 13.8 us at B = 8192).
//
// Mathematics as linear_lane_kernel / mtg_std_device.h (linear_impl:277-379,
// 254-275, 113-130 with H_s(T) = T^(1-2r) S_T H(1) S_T and
// A_s^-1(T) = D_T^-1 A(1)^-1 S_T); N = 10, r = 4, D = 3, 2 <= S <= 12.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_select_device.h"
#include "mtg_std_device.h"

namespace mtg {
namespace lane2 {

using stdp::AInvTab;
using stdp::rcp64_1;

template <int N, int R>
struct HTab {
  double v[N * N];
  constexpr HTab() : v() {
    for (int i = 0; i < N * N; ++i) v[i] = H1<N, R>::v[i];
  }
};

// Powers T^e, e in [EMIN, EMAX] (the exponents the blocks and the
// coefficients use), by the exact chains of stdp::Solver::powers.
template <int N, int R>
struct Pw {
  static constexpr int M = N / 2;
  static constexpr int EMIN = -(N - 1);
  static constexpr int EMAX = (M - 1) > (2 * M - 1 - 2 * R) ? (M - 1) : (2 * M - 1 - 2 * R);
  static constexpr int NE = EMAX - EMIN + 1;
  double p[NE];
  __device__ double operator[](int e) const { return p[e - EMIN]; }
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

// ldlt_apply that also returns w = D^-1 L^-1 r (the back substitution's
// start), with which G^T S^-1 r = (L^-1 G)^T w.
template <int MF>
__device__ inline void ldlt_apply_w(const double (&l)[MF][MF], const double (&inv)[MF],
                                    const double (&r)[MF], double (&x)[MF], double (&w)[MF]) {
  double y[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    double s = r[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s = fma(-l[i][k], y[k], s);
    y[i] = s;
    w[i] = s * inv[i];
  }
#pragma unroll
  for (int i = MF - 1; i >= 0; --i) {
    double s = w[i];
#pragma unroll
    for (int k = i + 1; k < MF; ++k) s = fma(-l[k][i], x[k], s);
    x[i] = s;
  }
}

// One half of the twisted elimination for one (trajectory, dimension):
// BW = false eliminates forward over v = 1 .. MID-1 (step k: v = 1 + k),
// BW = true backward over v = S-1 .. MID+1 (step k: v = S - 1 - k).  The
// direction is a template parameter: each wave of the kernel runs one
// direction, so every index is compile-time and no lane selects.
template <int N, int R, int D, int S, bool BW>
struct Half {
  static constexpr int M = N / 2, MF = M - 1;
  static constexpr int NF = 2 * M + S - 1;     // fixed derivatives per dimension
  static constexpr int NL = MF * (MF - 1) / 2;
  static constexpr int NT = MF * (MF + 1) / 2;  // lower triangle of a block
  static constexpr int MID = S / 2;             // middle vertex, 1 <= MID <= S-1
  static constexpr int NST = BW ? S - 1 - MID : MID - 1;  // elimination steps
  static constexpr int NSEG = BW ? S - MID : MID;         // segments of this half
  static constexpr int NSTc = NST > 0 ? NST : 1;

  __device__ static constexpr int ex(int a, int b) { return 1 - 2 * R + a % M + b % M; }
  __device__ static constexpr int vert(int k) { return BW ? S - 1 - k : 1 + k; }

  double T[S], x0[M], xS[M], pos[S + 1];
  double Lf[NSTc][NL > 0 ? NL : 1], If[NSTc][MF], z[NSTc][MF];
  // The last step's Y = L^-1 G, D^-1 Y and w = D^-1 L^-1 r: the next
  // step's (or the middle's) Schur terms are G^T S^-1 G = Y^T D^-1 Y and
  // G^T S^-1 r = Y^T w.
  double Yp[MF][MF], DYp[MF][MF], wp[MF];
  double pmin;
  bool bad;

  // Coupling toward the next vertex of the sweep: forward C_v = H01(T_v),
  // backward C_(v-1)^T = H01(T_(v-1))^T; P: powers of that segment's time.
  __device__ static void coupling(const Pw<N, R>& P, double (&G)[MF][MF]) {
    constexpr HTab<N, R> kH{};
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        const int e = ex(i + 1, j + 1);
        G[i][j] = BW ? kH.v[(j + 1) * N + M + i + 1] * P[e] : kH.v[(i + 1) * N + M + j + 1] * P[e];
      }
  }

  // A_v (lower triangle) and b_v for vertex v with left / right segment
  // powers Pl (T_(v-1)) and Pr (T_v) and positions of v-1, v, v+1;
  // left_end / right_end: vertex v-1 / v+1 is the fully fixed start / end.
  __device__ void assemble(const Pw<N, R>& Pl, const Pw<N, R>& Pr, int v, bool left_end,
                           bool right_end, double (&A)[MF][MF], double (&rr)[MF]) const {
    constexpr HTab<N, R> kH{};
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int k = i + 1;
#pragma unroll
      for (int j = 0; j <= i; ++j) {
        const int l = j + 1;
        A[i][j] = fma(kH.v[(M + k) * N + M + l], Pl[ex(k, l)], kH.v[k * N + l] * Pr[ex(k, l)]);
      }
      const double cprev = kH.v[(M + k) * N] * Pl[ex(k, 0)];
      const double cpos = fma(kH.v[(M + k) * N + M], Pl[ex(k, 0)], kH.v[k * N] * Pr[ex(k, 0)]);
      const double cnext = kH.v[k * N + M] * Pr[ex(k, 0)];
      double s = cpos * pos[v];
      s = fma(cprev, pos[v - 1], s);
      s = fma(cnext, pos[v + 1], s);
      if (left_end) {
#pragma unroll
        for (int l = 1; l < M; ++l) s = fma(kH.v[(M + k) * N + l] * Pl[ex(k, l)], x0[l], s);
      }
      if (right_end) {
#pragma unroll
        for (int l = 1; l < M; ++l) s = fma(kH.v[k * N + M + l] * Pr[ex(k, l)], xS[l], s);
      }
      rr[i] = -s;
    }
  }

  // Coefficients of a segment from its vertex derivatives e0 (start), e1
  // (end) at powers P of its time; returns 0.5 c^T Q c (out may be null).
  __device__ static double segment(const double (&e0)[M], const double (&e1)[M],
                                   const Pw<N, R>& P, double* __restrict__ out) {
    constexpr AInvTab<N> kA{};
    double f[N], hh[N];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      f[j] = e0[j] * P[j];
      f[M + j] = e1[j] * P[j];
    }
#pragma unroll
    for (int i = 0; i < M; ++i) hh[i] = kA.v[i * N + i] * f[i];
#pragma unroll
    for (int i = M; i < N; ++i) {
      double t = 0.0;
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (kA.v[i * N + j] != 0.0) t = fma(kA.v[i * N + j], f[j], t);
      hh[i] = t;
    }
    if (out) {
      double2* o2 = reinterpret_cast<double2*>(out);
#pragma unroll
      for (int i = 0; i < N / 2; ++i)
        o2[i] = make_double2(hh[2 * i] * P[-2 * i], hh[2 * i + 1] * P[-2 * i - 1]);
    }
    return stdp::Solver<N, R, D>::q_form(hh) * P[1 - 2 * R];
  }

  __device__ void load(int64_t b, int d, const double* __restrict__ fixed_vals,
                       const double* __restrict__ times) {
    bad = false;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      T[s] = times[b * S + s];
      bad = bad || !(T[s] > 0.0) || !(T[s] < 1e300);
    }
    const double* fb = fixed_vals + (b * D + d) * NF;
#pragma unroll
    for (int k = 0; k < M; ++k) {
      x0[k] = fb[k];
      xS[k] = fb[M + S - 1 + k];
    }
    pos[0] = x0[0];
    pos[S] = xS[0];
#pragma unroll
    for (int v = 1; v < S; ++v) pos[v] = fb[M + v - 1];
  }

  // Elimination over the half.  Kept per step: the LDL^T factors of the
  // Schur complement and z = S^-1 r; the coupling is recomputed in the back
  // pass.  Leaves the last step's Y = L^-1 G, D^-1 Y and w for the middle.
  // Consecutive steps share a segment (forward: step k's right segment is
  // step k+1's left one; backward the reverse), so its powers are formed
  // once.
  __device__ void eliminate() {
    pmin = 1.0;
    Pw<N, R> Ps;  // the shared segment's powers from the previous step
#pragma unroll
    for (int k = 0; k < NST; ++k) {
      const int v = vert(k);
      Pw<N, R> Pl, Pr;
      if (k == 0 || BW) Pl.set(T[v - 1]); else Pl = Ps;
      if (k == 0 || !BW) Pr.set(T[v]); else Pr = Ps;
      double A[MF][MF], rr[MF], G[MF][MF];
      assemble(Pl, Pr, v, !BW && k == 0, BW && k == 0, A, rr);
      coupling(BW ? Pl : Pr, G);
      if (k > 0) {
        // S_v = A_v - Y^T D^-1 Y;  r_v = b_v - Y^T w
#pragma unroll
        for (int i = 0; i < MF; ++i) {
#pragma unroll
          for (int j = 0; j <= i; ++j) {
            double s = A[i][j];
#pragma unroll
            for (int m = 0; m < MF; ++m) s = fma(-Yp[m][i], DYp[m][j], s);
            A[i][j] = s;
          }
          double s = rr[i];
#pragma unroll
          for (int m = 0; m < MF; ++m) s = fma(-Yp[m][i], wp[m], s);
          rr[i] = s;
        }
      }
      Ps = BW ? Pl : Pr;
      double l[MF][MF];
      ldlt<MF>(A, l, If[k], pmin);
      {
        int q = 0;
#pragma unroll
        for (int i = 1; i < MF; ++i)
#pragma unroll
          for (int j = 0; j < i; ++j) Lf[k][q++] = l[i][j];
      }
      ldlt_apply_w<MF>(l, If[k], rr, z[k], wp);
      // Y = L^-1 G (unit lower triangular), D^-1 Y
#pragma unroll
      for (int c = 0; c < MF; ++c) {
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          double s = G[i][c];
#pragma unroll
          for (int m = 0; m < i; ++m) s = fma(-l[i][m], Yp[m][c], s);
          Yp[i][c] = s;
          DYp[i][c] = s * If[k][i];
        }
      }
    }
  }

  // This half's Schur terms at the middle vertex: Y^T D^-1 Y = G^T S^-1 G
  // (lower triangle, row-major) and Y^T w = G^T z.
  __device__ void terms(double (&tm)[NT], double (&rm)[MF]) const {
    int q = 0;
#pragma unroll
    for (int i = 0; i < MF; ++i) {
#pragma unroll
      for (int j = 0; j <= i; ++j) {
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < MF; ++m) s = fma(Yp[m][i], DYp[m][j], s);
        tm[q++] = NST > 0 ? s : 0.0;
      }
      double s = 0.0;
#pragma unroll
      for (int m = 0; m < MF; ++m) s = fma(Yp[m][i], wp[m], s);
      rm[i] = NST > 0 ? s : 0.0;
    }
  }

  // Middle vertex from the forward (tf, rf) and backward (tb, rb) terms,
  // S_mid = (A_mid - T_f) - T_b in that order on both waves (bit-identical
  // middle values), then the back substitution outward fused with the
  // coefficients and cost of the half's segments.  Returns the cost share.
  __device__ double finish(int64_t b, int d, const double (&tf)[NT], const double (&rf)[MF],
                           const double (&tb)[NT], const double (&rb)[MF],
                           double* __restrict__ cb, double* __restrict__ free_vals) {
    double Amid[MF][MF], rmid[MF];
    {
      double tl = T[MID - 1], tr = T[MID];
      asm volatile("" : "+v"(tl), "+v"(tr));
      Pw<N, R> Pl, Pr;
      Pl.set(tl);
      Pr.set(tr);
      assemble(Pl, Pr, MID, MID == 1, MID == S - 1, Amid, rmid);
    }
    {
      int q = 0;
#pragma unroll
      for (int i = 0; i < MF; ++i) {
#pragma unroll
        for (int j = 0; j <= i; ++j, ++q) Amid[i][j] = (Amid[i][j] - tf[q]) - tb[q];
        rmid[i] = (rmid[i] - rf[i]) - rb[i];
      }
    }
    double xm[MF];
    {
      double l[MF][MF], inv[MF];
      ldlt<MF>(Amid, l, inv, pmin);
      ldlt_apply<MF>(l, inv, rmid, xm);
    }
    constexpr int np = (S - 1) * MF;
    if (free_vals && !BW) {
#pragma unroll
      for (int i = 0; i < MF; ++i) free_vals[(b * D + d) * np + (MID - 1) * MF + i] = xm[i];
    }
    // Segment j of the half (j = 0 next to MID): near vertex x_near (x_MID,
    // then the previous far vertex), far vertex = step k = NST-1-j
    // (x_far = z_k - S_k^-1 (G_k x_near)) or the fixed end when j = NST.
    double acc = 0.0;
    double xn[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) xn[i] = xm[i];
#pragma unroll
    for (int j = 0; j < NSEG; ++j) {
      const int k = NST - 1 - j;
      // segment s between vertices s and s+1: forward far = s, near = s+1;
      // backward near = s, far = s+1
      const int s = BW ? MID + j : MID - 1 - j;
      // Recompute the powers: CSE with the elimination's copies would keep
      // them live across the whole kernel.
      double ts = T[s];
      asm volatile("" : "+v"(ts));
      Pw<N, R> P;
      P.set(ts);
      double xf[MF];
      if (k >= 0) {
        // The step's coupling lives on segment s as well: forward C_v with
        // v = s + 1 - 1 ... = the far vertex's right segment (s), backward
        // C_(v-1)^T with v - 1 = s.
        // G x_near with G[i][m] = K[i][m] T^(ex(i+1, m+1)) split as
        // T^(1-2r+i+1) sum_m K[i][m] (T^(m+1) x_m): the constant K as
        // literals, 8 multiplications instead of coupling()'s 16.
        constexpr HTab<N, R> kH{};
        double l[MF][MF];
        int q = 0;
#pragma unroll
        for (int i = 1; i < MF; ++i)
#pragma unroll
          for (int jj = 0; jj < i; ++jj) l[i][jj] = Lf[k >= 0 ? k : 0][q++];
        double gx[MF], w[MF], u[MF];
#pragma unroll
        for (int m = 0; m < MF; ++m) u[m] = xn[m] * P[m + 1];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          double t = 0.0;
#pragma unroll
          for (int m = 0; m < MF; ++m) {
            const double kim = BW ? kH.v[(m + 1) * N + M + i + 1] : kH.v[(i + 1) * N + M + m + 1];
            t = fma(kim, u[m], t);
          }
          gx[i] = t * P[1 - 2 * R + i + 1];
        }
        ldlt_apply<MF>(l, If[k >= 0 ? k : 0], gx, w);
#pragma unroll
        for (int i = 0; i < MF; ++i) xf[i] = z[k >= 0 ? k : 0][i] - w[i];
      } else {
#pragma unroll
        for (int i = 0; i < MF; ++i) xf[i] = BW ? xS[i + 1] : x0[i + 1];
      }
      double e0[M], e1[M];
      e0[0] = pos[s];
      e1[0] = pos[s + 1];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        e0[i + 1] = BW ? xn[i] : xf[i];
        e1[i + 1] = BW ? xf[i] : xn[i];
      }
      acc += segment(e0, e1, P, cb ? cb + (s * D + d) * N : nullptr);
      if (k >= 0 && free_vals) {
        const int vfar = BW ? s + 1 : s;
#pragma unroll
        for (int i = 0; i < MF; ++i) free_vals[(b * D + d) * np + (vfar - 1) * MF + i] = xf[i];
      }
#pragma unroll
      for (int i = 0; i < MF; ++i) xn[i] = xf[i];
    }
    return acc;
  }

  // Bad segment time: NaN coefficients of the half's segments and NaN free
  // values of the half's vertices (forward 1..MID, backward MID+1..S-1, the
  // vertices finish() writes), as every other linear kernel reports them.
  __device__ void write_bad(int64_t b, int d, double* __restrict__ cb,
                            double* __restrict__ free_vals) const {
    if (cb) {
#pragma unroll
      for (int j = 0; j < NSEG; ++j) {
        const int s = BW ? MID + j : MID - 1 - j;
#pragma unroll
        for (int i = 0; i < N; ++i) cb[(s * D + d) * N + i] = NAN;
      }
    }
    if (free_vals) {
      constexpr int np = (S - 1) * MF;
      constexpr int v0 = BW ? MID + 1 : 1, v1 = BW ? S - 1 : MID;
#pragma unroll
      for (int v = v0; v <= v1; ++v)
#pragma unroll
        for (int i = 0; i < MF; ++i) free_vals[(b * D + d) * np + (v - 1) * MF + i] = NAN;
    }
  }
};

// One wave's half of the workgroup: wave 0 forward, wave 1 backward, same
// lane -> (trajectory, dimension) map.  The two exchange their Schur terms
// at the middle vertex through LDS; wave 1 then hands its cost shares and
// status to wave 0, which forms the per-trajectory cost and status.
template <int N, int R, int D, int S, bool BW>
__device__ __attribute__((always_inline)) inline void lane2_half(
    int64_t B, int blk, const double* __restrict__ fixed_vals, const double* __restrict__ times,
    double* __restrict__ coeffs, double* __restrict__ cost, double* __restrict__ free_vals,
    int32_t* __restrict__ status, const SelectArgs& sel, double* xch, double* cxch, int* sxch,
    double* stage) {
  using H = Half<N, R, D, S, BW>;
  constexpr int NT = H::NT, MF = H::MF;
  constexpr int TPW = kWave / D;
  const int lane = threadIdx.x & (kWave - 1);
  const int tl = lane / D, d = lane - tl * D;
  const int64_t b = static_cast<int64_t>(blk) * TPW + tl;
  const bool act = tl < TPW && b < B;
  // Inactive lanes run trajectory 0 with no outputs: every lane reaches the
  // barriers with defined data.
  const int64_t bb = act ? b : 0;
  H h;
  h.load(bb, d, fixed_vals, times);
  h.eliminate();
  double tm[NT], rm[MF];
  h.terms(tm, rm);
  constexpr int W = NT + MF;
  double* mine = xch + (BW ? 1 : 0) * W * kWave;
  double* other = xch + (BW ? 0 : 1) * W * kWave;
#pragma unroll
  for (int q = 0; q < NT; ++q) mine[q * kWave + lane] = tm[q];
#pragma unroll
  for (int i = 0; i < MF; ++i) mine[(NT + i) * kWave + lane] = rm[i];
  __syncthreads();
  double to[NT], ro[MF];
#pragma unroll
  for (int q = 0; q < NT; ++q) to[q] = other[q * kWave + lane];
#pragma unroll
  for (int i = 0; i < MF; ++i) ro[i] = other[(NT + i) * kWave + lane];
  // From kLane2StageMinBatch trajectories the coefficients go to the
  // workgroup's staging area in LDS (the output layout of its TPW
  // trajectories) and leave in one coalesced copy below; under it each lane
  // stores its own (the copy's barrier and latency then cost more than the
  // scattered stores: B = 2048 7.09 -> 7.69 us staged).
  constexpr int PER = S * D * N;
  const bool stg = B >= kLane2StageMinBatch;
  double* cb = !coeffs ? nullptr
               : stg   ? (tl < TPW ? stage + tl * PER : nullptr)
                       : (act ? coeffs + b * PER : nullptr);
  double* fv = act ? free_vals : nullptr;
  double part;
  // A bad time's solve values are not stored (write_bad fills NaN).
  double* fv_ok = h.bad ? nullptr : fv;
  if (BW)
    part = h.finish(bb, d, to, ro, tm, rm, cb, fv_ok);
  else
    part = h.finish(bb, d, tm, rm, to, ro, cb, fv_ok);
  int st = h.bad ? 1 : (h.pmin > 0.0 ? 0 : 2);
  if (h.bad) {
    h.write_bad(bb, d, cb, fv);
    part = NAN;
  }
  if (BW) {
    cxch[lane] = part;
    sxch[lane] = st;
  }
  __syncthreads();
  if (coeffs && stg) {
    // The workgroup's TPW x S x D x N coefficients are one contiguous range
    // of the output: both waves copy it out in 16-byte pieces, consecutive
    // lanes on consecutive addresses (the per-lane stores touch 64 cache
    // lines per instruction: B = 8192 13.0 -> 10.9 us).
    const int64_t b0 = static_cast<int64_t>(blk) * TPW;
    const int nt = B - b0 < TPW ? static_cast<int>(B - b0) : TPW;
    const int nch = nt * (PER / 2);
    const double2* src = reinterpret_cast<const double2*>(stage);
    double2* dst = reinterpret_cast<double2*>(coeffs + b0 * PER);
    const int t = static_cast<int>(threadIdx.x);
    if (nt == TPW) {
      copy_out16<2 * kWave, TPW * (PER / 2)>(src, dst, t);
    } else {
      for (int c = t; c < nch; c += 2 * kWave) dst[c] = src[c];
    }
  }
  if (BW) return;
  part += cxch[lane];
  st = max(st, sxch[lane]);
  double tot = 0.0;
  int stt = 0;
#pragma unroll
  for (int p = 0; p < D; ++p) {
    tot += __shfl(part, tl * D + p);
    stt = max(stt, __shfl(st, tl * D + p));
  }
  if (act && d == 0) {
    if (cost) cost[b] = tot;
    if (status)
      status[b] = stt == 1 ? MTG_TRAJ_BAD_TIME : (stt == 2 ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK);
  }
  if (sel.out) select_partial(sel, tot, act && d == 0 ? b : -1, blk);
}

}  // namespace lane2

// Workgroup = 2 waves (forward, backward) over 21 trajectories x 3
// dimensions; the direction is wave-uniform.  kPrev: the launch carries the
// deferred selection's workgroup (a template parameter so that the solves do
// not wait on the kernel arguments past the preloaded ones; mtg_linear_wave.hip).
template <int N, int R, int D, int S, bool kPrev>
__global__ __launch_bounds__(2 * kWave) void linear_lane2_kernel(
    int64_t B, const double* __restrict__ fixed_vals, const double* __restrict__ times,
    double* __restrict__ coeffs, double* __restrict__ cost, double* __restrict__ free_vals,
    int32_t* __restrict__ status, SelectArgs sel) {
  using H = lane2::Half<N, R, D, S, false>;
  __shared__ double xch[2 * (H::NT + H::MF) * kWave];
  __shared__ double cxch[kWave];
  __shared__ int sxch[kWave];
  // The deferred selection (the previous step's costs, SelectArgs::prev_*)
  // in one extra workgroup, dispatched first (block 0) so that it ends well
  // before the solves' (8192 costs: four rounds of loads by 128 threads).
  const int blk = static_cast<int>(blockIdx.x) - (kPrev ? 1 : 0);
  if (kPrev && blk < 0) {
    select_reduce_block<2 * kWave>(sel.prev_cost, sel.prev_count, sel.prev_start, sel.rank,
                                   sel.prev_out, cxch, reinterpret_cast<int64_t*>(xch));
    return;
  }
  // The staging area is static LDS on every launch (it is not used below
  // kLane2StageMinBatch): 50 KB at S = 10, 75 KB at S = 12 with the exchange
  // buffers.  Above 64 KB per workgroup this builds for gfx950 (160 KB LDS
  // per CU) only, the one target of this library; two workgroups per CU is
  // the occupancy one wave per SIMD allows anyway.
  static_assert(sizeof(double) * ((kWave / D) * S * D * N + 2 * (H::NT + H::MF) * kWave +
                                  kWave) + sizeof(int) * kWave <= 160 * 1024 / 2,
                "lane-pair LDS must leave room for two workgroups per gfx950 CU");
  __shared__ __attribute__((aligned(16))) double stage[(kWave / D) * S * D * N];
  if (threadIdx.x < kWave)
    lane2::lane2_half<N, R, D, S, false>(B, blk, fixed_vals, times, coeffs, cost, free_vals,
                                         status, sel, xch, cxch, sxch, stage);
  else
    lane2::lane2_half<N, R, D, S, true>(B, blk, fixed_vals, times, coeffs, cost, free_vals,
                                        status, sel, xch, cxch, sxch, stage);
}

namespace {

template <int N, int R, int D, int S>
hipError_t launch_lane2(int64_t B, const double* df, const double* times, double* coeffs,
                        double* cost, double* free_vals, int32_t* status, hipStream_t st,
                        const SelectArgs& sel) {
  constexpr int TPW = kWave / D;
  const int64_t blocks = (B + TPW - 1) / TPW;
  if (sel.prev_out)
    hipLaunchKernelGGL((linear_lane2_kernel<N, R, D, S, true>), dim3(static_cast<unsigned>(blocks + 1)),
                       dim3(2 * kWave), 0, st, B, df, times, coeffs, cost, free_vals, status, sel);
  else
    hipLaunchKernelGGL((linear_lane2_kernel<N, R, D, S, false>), dim3(static_cast<unsigned>(blocks)),
                       dim3(2 * kWave), 0, st, B, df, times, coeffs, cost, free_vals, status, sel);
  return hipGetLastError();
}

}  // namespace

int64_t lane2_blocks(int64_t B) {
  constexpr int TPW = kWave / 3;
  return (B + TPW - 1) / TPW;
}

hipError_t launch_linear_solve_lane2(const PlanDev& pl, int64_t B, const double* df,
                                     const double* times, double* coeffs, double* cost,
                                     double* free_vals, int32_t* status, hipStream_t st,
                                     const SelectArgs& sel) {
  if (!has_linear_lane(pl)) return hipErrorInvalidValue;
  switch (pl.S) {
#define MTG_LANE2_S(SS) \
    case SS: return launch_lane2<10, 4, 3, SS>(B, df, times, coeffs, cost, free_vals, status, st, sel);
    MTG_LANE2_S(2) MTG_LANE2_S(3) MTG_LANE2_S(4) MTG_LANE2_S(5) MTG_LANE2_S(6) MTG_LANE2_S(7)
    MTG_LANE2_S(8) MTG_LANE2_S(9) MTG_LANE2_S(10) MTG_LANE2_S(11) MTG_LANE2_S(12)
#undef MTG_LANE2_S
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
