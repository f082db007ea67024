// mtg_linear_lane2.hip — the batched linear solve of the standard vertex
// pattern with TWO lanes per (trajectory, dimension) (MTG_KERNEL_LANE_PAIR):
// a twisted block Thomas elimination.
//
// linear_lane_kernel (mtg_linear_lane.hip) gives every (trajectory,
// dimension) one lane, which walks the whole block recurrence over the S-1
// intermediate vertices: a launch lasts one lane's chain (~12 us), and at
// one config-4 shard (B = 8192) the 8192 x 3 lanes fill only 384 of the
// 1024 SIMDs.  Here the pair of lanes (lane ^ 1) splits the chain at the
// middle vertex m = S/2: the even lane eliminates forward over
// v = 1 .. m-1, the odd lane backward over v = S-1 .. m+1 (the same
// recurrence on the reversed chain, whose couplings are the transposed
// blocks C_(v-1)^T), so each lane walks half the vertices.  The two lanes
// then exchange their Schur terms at m through DPP (quad_perm [1,0,3,2]),
// both solve the middle block, and each back-substitutes its half outward,
// fused with the coefficients and cost of its half's segments.  The chain
// halves and twice as many waves cover the chip.
//
// Both lanes run ONE instruction stream: every difference between the two
// directions is data (the lane's segment times, neighbour positions and
// coupling orientation are chosen by selects between compile-time-indexed
// registers), so there is no divergence.
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

// The value of the partner lane (lane ^ 1) by DPP quad_perm [1, 0, 3, 2].
__device__ inline double partner(double x) {
  const long long u = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(u), 0xB1, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(u >> 32), 0xB1, 0xf, 0xf, false);
  return stdp::join64(lo, hi);
}

template <int N, int R, int D, int S>
struct PairSolve {
  static constexpr int M = N / 2, MF = M - 1;
  static constexpr int NF = 2 * M + S - 1;     // fixed derivatives per dimension
  static constexpr int NL = MF * (MF - 1) / 2;
  static constexpr int MID = S / 2;             // middle vertex, 1 <= MID <= S-1
  static constexpr int NFW = MID - 1;           // forward steps (v = 1 .. MID-1)
  static constexpr int NBW = S - 1 - MID;       // backward steps (v = S-1 .. MID+1)
  static constexpr int NST = NFW > NBW ? NFW : NBW;
  static constexpr int NSEG = (MID > S - MID ? MID : S - MID);  // segments per lane, at most

  __device__ static constexpr int ex(int a, int b) { return 1 - 2 * R + a % M + b % M; }

  // The lane's step k: its vertex v (forward 1+k, backward S-1-k) and the
  // compile-time indices of the neighbouring data, selected by h.
  // Coupling toward the next vertex of the sweep: forward C_v = H01(T_v),
  // backward C_(v-1)^T = H01(T_(v-1))^T.
  __device__ static void coupling(bool bw, const Pw<N, R>& Pl, const Pw<N, R>& Pr,
                                  double (&G)[MF][MF]) {
    constexpr HTab<N, R> kH{};
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        const int e = ex(i + 1, j + 1);
        const double f = kH.v[(i + 1) * N + M + j + 1] * Pr[e];
        const double b = kH.v[(j + 1) * N + M + i + 1] * Pl[e];
        G[i][j] = bw ? b : f;
      }
  }

  // A_v (lower triangle) and b_v for vertex v with left / right segment
  // powers Pl (T_(v-1)) and Pr (T_v) and positions of v-1, v, v+1;
  // left_end / right_end: vertex v-1 / v+1 is the fully fixed start / end.
  __device__ static void assemble(const Pw<N, R>& Pl, const Pw<N, R>& Pr, double pm, double p0,
                                  double pp, bool left_end, bool right_end,
                                  const double (&x0)[M], const double (&xS)[M],
                                  double (&A)[MF][MF], double (&rr)[MF]) {
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
      double s = cpos * p0;
      s = fma(cprev, pm, s);
      s = fma(cnext, pp, s);
      double el = 0.0, er = 0.0;
#pragma unroll
      for (int l = 1; l < M; ++l) {
        el = fma(kH.v[(M + k) * N + l] * Pl[ex(k, l)], x0[l], el);
        er = fma(kH.v[k * N + M + l] * Pr[ex(k, l)], xS[l], er);
      }
      s += (left_end ? el : 0.0) + (right_end ? er : 0.0);
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

  // h = 0 forward lane, 1 backward lane of (trajectory b, dimension d).
  // Returns 0 ok, 1 bad time, 2 not SPD; *cost_part = this lane's share.
  __device__ static int run(int64_t b, int d, int h, const double* __restrict__ fixed_vals,
                            const double* __restrict__ times, double* __restrict__ coeffs,
                            double* __restrict__ free_vals, double* cost_part) {
    const bool bw = h != 0;
    double T[S];
    bool bad = false;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      T[s] = times[b * S + s];
      bad = bad || !(T[s] > 0.0) || !(T[s] < 1e300);
    }
    double x0[M], xS[M], pos[S + 1];
    {
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
    double* cb = coeffs ? coeffs + b * S * D * N : nullptr;
    if (bad) {
      if (!cb) {
        *cost_part = NAN;
        return 1;
      }
      // Each lane of the pair writes half of the dimension's coefficients.
#pragma unroll
      for (int s = 0; s < S; ++s)
        if ((s < MID) != bw) {
#pragma unroll
          for (int i = 0; i < N; ++i) cb[(s * D + d) * N + i] = NAN;
        }
      *cost_part = NAN;
      return 1;
    }

    // ---- elimination over the lane's half ----------------------------------
    // Step k: vertex v = 1 + k (forward) or S - 1 - k (backward); the left
    // segment of v is v-1, the right v.  Kept per step: LDL^T factors of
    // the Schur complement and z = S^-1 r; G is recomputed in the back pass.
    double Lf[NST > 0 ? NST : 1][NL > 0 ? NL : 1], If[NST > 0 ? NST : 1][MF];
    double z[NST > 0 ? NST : 1][MF];
    double Zp[MF][MF], Gp[MF][MF], zp[MF];  // previous step's Z, G, z
    double pmin = 1.0;
#pragma unroll
    for (int k = 0; k < NST; ++k) {
      const bool act = bw ? (k < NBW) : (k < NFW);
      // Compile-time indices of the forward (f) and backward (b) vertex.
      const int vf = 1 + k, vb = S - 1 - k;
      const double tl = bw ? T[vb - 1 >= 0 ? vb - 1 : 0] : T[vf - 1];
      const double tr = bw ? T[vb < S ? vb : S - 1] : T[vf < S ? vf : S - 1];
      Pw<N, R> Pl, Pr;
      Pl.set(tl);
      Pr.set(tr);
      const double pm = bw ? pos[vb - 1 >= 0 ? vb - 1 : 0] : pos[vf - 1];
      const double p0 = bw ? pos[vb >= 0 ? vb : 0] : pos[vf <= S ? vf : S];
      const double pp = bw ? pos[vb + 1 <= S ? vb + 1 : S] : pos[vf + 1 <= S ? vf + 1 : S];
      double A[MF][MF], rr[MF], G[MF][MF];
      assemble(Pl, Pr, pm, p0, pp, !bw && k == 0, bw && k == 0, x0, xS, A, rr);
      coupling(bw, Pl, Pr, G);
      if (k > 0) {
        // S_v = A_v - Gp^T Zp;  r_v = b_v - Gp^T z_prev
#pragma unroll
        for (int i = 0; i < MF; ++i) {
#pragma unroll
          for (int j = 0; j <= i; ++j) {
            double s = A[i][j];
#pragma unroll
            for (int m = 0; m < MF; ++m) s = fma(-Gp[m][i], Zp[m][j], s);
            A[i][j] = s;
          }
          double s = rr[i];
#pragma unroll
          for (int m = 0; m < MF; ++m) s = fma(-Gp[m][i], zp[m], s);
          rr[i] = s;
        }
      }
      double l[MF][MF];
      double pk = 1.0;
      ldlt<MF>(A, l, If[k], pk);
      if (act) pmin = fmin(pmin, pk);
      {
        int q = 0;
#pragma unroll
        for (int i = 1; i < MF; ++i)
#pragma unroll
          for (int j = 0; j < i; ++j) Lf[k][q++] = l[i][j];
      }
      ldlt_apply<MF>(l, If[k], rr, z[k]);
#pragma unroll
      for (int c = 0; c < MF; ++c) {
        double col[MF], xc[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i) col[i] = G[i][c];
        ldlt_apply<MF>(l, If[k], col, xc);
        // A lane past its last step (the shorter half of an odd S) keeps the
        // state of its last real step for the middle vertex.
#pragma unroll
        for (int i = 0; i < MF; ++i) Zp[i][c] = act ? xc[i] : Zp[i][c];
      }
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        zp[i] = act ? z[k][i] : zp[i];
#pragma unroll
        for (int j = 0; j < MF; ++j) Gp[i][j] = act ? G[i][j] : Gp[i][j];
      }
    }

    // ---- middle vertex -------------------------------------------------------
    // Each lane's Schur term Gp^T Zp (and Gp^T z) at MID from its last step;
    // the partner's arrives by DPP.  S_mid = A_mid - term_f - term_b.
    const int nsteps = bw ? NBW : NFW;
    double Tm[MF][MF], Rm[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
#pragma unroll
      for (int j = 0; j <= i; ++j) {
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < MF; ++m) s = fma(Gp[m][i], Zp[m][j], s);
        Tm[i][j] = nsteps > 0 ? s : 0.0;
      }
      double s = 0.0;
#pragma unroll
      for (int m = 0; m < MF; ++m) s = fma(Gp[m][i], zp[m], s);
      Rm[i] = nsteps > 0 ? s : 0.0;
    }
    double Amid[MF][MF], rmid[MF];
    {
      Pw<N, R> Pl, Pr;
      Pl.set(T[MID - 1]);
      Pr.set(T[MID]);
      assemble(Pl, Pr, pos[MID - 1], pos[MID], pos[MID + 1], MID == 1, MID == S - 1, x0, xS,
               Amid, rmid);
    }
#pragma unroll
    for (int i = 0; i < MF; ++i) {
#pragma unroll
      for (int j = 0; j <= i; ++j) Amid[i][j] = (Amid[i][j] - Tm[i][j]) - partner(Tm[i][j]);
      rmid[i] = (rmid[i] - Rm[i]) - partner(Rm[i]);
    }
    // Both lanes form the same sum, in the same order, from the forward
    // lane's point of view: make them bit-identical by taking the forward
    // lane's result.
#pragma unroll
    for (int i = 0; i < MF; ++i) {
#pragma unroll
      for (int j = 0; j <= i; ++j) {
        const double o = partner(Amid[i][j]);
        Amid[i][j] = bw ? o : Amid[i][j];
      }
      const double o = partner(rmid[i]);
      rmid[i] = bw ? o : rmid[i];
    }
    double xm[MF];
    {
      double l[MF][MF], inv[MF];
      ldlt<MF>(Amid, l, inv, pmin);
      ldlt_apply<MF>(l, inv, rmid, xm);
    }
    const int np = (S - 1) * MF;
    if (free_vals && !bw) {
#pragma unroll
      for (int i = 0; i < MF; ++i) free_vals[(b * D + d) * np + (MID - 1) * MF + i] = xm[i];
    }

    // ---- back substitution outward, fused with the segments -----------------
    // Segment j of the lane (j = 0 next to MID): near vertex x_near (x_MID,
    // then the previous step's x), far vertex = the lane's step k = nsteps-1-j
    // (x_far = z_k - S_k^-1 (G_k x_near)) or the fixed end when j = nsteps.
    double acc = 0.0;
    double xn[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) xn[i] = xm[i];
#pragma unroll
    for (int j = 0; j < NSEG; ++j) {
      const int nseg = bw ? S - MID : MID;
      const bool seg_act = j < nseg;
      const int kf = NFW - 1 - j, kb = NBW - 1 - j;  // the lane's far step (< 0: fixed end)
      const bool far_fixed = bw ? kb < 0 : kf < 0;
      double xf[MF];
      if (NST > 0) {
        const int kfc = kf >= 0 ? kf : 0, kbc = kb >= 0 ? kb : 0;
        // Powers of the far step's coupling segment: forward C_v with
        // v = 1 + kf (segment v = MID-1-j .. its right = T[v]); backward
        // C_(v-1)^T with v = S-1-kb (segment v-1 = MID + j).
        double t = bw ? T[MID + j < S ? MID + j : S - 1] : T[MID - 1 - j >= 0 ? MID - 1 - j : 0];
        asm volatile("" : "+v"(t));  // recompute the powers, do not keep the forward copies
        Pw<N, R> Pc;
        Pc.set(t);
        double G[MF][MF];
        coupling(bw, Pc, Pc, G);
        double l[MF][MF], inv[MF], zk[MF];
        int q = 0;
#pragma unroll
        for (int i = 1; i < MF; ++i)
#pragma unroll
          for (int jj = 0; jj < i; ++jj) {
            l[i][jj] = bw ? Lf[kbc][q] : Lf[kfc][q];
            ++q;
          }
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          inv[i] = bw ? If[kbc][i] : If[kfc][i];
          zk[i] = bw ? z[kbc][i] : z[kfc][i];
        }
        double gx[MF], w[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          double s = 0.0;
#pragma unroll
          for (int m = 0; m < MF; ++m) s = fma(G[i][m], xn[m], s);
          gx[i] = s;
        }
        ldlt_apply<MF>(l, inv, gx, w);
#pragma unroll
        for (int i = 0; i < MF; ++i) xf[i] = zk[i] - w[i];
      } else {
#pragma unroll
        for (int i = 0; i < MF; ++i) xf[i] = 0.0;
      }
      // Segment index, times and vertex data.
      const int sf = MID - 1 - j, sb = MID + j;
      const int s = bw ? sb : sf;
      const double ts = bw ? T[sb < S ? sb : S - 1] : T[sf >= 0 ? sf : 0];
      Pw<N, R> P;
      P.set(ts);
      double e_near[M], e_far[M];
      // positions: forward near = vertex s+1, far = s; backward near = s,
      // far = s+1
      e_near[0] = bw ? pos[sb <= S ? sb : S] : pos[sf + 1 >= 0 ? sf + 1 : 0];
      e_far[0] = bw ? pos[sb + 1 <= S ? sb + 1 : S] : pos[sf >= 0 ? sf : 0];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        e_near[i + 1] = xn[i];
        e_far[i + 1] = far_fixed ? (bw ? xS[i + 1] : x0[i + 1]) : xf[i];
      }
      double e0[M], e1[M];
#pragma unroll
      for (int i = 0; i < M; ++i) {
        e0[i] = bw ? e_near[i] : e_far[i];
        e1[i] = bw ? e_far[i] : e_near[i];
      }
      if (seg_act) {
        acc += segment(e0, e1, P, cb ? cb + (s * D + d) * N : nullptr);
        if (!far_fixed && free_vals) {
          const int vfar = bw ? s + 1 : s;
#pragma unroll
          for (int i = 0; i < MF; ++i) free_vals[(b * D + d) * np + (vfar - 1) * MF + i] = xf[i];
        }
      }
#pragma unroll
      for (int i = 0; i < MF; ++i) xn[i] = xf[i];
    }
    *cost_part = acc;
    return pmin > 0.0 ? 0 : 2;
  }
};

}  // namespace lane2

// Lanes (trajectory t, dimension d, half h) = t * 2D + 2d + h; 10
// trajectories per wavefront at D = 3.
template <int N, int R, int D, int S>
__global__ __launch_bounds__(kWave) void linear_lane2_kernel(
    int64_t B, const double* __restrict__ fixed_vals, const double* __restrict__ times,
    double* __restrict__ coeffs, double* __restrict__ cost, double* __restrict__ free_vals,
    int32_t* __restrict__ status, SelectArgs sel) {
  constexpr int LPT = 2 * D;        // lanes per trajectory
  constexpr int TPW = kWave / LPT;  // trajectories per wavefront
  const int lane = threadIdx.x;
  const int tl = lane / LPT, r = lane - tl * LPT;
  const int d = r >> 1, h = r & 1;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * TPW + tl;
  const bool act = tl < TPW && b < B;
  double cpart = 0.0;
  int st = 0;
  // Lanes of a pair must run together (DPP exchange at the middle vertex):
  // inactive lanes run a valid dummy problem (trajectory 0) and discard it.
  {
    double dummy = 0.0;
    st = lane2::PairSolve<N, R, D, S>::run(act ? b : 0, act ? d : 0, h, fixed_vals, times,
                                           act ? coeffs : nullptr, act ? free_vals : nullptr,
                                           act ? &cpart : &dummy);
  }
  double tot = 0.0;
#pragma unroll
  for (int p = 0; p < LPT; ++p) tot += __shfl(cpart, tl * LPT + p);
  int stt = 0;
#pragma unroll
  for (int p = 0; p < LPT; ++p) stt = max(stt, __shfl(st, tl * LPT + p));
  if (act && r == 0) {
    if (cost) cost[b] = tot;
    if (status)
      status[b] = stt == 1 ? MTG_TRAJ_BAD_TIME : (stt == 2 ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK);
  }
  if (sel.out) select_epilogue(sel, tot, act && r == 0 ? b : -1, blockIdx.x, gridDim.x, B);
}

namespace {

template <int N, int R, int D, int S>
hipError_t launch_lane2(int64_t B, const double* df, const double* times, double* coeffs,
                        double* cost, double* free_vals, int32_t* status, hipStream_t st,
                        const SelectArgs& sel) {
  constexpr int TPW = kWave / (2 * D);
  const int64_t blocks = (B + TPW - 1) / TPW;
  hipLaunchKernelGGL((linear_lane2_kernel<N, R, D, S>), dim3(static_cast<unsigned>(blocks)),
                     dim3(kWave), 0, st, B, df, times, coeffs, cost, free_vals, status, sel);
  return hipGetLastError();
}

}  // namespace

int64_t lane2_blocks(int64_t B) {
  constexpr int TPW = kWave / 6;
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
