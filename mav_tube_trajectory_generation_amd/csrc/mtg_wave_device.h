// mtg_wave_device.h — the standard-pattern solver with the segment count S
// a compile-time constant (wave::Solver<N, R, D, S>): the per-trajectory
// body of the C2 kernel (mtg_linear_wave.hip) and of the compile-time-S
// time-allocation kernels (mtg_time_std.hip).  Same mathematics as
// stdp::Solver (mtg_std_device.h: updateSegmentTimes + solveLinear +
// computeCost, linear_impl:277-379, 113-130, with the exact time scaling
// H_s(T) = T^(1-2r) S_T H(1) S_T, A_s^-1(T) = D_T^-1 A(1)^-1 S_T), laid out
// so that a step of the elimination issues as few instructions and as
// little LDS traffic as possible (at C2 the four waves of a CU share its
// LDS and L1):
//   * every loop is unrolled and every LDS address of the sweep and the back
//     substitution is a per-lane base plus an immediate offset;
//   * chain slots: the forward chain's vertices v = 1 .. MID-1 and the
//     backward chain's v = S-1 .. MID+1 sit in the slots (chain, step) in
//     elimination order, each slot holding the vertex's Schur block (packed
//     lower triangle), the step's coupling P^T by rows, the right-hand sides
//     (then z) and Z by rows; slot (0, MID-1) is the middle vertex, slot
//     (1, NB) receives the backward chain's terms;
//   * a step runs on lanes (chain, column j, row i): column lanes j < 4 solve
//     for column j of the coupling, right-hand-side lanes j = 4 + d for
//     dimension d, and each lane of the four rows i forms only row i of its
//     output (out_i = a_i - P[:, i] . x): 4 FMAs instead of 16 per lane, and
//     stores only x_i;
//   * powers of T are formed in the lanes that use them (no LDS power table,
//     no phase boundary between the powers and the assembly);
//   * the constants a solve reads (d_f, H(1)) sit in LDS, loaded from HBM
//     once per trajectory by one lane each.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtg_std_device.h"

namespace mtg {
namespace wave {

using stdp::AInvTab;
using stdp::block2_solve;
using stdp::quad_bcast;
using stdp::rcp64_1;
using stdp::wave_sum_dpp;

template <int N, int R, int D, int S>
struct Geo {
  static constexpr int M = N / 2, MF = M - 1, MP = (M + 1) & ~1;
  static constexpr int MID = S / 2;                // middle vertex, 1 <= MID <= S-1
  static constexpr int NFW = MID - 1;              // forward steps: v = 1 .. MID-1
  static constexpr int NBW = S - 1 - MID;          // backward steps: v = S-1 .. MID+1
  static constexpr int NK = NFW > NBW ? NFW : NBW;
  static constexpr int NSL = NK + 1;               // slots per chain (+ terminal)
  static constexpr int NFIX = 2 * M + S - 1;       // fixed derivatives per dimension
  static constexpr int NROW = (S - 1) * MF;        // assembly rows
  static constexpr int TRI = MF * (MF + 1) / 2;
  // Slot layout (doubles; every piece 16-byte aligned).
  static constexpr int O_S = 0;                    // Schur block, packed lower triangle
  static constexpr int O_P = (TRI + 1) & ~1;       // P^T by rows (MF x MF)
  static constexpr int O_R = O_P + MF * MF;        // right-hand sides, then z (D x MF)
  static constexpr int O_Z = O_R + D * MF;         // Z = S^-1 P by rows (MF x MF)
  static constexpr int SLOT = O_Z + MF * MF;
  // LDS carve-up (doubles).
  static constexpr int L_DV = 0;                          // (S+1) x D x MP vertex derivatives
  static constexpr int L_SL = L_DV + (S + 1) * D * MP;    // 2 x NSL slots
  static constexpr int L_JUNK = L_SL + 2 * NSL * SLOT;    // stores nobody reads
  static constexpr int L_H = L_JUNK + 16;                 // H(1), N x N
  static constexpr int L_AUX = L_H + N * N;               // times and optimiser state
  static constexpr int NAUX = (6 * S + 8 + 1) & ~1;
  static constexpr int L_N = L_AUX + NAUX;
  static_assert(MF == 4, "4 x 4 blocks (block2_solve)");
  static_assert(NROW <= kWave && S * D <= kWave && 2 * 4 * (MF + D) <= kWave && D <= 3,
                "one pass of the wave per phase");
  static_assert((SLOT & 1) == 0 && (L_SL & 1) == 0 && (L_AUX & 1) == 0,
                "16-byte aligned slots");
};

__device__ constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }

// t^E for a compile-time integer E from t and 1/t (square-and-multiply).
template <int E>
__device__ inline double ipow(double t, double inv) {
  constexpr int A = E < 0 ? -E : E;
  double base = E < 0 ? inv : t, r = 1.0;
  bool first = true;
#pragma unroll
  for (int bit = 0; bit < 8; ++bit) {
    if ((A >> bit) & 1) {
      r = first ? base : r * base;
      first = false;
    }
    if ((A >> (bit + 1)) == 0) break;
    base *= base;
  }
  return r;
}

// q[l] = t^(1-2R+k+l), l = 0..M-1, for the row k = i+1 of the lane
// (selectors: i == 1, 2, 3).
template <int M, int R>
__device__ inline void row_powers(double t, bool i1, bool i2, bool i3, double (&q)[M]) {
  const double inv = rcp64_1(t);
  const double t2 = t * t, t3 = t2 * t;
  double ti = i1 ? t : 1.0;
  ti = i2 ? t2 : ti;
  ti = i3 ? t3 : ti;
  q[0] = ipow<2 - 2 * R>(t, inv) * ti;
  double tl = t;
#pragma unroll
  for (int l = 1; l < M; ++l) {
    q[l] = q[0] * tl;
    tl = l == 1 ? t2 : (l == 2 ? t3 : tl * t);
  }
}

template <int K>
__device__ inline void lds_ld(const double* p, double (&v)[K]) {
#pragma unroll
  for (int i = 0; i + 1 < K; i += 2) {
    const double2 x = *reinterpret_cast<const double2*>(p + i);
    v[i] = x.x;
    v[i + 1] = x.y;
  }
  if (K & 1) v[K - 1] = p[K - 1];
}
template <int K>
__device__ inline void lds_st(double* p, const double (&v)[K]) {
#pragma unroll
  for (int i = 0; i + 1 < K; i += 2)
    *reinterpret_cast<double2*>(p + i) = make_double2(v[i], v[i + 1]);
  if (K & 1) p[K - 1] = v[K - 1];
}

// Compiler-only memory fence: LDS operations of one wavefront complete in
// issue order, so a value another lane stored is visible to every later
// load; this keeps the compiler from moving a load above such a store.
__device__ inline void lds_order() { asm volatile("" ::: "memory"); }

template <int N, int R, int D, int S>
struct Solver {
  using G = Geo<N, R, D, S>;
  static constexpr int M = G::M, MF = G::MF, MP = G::MP, NFIX = G::NFIX, MID = G::MID;
  static constexpr int NFW = G::NFW, NBW = G::NBW, NK = G::NK, NSL = G::NSL, SLOT = G::SLOT;
  static constexpr int O_S = G::O_S, O_P = G::O_P, O_R = G::O_R, O_Z = G::O_Z;

  double *sm, *dv, *slots, *hh, *junk;
  int lane;
  // Lane roles: assembly row (av, ai) (lanes past the last row repeat vertex
  // S-1's rows, same row i = lane % MF, which the end-term lanes also use),
  // coefficient lane (cs, cd), end-term lane (ee, ed), sweep lane (g, jj, ii).
  int ai, av, cs, cd, ee, ed, g, q, jj, ii;
  bool i1, i2, i3;

  __device__ void init(double* smem) {
    sm = smem;
    dv = sm + G::L_DV;
    slots = sm + G::L_SL;
    hh = sm + G::L_H;
    junk = sm + G::L_JUNK;
    lane = threadIdx.x & (kWave - 1);
    ai = lane % MF;
    av = lane / MF + 1 < S - 1 ? lane / MF + 1 : S - 1;
    const int sd = lane < S * D ? lane : S * D - 1;
    cs = sd / D;
    cd = sd - cs * D;
    ee = (lane / (D * MF)) & 1;
    ed = (lane / MF) % D;
    g = lane >> 5;
    q = lane & 31;
    jj = q >> 2;
    ii = q & 3;
    i1 = ai == 1;
    i2 = ai == 2;
    i3 = ai == 3;
  }
  __device__ double* aux() const { return sm + G::L_AUX; }

  // Fixed value i of d_f (D x NFIX, the standard order of linear_impl:171-252:
  // vertex 0 derivatives 0..M-1, intermediate positions, vertex S
  // derivatives 0..M-1) into dv[v][d][k].
  __device__ void put_fixed(int i, double val) {
    int d = 0;
#pragma unroll
    for (int d2 = 1; d2 < D; ++d2) d += i >= d2 * NFIX ? 1 : 0;
    const int f = i - d * NFIX;
    const int v = f < M ? 0 : (f < M + S - 1 ? f - M + 1 : S);
    const int k = f < M ? f : (f < M + S - 1 ? 0 : f - (M + S - 1));
    dv[(v * D + d) * MP + k] = val;
  }

  // The per-trajectory constants into LDS: d_f (fb, D x NFIX) into dv and
  // H(1) (tab) into hh, one global load per lane each.  Caller orders LDS
  // (lds_order) before the first solve.
  __device__ void load_constants(const double* __restrict__ tab, const double* __restrict__ fb) {
    const double f0 = fb[lane < D * NFIX ? lane : D * NFIX - 1];
    double f1 = 0.0;
    if constexpr (D * NFIX > kWave)
      f1 = fb[lane + kWave < D * NFIX ? lane + kWave : D * NFIX - 1];
    const double2 h_own =
        *reinterpret_cast<const double2*>(tab + 2 * (lane < N * N / 2 ? lane : 0));
    store_constants(f0, f1, h_own);
  }
  __device__ void store_constants(double f0, double f1, double2 h_own) {
    if (lane < D * NFIX) put_fixed(lane, f0);
    if constexpr (D * NFIX > kWave)
      if (lane + kWave < D * NFIX) put_fixed(lane + kWave, f1);
    if (lane < N * N / 2) *reinterpret_cast<double2*>(hh + 2 * lane) = h_own;
  }

  // A solve at the segment times T (LDS, S valid values): dv receives every
  // vertex derivative.  Returns true if a pivot was not positive
  // (wave-uniform).  All lanes call.
  __device__ bool solve(const double* T) {
    // With no backward step (S = 2) the middle vertex reads the backward
    // chain's terminal slot as zero; otherwise its last step writes it.
    if constexpr (NBW == 0) {
      double* term = slots + NSL * SLOT;
      if (lane < G::TRI) term[O_S + lane] = 0.0;
      if (lane < D * MF) term[O_R + lane] = 0.0;
    }
    // ---- assembly.  Lane (v, i): row i (derivative k = i+1) of A_v =
    // H11(v-1) + H00(v), of C_v = H01(v) and b_v = -R_pf d_f on that row.
    // Exponent of H(a, b) at T: 1 - 2r + (a mod M) + (b mod M).
    const double tl = T[av - 1], tr = T[av], te = T[ee ? S - 1 : 0];
    double hk[N], hMk[N];
    lds_ld(hh + (ai + 1) * N, hk);
    lds_ld(hh + (M + ai + 1) * N, hMk);
    double pos[3][D], endd[M - 1];
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int d = 0; d < D; ++d) pos[w][d] = dv[((av - 1 + w) * D + d) * MP];
    {
      const double* de = dv + ((ee ? S : 0) * D + ed) * MP;
#pragma unroll
      for (int l = 1; l < M; ++l) endd[l - 1] = de[l];
    }
    auto slot_of = [&](int v) {  // v <= MID: forward slot v-1; else backward S-1-v
      return slots + (v <= MID ? v - 1 : NSL + S - 1 - v) * SLOT;
    };
    {
      double ql[M], qr[M];
      row_powers<M, R>(tl, i1, i2, i3, ql);
      row_powers<M, R>(tr, i1, i2, i3, qr);
      double Ar[MF], Cr[MF];
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        Ar[j] = fma(hMk[M + j + 1], ql[j + 1], hk[j + 1] * qr[j + 1]);
        Cr[j] = hk[M + j + 1] * qr[j + 1];
      }
      const double cpos = fma(hMk[M], ql[0], hk[0] * qr[0]);  // p_v
      const double cprev = hMk[0] * ql[0];                     // p_{v-1}
      const double cnext = hk[M] * qr[0];                      // p_{v+1}
      MTG_STAMP(1);
      double* sl = slot_of(av);
#ifndef MTG_ABL_NOB  // diagnostic ablation builds only (tools/gpu_r05_abl.sh)
#pragma unroll
      for (int d = 0; d < D; ++d) {
        double s = cpos * pos[1][d];
        s = fma(cprev, pos[0][d], s);
        s = fma(cnext, pos[2][d], s);
        sl[O_R + d * MF + ai] = -s;
      }
#endif
      // lower triangle of row i (entries j > i go to the slot's Z area,
      // written again by the sweep before it is read)
      const int rbase = O_S + tri(ai, 0);
#pragma unroll
      for (int j = 0; j < MF; ++j) sl[j <= ai ? rbase + j : O_Z + 4 * ai + j] = Ar[j];
      // forward step at v (v < MID): P = C_v, P^T by rows = C_v by columns;
      // backward step at v+1 (MID <= v <= S-2): P = C_v^T, P^T = C_v by rows.
      // A lane needs at most one of the two, so one set of stores with a
      // per-lane base and stride (LDS stores cost about three times a read's
      // time per byte and the four waves of a CU share them); lanes that
      // need neither store to the junk area.
      const bool fw = av < MID, bk = av >= MID && av < S - 1;
      double* pc = fw ? sl + O_P + ai : (bk ? slot_of(av + 1) + O_P + ai * MF : junk);
      const int ps = fw ? MF : 1;
#ifndef MTG_ABL_NOC
#pragma unroll
      for (int j = 0; j < MF; ++j) pc[j * ps] = Cr[j];
#endif
    }
    lds_order();
    MTG_STAMP(12);
    // The fully fixed end vertices' part of b_1 (segment 0) and b_(S-1)
    // (segment S-1): lane (e, d, i) adds -sum_l H_seg(k, l) d_f(l) for its row.
#ifndef MTG_ABL_NOEND
    {
      double qe[M];
      row_powers<M, R>(te, i1, i2, i3, qe);
      double s = 0.0;
#pragma unroll
      for (int l = 1; l < M; ++l) s = fma((ee ? hk[M + l] : hMk[l]) * qe[l], endd[l - 1], s);
      // lanes past the 2 D MF end lanes repeat one and add nothing
      atomicAdd(slot_of(ee ? S - 1 : 1) + O_R + ed * MF + ai, lane < 2 * D * MF ? -s : 0.0);
    }
#endif
    lds_order();
    MTG_STAMP(2);

    // ---- twisted block LDL^T.  Lane (g, j, i): chain g (0 forward, 1
    // backward), column j (< MF: coupling column; MF + d: right-hand side d),
    // row i.  Step k eliminates the chain's slot k: x = S^-1 u (u = P[:, j] or
    // r[d]), out_i = a_i - P[:, i] . x into slot k+1 (the next Schur block or
    // right-hand side), x_i into slot k (Z[i][j], or z[d][i] in place of r).
    double pmin = 1.0;
    {
      // lanes past the MF + D columns repeat column 0 (same values, same
      // addresses), so the sweep needs no execution mask
      const int jc = jj < MF + D ? jj : 0;
      const bool colj = jc < MF;
      const int dd = jc - MF;
      double* base = slots + g * NSL * SLOT;
      const double* Up = base + (colj ? O_P + jc * MF : O_R + dd * MF);
      const double* Pp = base + O_P + ii * MF;
      // a: entry (i, j) of the next Schur block (stored lower: (max, min)) or
      // b_next[d][i]; out goes to the same place, column lanes above the
      // diagonal to the next slot's Z area (their values duplicate (j, i)).
      const int mx = ii > jc ? ii : jc, mn = ii > jc ? jc : ii;
      const int lowr = O_S + ((mx * (mx + 1)) >> 1) + mn;
      const int aoff = colj ? lowr : O_R + dd * MF + ii;
      const int ooff = colj ? (ii >= jc ? lowr : O_Z + 4 * jc + ii) : aoff;
      const double* Ap = base + SLOT + aoff;
      double* Xp = base + (colj ? O_Z + ii * MF + jc : O_R + dd * MF + ii);
      double* Op = base + SLOT + ooff;
      const int nst = g ? NBW : NFW;
      if constexpr (NK > 0) {
        double pc[MF], a;
        lds_ld(Pp, pc);
        a = Ap[0];
#pragma unroll
        for (int k = 0; k < NK; ++k) {
          MTG_STAMP(100 + 2 * k);
          if (NFW == NBW || k < nst) {
            double Sv[MF][MF], u[MF], x[MF];
            {
              double t[G::TRI];
              lds_ld(base + k * SLOT + O_S, t);
#pragma unroll
              for (int r = 0; r < MF; ++r)
#pragma unroll
                for (int c = 0; c <= r; ++c) Sv[r][c] = t[tri(r, c)];
            }
            lds_ld(Up + k * SLOT, u);
            double pcn[MF], an = 0.0;
            if (k + 1 < NK) {  // next step's coupling row and Schur / rhs entry
              lds_ld(Pp + (k + 1) * SLOT, pcn);
              an = Ap[(k + 1) * SLOT];
            }
            block2_solve(Sv, u, x, pmin);
            // The backward chain's last step stores 0 - P^T x into its
            // terminal slot (the backward terms of the middle vertex): a is
            // 0 there instead of a zeroed slot's entry (no zeroing stores).
            if (k == NBW - 1) a = g ? 0.0 : a;
            // block2_solve finishes x[2], x[3] first
            double o = fma(-pc[2], x[2], a);
            o = fma(-pc[3], x[3], o);
            o = fma(-pc[0], x[0], o);
            o = fma(-pc[1], x[1], o);
            // x is the same in the four row lanes: each stores its row's entry
            double xi = i1 ? x[1] : x[0];
            xi = i2 ? x[2] : xi;
            xi = i3 ? x[3] : xi;
            Xp[k * SLOT] = xi;
            Op[k * SLOT] = o;
            lds_order();
            if (k + 1 < NK) {
#pragma unroll
              for (int m = 0; m < MF; ++m) pc[m] = pcn[m];
              a = an;
            }
          }
        }
      }
    }
    lds_order();
    MTG_STAMP(3);

    // ---- middle vertex (both halves, redundantly) and back substitution
    // outward: x_v = z_v - Z_v x_(toward MID).  Lane (g, d, i) owns row i of
    // dimension d of its chain; the other rows come from its quad by DPP.
    {
      const int d = jj;  // q = 4 d + i
      const bool p_act = q < 4 * D;
      const double* mf = slots + NFW * SLOT;          // slot (0, NFW): A_m - forward terms
      const double* mb = slots + (NSL + NBW) * SLOT;  // slot (1, NBW): -backward terms
      double Sv[MF][MF], rr[MF], x[MF];
      const int dc = p_act ? d : 0;
      {
        double t0[G::TRI], t1[G::TRI];
        lds_ld(mf + O_S, t0);
        lds_ld(mb + O_S, t1);
#pragma unroll
        for (int r = 0; r < MF; ++r)
#pragma unroll
          for (int c = 0; c <= r; ++c) Sv[r][c] = t0[tri(r, c)] + t1[tri(r, c)];
        double r0[MF], r1[MF];
        lds_ld(mf + O_R + dc * MF, r0);
        lds_ld(mb + O_R + dc * MF, r1);
#pragma unroll
        for (int r = 0; r < MF; ++r) rr[r] = r0[r] + r1[r];
      }
      // every back-substitution operand in flight before the middle solve
      const int nst = g ? NBW : NFW;
      const double* zb = slots + g * NSL * SLOT + O_R + dc * MF + ii;
      const double* Zb = slots + g * NSL * SLOT + O_Z + ii * MF;  // row i of Z
      double zz[NK > 0 ? NK : 1], zr[NK > 0 ? NK : 1][MF];
#pragma unroll
      for (int t = 0; t < NK; ++t) {
        const int sidx = NFW == NBW ? NK - 1 - t : (nst - 1 - t > 0 ? nst - 1 - t : 0);
        zz[t] = zb[sidx * SLOT];
        lds_ld(Zb + sidx * SLOT, zr[t]);
      }
      block2_solve(Sv, rr, x, pmin);
      double xi = i1 ? x[1] : x[0];
      xi = i2 ? x[2] : xi;
      xi = i3 ? x[3] : xi;
      *(p_act && g == 0 ? dv + (MID * D + d) * MP + 1 + ii : junk + ii) = xi;
#pragma unroll
      for (int t = 0; t < NK; ++t) {
        if (NFW == NBW || t < nst) {
          const double xb0 = quad_bcast<0>(xi), xb1 = quad_bcast<1>(xi);
          const double xb2 = quad_bcast<2>(xi), xb3 = quad_bcast<3>(xi);
          double s2 = fma(-zr[t][0], xb0, zz[t]);
          s2 = fma(-zr[t][1], xb1, s2);
          s2 = fma(-zr[t][2], xb2, s2);
          xi = fma(-zr[t][3], xb3, s2);
          const int sidx = NFW == NBW ? NK - 1 - t : nst - 1 - t;
          const int v = g ? S - 1 - sidx : 1 + sidx;
          *(p_act ? dv + (v * D + d) * MP + 1 + ii : junk + 4 + ii) = xi;
        }
      }
    }
    const bool not_spd = __any(!(pmin > 0.0));
    lds_order();
    MTG_STAMP(5);
    return not_spd;
  }

  // computeCost (wave-uniform) at the times T after solve(); the
  // coefficients (S x D x N) go to out (global or LDS, 16-byte aligned) when
  // out != nullptr.  Lane (s, d): f_j = e_j T^(j mod M), h = A(1)^-1 f,
  // c_i = T^-i h_i, 0.5 c^T Q c = T^(1-2r) sum w_ij h_i h_j (A(1)^-1 and w
  // are instruction literals).
  __device__ double coeff_cost(const double* T, double* out) const {
    double acc = 0.0;
    if (lane < S * D) {
      constexpr AInvTab<N> kA{};
      const double ts = T[cs];
      double e[N], f[N], h[N];
      {
        double e0[MP], e1[MP];
        lds_ld(dv + (cs * D + cd) * MP, e0);
        lds_ld(dv + ((cs + 1) * D + cd) * MP, e1);
#pragma unroll
        for (int j = 0; j < M; ++j) {
          e[j] = e0[j];
          e[M + j] = e1[j];
        }
      }
      const double inv = rcp64_1(ts);
      double tp[M], tn[N];
      tp[0] = 1.0;
      tn[0] = 1.0;
#pragma unroll
      for (int j = 1; j < M; ++j) tp[j] = (j & 1) ? tp[j - 1] * ts : tp[j / 2] * tp[j / 2];
#pragma unroll
      for (int j = 1; j < N; ++j) tn[j] = (j & 1) ? tn[j - 1] * inv : tn[j / 2] * tn[j / 2];
#pragma unroll
      for (int j = 0; j < N; ++j) f[j] = e[j] * tp[j % M];
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
        double cc[N];
#pragma unroll
        for (int i = 0; i < N; ++i) cc[i] = h[i] * tn[i];
        double2* o2 = reinterpret_cast<double2*>(out + static_cast<int64_t>(lane) * N);
#pragma unroll
        for (int i = 0; i < N / 2; ++i) o2[i] = make_double2(cc[2 * i], cc[2 * i + 1]);
      }
      acc = stdp::Solver<N, R, D>::q_form(h) * ipow<1 - 2 * R>(ts, inv);
    }
    return wave_sum_dpp(acc);
  }

  // sum_d e_s^T H_s(tau) e_s with the vertex derivatives of dv held fixed
  // (getCostAndGradientDerivative's J_d = d^T R d restricted to segment s,
  // nonlinear_impl:1537-1606, 2495-2584).  Called by one lane.
  __device__ double seg_energy(int s, double tau) const {
    constexpr AInvTab<N> kA{};
    const double inv = rcp64_1(tau);
    double tp[M];
    tp[0] = 1.0;
#pragma unroll
    for (int j = 1; j < M; ++j) tp[j] = tp[j - 1] * tau;
    const double tn = ipow<1 - 2 * R>(tau, inv);
    double tot = 0.0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      double f[N], h[N];
#pragma unroll
      for (int j = 0; j < N; ++j) f[j] = dv[((s + j / M) * D + d) * MP + j % M] * tp[j % M];
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
      tot += stdp::Solver<N, R, D>::q_form(h);
    }
    return 2.0 * tn * tot;  // e^T H e = c^T Q c = 2 * computeCost's share
  }
};

}  // namespace wave
}  // namespace mtg
