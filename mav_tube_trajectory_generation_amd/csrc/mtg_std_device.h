// mtg_std_device.h — per-trajectory FP64 solver for the standard vertex
// pattern (start and end vertex fully fixed, intermediate vertices position
// only: createRandomVertices / makeStartOrEnd, vertex.cpp:27-82, 147-153),
// run by one 64-lane wavefront (one workgroup).  Used by the standard-pattern
// linear-solve kernel (mtg_linear_std.hip) and the standard-pattern
// time-allocation kernels (mtg_time_std.hip).
//
// Same mathematics as the generic solver (mtg_device.h: linear_impl:277-379,
// 254-275, 113-130 restated with the exact time scaling
// H_s(T) = T^(1-2r) S_T H(1) S_T, A_s^-1(T) = D_T^-1 A(1)^-1 S_T), organised
// for the shortest instruction stream on one gfx950 wave.  A single wave
// issues one FP64 FMA per ~4.5 cycles with no extra dependency stall and
// v_rcp_f64 per 16 cycles (tools/ubench/fp64_latency.hip), so at one wave
// per SIMD the time of a solve is the wave's instruction count; every phase
// is written to minimise it:
//   * free unknowns are the MF = M-1 non-position derivatives of the S-1
//     intermediate vertices; the system is block tridiagonal with MF x MF
//     blocks (4 x 4 at N = 10 instead of the generic solver's pinned 5 x 5);
//   * assembly: lane (v, i) builds row i of A_v = H11(v-1) + H00(v), of the
//     coupling C_v = H01(v) (and column i of C_v^T) and b_v[i] from the rows
//     k, M+k of H(1), held in registers;
//   * twisted block LDL^T: lanes 0.. sweep forward over v = 1..m-1, lanes
//     32.. backward over v = S-1..m+1 in one instruction stream; in a chain
//     lane c < MF maps coupling column c, lane MF + d right-hand side d, all
//     through the same code with the step's coupling P (x = S^-1 u,
//     out = a - P^T x: the next Schur column, or the next right-hand side
//     b_next - P^T z_v; the data decides the role).  Every operand is a contiguous row (C_v and
//     C_v^T are both stored, Schur complements by rows), so a lane's
//     addresses are one base plus immediate offsets; next-step operands are
//     prefetched before the barrier;
//   * middle vertex and back substitution: a quad of lanes per (half,
//     dimension) solves the middle block redundantly and then walks its half
//     outward, one row of x per lane in registers, the other rows broadcast
//     inside the quad by DPP, the next step's Z row and z prefetched;
//   * coefficients and cost: lane (s, d); h_i = (A(1)^-1 f)_i with
//     f_j = e_j T^(j mod M), c_i = T^-i h_i, and computeCost's
//     0.5 c^T Q c = T^(1-2r) sum_ij w_ij h_i h_j with
//     w_ij = base(r,i) base(r,j) / (i+j-2r+1).  A(1)^-1 (exact rationals,
//     tools/gen_tables.py) and w are compile-time constants, so this phase
//     issues no table loads; the batch cost is a DPP wave reduction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtg_device.h"
#include "mtg_internal.h"
#include "mtg_tables_gen.h"

namespace mtg {
namespace stdp {

// One Newton step after v_rcp_f64: the seed is accurate to far more than
// the 27 bits one step needs to reach full FP64 precision.
__device__ inline double rcp64_1(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  const double e = fma(-d, r, 1.0);
  return fma(r, e, r);
}

// x = S^-1 r for a symmetric MF x MF block (lower triangle of S used) by
// LDL^T in registers.  pmin <- min(pmin, pivots): a non-positive value flags
// a matrix that is not positive definite (the caller reports it; the values
// computed from such a pivot are not used).
template <int MF>
__device__ inline void ldlt_solve(const double (&S)[MF][MF], const double (&r)[MF],
                                  double (&x)[MF], double& pmin) {
  double Lr[MF][MF];  // Lr[i][j] = L_ij * d_j (i > j)
  double l[MF][MF];   // l[i][j]  = L_ij
  double inv[MF];
#pragma unroll
  for (int j = 0; j < MF; ++j) {
    double dj = S[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) dj = fma(-Lr[j][k], l[j][k], dj);
    pmin = fmin(pmin, dj);
    inv[j] = rcp64_1(dj);
#pragma unroll
    for (int i = j + 1; i < MF; ++i) {
      double s = S[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) s = fma(-Lr[i][k], l[j][k], s);
      Lr[i][j] = s;
      l[i][j] = s * inv[j];
    }
  }
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

// x = S^-1 r for a symmetric 4 x 4 block by 2 x 2 blocks, S = [P Q; Q^T W]:
// P^-1 and (W - Q^T P^-1 Q)^-1 from their adjugates and one reciprocal of
// each determinant.  The dependent chain is two reciprocals deep (18 FP64
// operations) instead of LDL^T's four (about 28), which is what a sweep step
// waits on at one wave per SIMD.  pmin as ldlt_solve: the leading minors
// p00, det P, w00, det W' are all positive exactly when S is.
__device__ inline void block2_solve(const double (&S)[4][4], const double (&r)[4],
                                    double (&x)[4], double& pmin) {
  const double p00 = S[0][0], p10 = S[1][0], p11 = S[1][1];
  const double detP = fma(p00, p11, -(p10 * p10));
  const double ip = rcp64_1(detP);
  const double Pi00 = p11 * ip, Pi11 = p00 * ip, Pi10 = -p10 * ip;
  // Qt[a][b] = S[2+a][b] (= Q^T); Y = P^-1 Q, column a = P^-1 Qt[a][:]^T.
  const double Y00 = fma(Pi10, S[2][1], Pi00 * S[2][0]);
  const double Y10 = fma(Pi11, S[2][1], Pi10 * S[2][0]);
  const double Y01 = fma(Pi10, S[3][1], Pi00 * S[3][0]);
  const double Y11 = fma(Pi11, S[3][1], Pi10 * S[3][0]);
  // W' = W - Q^T Y (symmetric).
  const double w00 = fma(-S[2][1], Y10, fma(-S[2][0], Y00, S[2][2]));
  const double w10 = fma(-S[3][1], Y10, fma(-S[3][0], Y00, S[3][2]));
  const double w11 = fma(-S[3][1], Y11, fma(-S[3][0], Y01, S[3][3]));
  const double detW = fma(w00, w11, -(w10 * w10));
  const double iw = rcp64_1(detW);
  // y1 = P^-1 r_1, r2' = r_2 - Q^T y1, x_2 = W'^-1 r2', x_1 = y1 - Y x_2.
  const double y0 = fma(Pi10, r[1], Pi00 * r[0]);
  const double y1 = fma(Pi11, r[1], Pi10 * r[0]);
  const double s0 = fma(-S[2][1], y1, fma(-S[2][0], y0, r[2]));
  const double s1 = fma(-S[3][1], y1, fma(-S[3][0], y0, r[3]));
  x[2] = fma(-w10, s1, w11 * s0) * iw;
  x[3] = fma(-w10, s0, w00 * s1) * iw;
  x[0] = fma(-Y01, x[3], fma(-Y00, x[2], y0));
  x[1] = fma(-Y11, x[3], fma(-Y10, x[2], y1));
  pmin = fmin(pmin, fmin(fmin(p00, detP), fmin(w00, detW)));
}

template <int MF>
__device__ inline void block_solve(const double (&S)[MF][MF], const double (&r)[MF],
                                   double (&x)[MF], double& pmin) {
  if constexpr (MF == 4)
    block2_solve(S, r, x, pmin);
  else
    ldlt_solve<MF>(S, r, x, pmin);
}

// K doubles from / to LDS, 16-byte accesses for the pairs (callers keep the
// addresses of rows 16-byte aligned).
template <int K>
__device__ inline void lds_load(const double* p, double (&v)[K]) {
#pragma unroll
  for (int i = 0; i + 1 < K; i += 2) {
    const double2 t = *reinterpret_cast<const double2*>(p + i);
    v[i] = t.x;
    v[i + 1] = t.y;
  }
  if (K & 1) v[K - 1] = p[K - 1];
}
template <int K>
__device__ inline void lds_store(double* p, const double (&v)[K]) {
#pragma unroll
  for (int i = 0; i + 1 < K; i += 2)
    *reinterpret_cast<double2*>(p + i) = make_double2(v[i], v[i + 1]);
  if (K & 1) p[K - 1] = v[K - 1];
}

__device__ inline double join64(int lo, int hi) {
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) |
                                        static_cast<unsigned int>(lo));
}

// x + (x moved by DPP control CTRL), rows/banks masked as given; lanes with
// no source (or in disabled rows) add 0.
template <int CTRL, int RM, int BM>
__device__ inline double dpp_add(double x) {
  const long long u = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(u), CTRL, RM, BM, false);
  const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(u >> 32), CTRL, RM, BM, false);
  return x + join64(lo, hi);
}

// Value of lane j of this lane's quad (DPP quad_perm [j, j, j, j]).  Every
// source lane is valid, so the DPP `old` operand is left undefined (mov_dpp):
// one v_mov_b32_dpp per half, no initialisation of the destination.
template <int J>
__device__ inline double quad_bcast(double x) {
  const long long u = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(u), J * 0x55, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(u >> 32), J * 0x55, 0xf, 0xf, false);
  return join64(lo, hi);
}

// x + (x moved by DPP control CTRL) with every row enabled: lanes with no
// source read 0 through bound_ctrl, so no zeroed destination is needed.
template <int CTRL>
__device__ inline double dpp_add_bc(double x) {
  const long long u = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(u), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(u >> 32), CTRL, 0xf, 0xf, true);
  return x + join64(lo, hi);
}

// Sum over the 64 lanes (all active), returned wave-uniform: inclusive scan
// in rows of 16 (row_shr 1, 2, 4, 8), then row_bcast 15 and 31; lane 63
// holds the total.
__device__ inline double wave_sum_dpp(double x) {
  x = dpp_add_bc<0x111>(x);
  x = dpp_add_bc<0x112>(x);
  x = dpp_add_bc<0x114>(x);
  x = dpp_add_bc<0x118>(x);
  x = dpp_add<0x142, 0xa, 0xf>(x);
  x = dpp_add<0x143, 0xc, 0xf>(x);
  const long long u = __builtin_bit_cast(long long, x);
  return join64(__builtin_amdgcn_readlane(static_cast<int>(u), 63),
                __builtin_amdgcn_readlane(static_cast<int>(u >> 32), 63));
}

// A(1)^-1 as a local compile-time object (a static constexpr array read
// from device code is materialised in memory and loaded; a constexpr local
// object folds into instruction literals).
template <int N>
struct AInvTab {
  double v[N * N];
  constexpr AInvTab() : v() {
    for (int i = 0; i < N * N; ++i) v[i] = AInv1<N>::v[i];
  }
};

// computeCost weights w_ij = base(r,i) base(r,j) / (i+j-2r+1), i, j >= r
// (computeQuadraticCostJacobian, linear_impl:557-573, with its factor 2 and
// computeCost's 0.5 cancelled and T scaled out).
template <int N, int R>
struct CostW {
  double v[N][N];
  static constexpr double falling(int n, int i) {
    double p = 1.0;
    for (int m = 0; m < n; ++m) p *= static_cast<double>(i - m);
    return i < n ? 0.0 : p;
  }
  constexpr CostW() : v() {
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j)
        v[i][j] = (i >= R && j >= R)
                      ? falling(R, i) * falling(R, j) / static_cast<double>(i + j - 2 * R + 1)
                      : 0.0;
  }
};

// LDS carve-up in doubles.  Block rows have stride RS = MF rounded up to
// even and blocks BS = MF * RS, so every row read as a vector starts 16-byte
// aligned.
struct Layout {
  int pw;    // S * 2N: T_s^e at [s*2N + N + e], e in [-(N-1), N-1]
  int dv;    // (S+1) * D * MP: vertex derivatives [v][d][k] (MP = M rounded up even)
  int Sb;    // (S+1) * BS: A_v, then Schur complements, by rows
  int Cs;    // (S+1) * BS: C_v = coupling v -> v+1, [v][i][j]
  int Ct;    // (S+1) * BS: C_v^T
  int Zt;    // (S+1) * BS: Z_v^T (row c = column c of Z_v)
  int bz;    // (S+1) * D * RS: b_v, then z_v, [v][d][i]
  int Tm;    // BS: backward chain's Schur term at the middle vertex
  int Rmb;   // D * RS: backward chain's right-hand-side term at the middle vertex
  int aux;   // 6S + 8: segment times and optimiser state (time kernels)
  int n;
};

__host__ __device__ inline int even(int x) { return (x + 1) & ~1; }

__host__ __device__ inline Layout layout(int N, int S, int D) {
  const int M = N / 2, MF = M - 1, RS = even(MF), BS = MF * RS, MP = even(M);
  Layout l;
  int o = 0;
  l.pw = o; o += S * 2 * N;
  l.dv = o; o += (S + 1) * D * MP;
  l.Sb = o; o += (S + 1) * BS;
  l.Cs = o; o += (S + 1) * BS;
  l.Ct = o; o += (S + 1) * BS;
  l.Zt = o; o += (S + 1) * BS;
  l.bz = o; o += (S + 1) * D * RS;
  l.Tm = o; o += BS;
  l.Rmb = o; o += D * RS;
  l.aux = o; o += even(6 * S + 8);
  l.n = o;
  return l;
}

template <int N, int R, int D>
struct Solver {
  static constexpr int M = N / 2, MF = M - 1, RS = (MF + 1) & ~1, BS = MF * RS, PWP = 2 * N,
                       MP = (M + 1) & ~1;
  int S, lane, nf;
  Layout L;
  double* sm;
  double hk[N], hMk[N];  // rows k and M+k of H(1) for this lane's first assembly row

  __device__ double* pw() const { return sm + L.pw; }
  __device__ double* dv() const { return sm + L.dv; }
  __device__ double* aux() const { return sm + L.aux; }

  // tab == nullptr: the caller issues its own input loads first and calls
  // load_first_rows(tab) afterwards (vector loads retire in issue order, so
  // the inputs are then not held back behind the table rows).
  __device__ void init(int S_, double* smem, const double* __restrict__ tab) {
    S = S_;
    lane = threadIdx.x;
    nf = 2 * M + S - 1;
    L = layout(N, S, D);
    sm = smem;
    if (tab) load_first_rows(tab);
  }

  __device__ void load_first_rows(const double* __restrict__ tab) {
    load_rows(tab, lane % MF + 1);
  }

  __device__ void load_rows(const double* __restrict__ tab, int k) {
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      const double2 x = *reinterpret_cast<const double2*>(tab + k * N + j);
      const double2 y = *reinterpret_cast<const double2*>(tab + (M + k) * N + j);
      hk[j] = x.x;
      hk[j + 1] = x.y;
      hMk[j] = y.x;
      hMk[j + 1] = y.y;
    }
  }

  // Fixed value i of d_f (D x nf, standard order of linear_impl:171-252:
  // vertex 0 derivatives 0..M-1, intermediate positions, vertex S
  // derivatives 0..M-1) into dv.
  __device__ void put_fixed(int i, double val) {
    int d = 0;  // i / nf without an integer division (D <= 4)
#pragma unroll
    for (int d2 = 1; d2 < D; ++d2) d += i >= d2 * nf ? 1 : 0;
    const int f = i - d * nf;
    int v, k;
    if (f < M) {
      v = 0;
      k = f;
    } else if (f < M + S - 1) {
      v = f - M + 1;
      k = 0;
    } else {
      v = S;
      k = f - (M + S - 1);
    }
    dv()[(v * D + d) * MP + k] = val;
  }

  // Powers T_s^e by exact multiplication chains (1/T by rcp + Newton);
  // returns true if t is not a valid segment time.
  __device__ bool powers(int s, double t) {
    const bool bad = !(t > 0.0) || !(t < 1e300);
    const double inv = rcp64(t);
    double* p = pw() + s * PWP + N;
    double up = 1.0, dn = 1.0;
    p[0] = 1.0;
#pragma unroll
    for (int e = 1; e < N; ++e) {
      up *= t;
      dn *= inv;
      p[e] = up;
      p[-e] = dn;
    }
    return bad;
  }

  // Tm and Rmb (contiguous) start at zero: a chain with no steps leaves them.
  __device__ void clear_mid_terms() {
    for (int i = lane; i < BS + D * RS; i += kWave) sm[L.Tm + i] = 0.0;
  }

  // Powers of every segment from times in LDS (all lanes call; wave-uniform
  // result: any invalid time).  Also clears Tm.  Caller barriers after.
  __device__ bool powers_from(const double* T) {
    bool bad = false;
    for (int s = lane; s < S; s += kWave) bad = powers(s, T[s]) || bad;
    clear_mid_terms();
    return __any(bad);
  }

  // Assembly.  Lane (v, i): row i (derivative k = i+1) of A_v = H11(v-1) +
  // H00(v), C_v = H01(v) and b_v = -R_pf d_f restricted to that row.
  // Exponent of H(a, b) at T: 1 - 2r + (a mod M) + (b mod M).
  __device__ void assemble_row(int row) {
    double* pwp = pw();
    double* dvp = dv();
    const int v = row / MF + 1, i = row % MF, k = i + 1;
    const double* pl = pwp + (v - 1) * PWP + N + 1 - 2 * R + k;  // left segment
    const double* pr = pwp + v * PWP + N + 1 - 2 * R + k;        // right segment
    double ql[M], qr[M];
#pragma unroll
    for (int l = 0; l < M; ++l) {
      ql[l] = pl[l];
      qr[l] = pr[l];
    }
    double Ar[MF], Cr[MF];
#pragma unroll
    for (int j = 0; j < MF; ++j) {
      Ar[j] = fma(hMk[M + j + 1], ql[j + 1], hk[j + 1] * qr[j + 1]);
      Cr[j] = hk[M + j + 1] * qr[j + 1];
    }
    const double cpos = fma(hMk[M], ql[0], hk[0] * qr[0]);  // p_v
    const double cprev = hMk[0] * ql[0];                     // p_{v-1}
    const double cnext = hk[M] * qr[0];                      // p_{v+1}
#pragma unroll
    for (int d = 0; d < D; ++d) {
      double s = cpos * dvp[(v * D + d) * MP];
      s = fma(cprev, dvp[((v - 1) * D + d) * MP], s);
      s = fma(cnext, dvp[((v + 1) * D + d) * MP], s);
      sm[L.bz + (v * D + d) * RS + i] = -s;
    }
    lds_store(sm + L.Sb + v * BS + i * RS, Ar);
    lds_store(sm + L.Cs + v * BS + i * RS, Cr);
#pragma unroll
    for (int j = 0; j < MF; ++j) sm[L.Ct + v * BS + j * RS + i] = Cr[j];
  }

  // The fully fixed end vertices' part of b_1 (vertex 0, segment 0) and of
  // b_(S-1) (vertex S, segment S-1): lane (e, d, i) adds
  // -sum_l H_seg(k, l) d_f(l) for its row after the row lanes stored theirs,
  // so these 2 D MF products run once instead of in every row lane.  Needs
  // the lane's H(1) rows at k = lane % MF + 1.
  __device__ void assemble_ends() {
    if (lane < 2 * D * MF) {
      const int i = lane % MF, k = i + 1, ed = lane / MF;
      const bool right = ed >= D;
      const int d = right ? ed - D : ed;
      const double* pp = pw() + (right ? S - 1 : 0) * PWP + N + 1 - 2 * R + k;
      const double* dd = dv() + ((right ? S : 0) * D + d) * MP;
      double s = 0.0;
#pragma unroll
      for (int l = 1; l < M; ++l) s = fma((right ? hk[M + l] : hMk[l]) * pp[l], dd[l], s);
      atomicAdd(sm + L.bz + ((right ? S - 1 : 1) * D + d) * RS + i, -s);
    }
  }

  // All rows; rows beyond the first pass (S > 17) reload their H(1) rows.
  // Caller barriers after.
  __device__ void assemble(const double* __restrict__ tab) {
    const int nrows = (S - 1) * MF;
    if (lane < nrows) assemble_row(lane);
    for (int row = lane + kWave; row < nrows; row += kWave) {
      load_rows(tab, row % MF + 1);
      assemble_row(row);
    }
    if (nrows > kWave) load_rows(tab, lane % MF + 1);
    asm volatile("" ::: "memory");  // the rows' b stores precede the end terms
    assemble_ends();
  }

  // Twisted block LDL^T, middle vertex and back substitution: on return (after
  // the final barrier) dv holds every vertex derivative.  Returns true if a
  // pivot was not positive (wave-uniform).
  __device__ bool solve() {
    const int m = S / 2;  // middle vertex, 1 <= m <= S-1
    const int g = lane >> 5, q = lane & 31;
    double pmin = 1.0;  // smallest pivot seen by this lane
    {
      const bool cpl = q < MF;  // coupling-column lane
      const bool rhs = q >= MF && q < MF + D;
      const int c = cpl ? q : 0, dd = rhs ? q - MF : 0;
      const int nst = g == 0 ? m - 1 : S - 1 - m;
      const int kmax = (m - 1) > (S - 1 - m) ? (m - 1) : (S - 1 - m);
      const int dir = g == 0 ? 1 : -1;
      const int v0 = g == 0 ? 1 : S - 1;
      // Every lane of a chain uses the same coupling P of its step (forward
      // C_v, backward C_{v-1}^T) and computes x = S_v^-1 u, out = a - P^T x:
      //   coupling lane c: u = P[:, c] (= row c of P^T), a = row c of A_next;
      //     x -> row c of Z_v^T, out -> row c of S_next;
      //   rhs lane d: u = r_v[d] (b_v at the first step), a = b_next[d];
      //     x = z_v -> in place of r_v, out = r_next = b_next - P^T z_v -> in
      //     place of b_next, where the next step reads it as u.
      // The forward chain's last step leaves S_m and r_m with its term
      // subtracted in place; the backward chain's last step (a = 0) stores its
      // terms alone into Tm and Rmb.
      const int gofs = g == 0 ? L.Cs + v0 * BS : L.Ct + (v0 - 1) * BS;
      const int gstep = dir * BS;
      const int uofs = cpl ? (g == 0 ? L.Ct + v0 * BS : L.Cs + (v0 - 1) * BS) + c * RS
                           : L.bz + (v0 * D + dd) * RS;
      const int ustep = cpl ? dir * BS : dir * D * RS;
      const int aofs = cpl ? L.Sb + (v0 + dir) * BS + c * RS : L.bz + ((v0 + dir) * D + dd) * RS;
      const int xofs = cpl ? L.Zt + v0 * BS + c * RS : uofs;
      const int mofs = cpl ? L.Tm + c * RS : L.Rmb + dd * RS;  // backward last step
      double G[MF][MF], u[MF], a[MF];
      auto load_ops = [&](int k) {
        const double* Gp = sm + gofs + k * gstep;
#pragma unroll
        for (int i = 0; i < MF; ++i) lds_load(Gp + i * RS, G[i]);
        lds_load(sm + uofs + k * ustep, u);
        lds_load(sm + aofs + k * ustep, a);
      };
      const bool lane_act = cpl || rhs;
      if (lane_act && nst > 0) load_ops(0);
      for (int k = 0; k < kmax; ++k) {
        MTG_STAMP(100 + 2 * k);
        if (lane_act && k < nst) {
          const int v = v0 + k * dir;
          double Sv[MF][MF];
#pragma unroll
          for (int i = 0; i < MF; ++i) {
            double row[MF];
            lds_load(sm + L.Sb + v * BS + i * RS, row);
#pragma unroll
            for (int j = 0; j <= i; ++j) Sv[i][j] = row[j];
          }
          double x[MF];
          block_solve<MF>(Sv, u, x, pmin);
          const bool last_b = g == 1 && k == nst - 1;
          const double af = last_b ? 0.0 : 1.0;
          double out[MF];
#pragma unroll
          for (int i = 0; i < MF; ++i) {
            double s = a[i] * af;
#pragma unroll
            for (int jj = 0; jj < MF; ++jj) {
              // block2_solve finishes x[2], x[3] first: take them first.
              const int j = MF == 4 ? (jj + 2) & 3 : jj;
              s = fma(-G[j][i], x[j], s);
            }
            out[i] = s;
          }
          lds_store(sm + xofs + k * ustep, x);
          lds_store(sm + (last_b ? mofs : aofs + k * ustep), out);
          if (k + 1 < nst) load_ops(k + 1);
        }
        __syncthreads();
      }
    }
    MTG_STAMP(3);

    // Middle vertex and back substitution outward from it:
    //   S_m = (A_m - forward term) + Tm,  r_m = (b_m - forward term) + Rmb
    //   (= b_m - C_{m-1}^T z_{m-1} - C_m z'_{m+1}),  x_v = z_v - Z_v x_(toward m).
    // Lanes: for MF <= 4 a quad per (half g, dimension d), lane = g*32 + 4d + i
    // owning row i (the middle block is solved redundantly by all of them, so
    // no exchange precedes the back substitution, whose x_next rows are
    // broadcast inside the quad by DPP quad_perm); for MF = 5 one lane per
    // (g, d) holding all rows.
    constexpr bool kQuad = MF <= 4;
    const int pd = kQuad ? (q >> 2) : q;
    const int pi = kQuad ? (q & 3) : 0;
    const bool p_act = kQuad ? (pd < D && pi < MF) : (q < D);
    double* dvp = dv();
    const double* Zt = sm + L.Zt;
    const double* bz = sm + L.bz;
    if (p_act) {
      const int d = pd;
      double Sv[MF][MF], rr[MF], x[MF];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        double row[MF], tm[MF];
        lds_load(sm + L.Sb + m * BS + i * RS, row);
        lds_load(sm + L.Tm + i * RS, tm);
#pragma unroll
        for (int j = 0; j <= i; ++j) Sv[i][j] = row[j] + tm[j];
      }
      {
        double r0[MF], r1[MF];
        lds_load(bz + (m * D + d) * RS, r0);
        lds_load(sm + L.Rmb + d * RS, r1);
#pragma unroll
        for (int i = 0; i < MF; ++i) rr[i] = r0[i] + r1[i];
      }
      block_solve<MF>(Sv, rr, x, pmin);
      MTG_STAMP(4);
      const int n_back = g == 0 ? m - 1 : S - 1 - m;
      const int vstep = g == 0 ? -1 : 1;
      if constexpr (kQuad) {
        double xi = x[0];  // own row of x_m
#pragma unroll
        for (int i = 1; i < MF; ++i) xi = pi == i ? x[i] : xi;
        if (g == 0) dvp[(m * D + d) * MP + 1 + pi] = xi;
        MTG_STAMP(8);
        auto step = [&](const double (&zr)[MF], double zz) {
          double xb[4];
          xb[0] = quad_bcast<0>(xi);
          if (MF > 1) xb[1] = quad_bcast<1>(xi);
          if (MF > 2) xb[2] = quad_bcast<2>(xi);
          if (MF > 3) xb[3] = quad_bcast<3>(xi);
          double s2 = zz;
#pragma unroll
          for (int j = 0; j < MF; ++j) s2 = fma(-zr[j], xb[j], s2);
          xi = s2;
        };
        // x_next row pi from Z_v's row pi and the broadcast rows of x (the
        // next step's operands are loaded before this step's chain).  A DPP
        // broadcast after a VALU result costs ~20 cycles of latency
        // (tools/ubench/fp64_latency.hip), so a step is ~70 cycles.
        double zr[MF], zz = 0.0;
        auto load_b = [&](int vv) {
#pragma unroll
          for (int c2 = 0; c2 < MF; ++c2) zr[c2] = Zt[vv * BS + c2 * RS + pi];
          zz = bz[(vv * D + d) * RS + pi];
        };
        int v = m + vstep;
        constexpr int kPre = 4;
        if (n_back <= kPre) {
          // Every step's operands in flight before the first step (S <= 10).
          double zr4[kPre][MF], zz4[kPre];
#pragma unroll
          for (int k = 0; k < kPre; ++k) {
            if (k < n_back) {
              load_b(v + k * vstep);
#pragma unroll
              for (int c2 = 0; c2 < MF; ++c2) zr4[k][c2] = zr[c2];
              zz4[k] = zz;
            }
          }
#pragma unroll
          for (int k = 0; k < kPre; ++k) {
            if (k < n_back) {
              step(zr4[k], zz4[k]);
              dvp[((v + k * vstep) * D + d) * MP + 1 + pi] = xi;
            }
          }
        } else {
          if (n_back > 0) load_b(v);
          for (int k = 0; k < n_back; ++k, v += vstep) {
            double zc[MF], zzc = zz;
#pragma unroll
            for (int c2 = 0; c2 < MF; ++c2) zc[c2] = zr[c2];
            if (k + 1 < n_back) load_b(v + vstep);
            step(zc, zzc);
            dvp[(v * D + d) * MP + 1 + pi] = xi;
          }
        }
      } else {
        if (g == 0) {
#pragma unroll
          for (int i = 0; i < MF; ++i) dvp[(m * D + d) * MP + 1 + i] = x[i];
        }
        double Zc[MF][MF], zc[MF];
        auto load_back = [&](int vv) {
#pragma unroll
          for (int j = 0; j < MF; ++j) lds_load(Zt + vv * BS + j * RS, Zc[j]);
          lds_load(bz + (vv * D + d) * RS, zc);
        };
        int v = m + vstep;
        if (n_back > 0) load_back(v);
        for (int k = 0; k < n_back; ++k, v += vstep) {
          double xn[MF];
#pragma unroll
          for (int i = 0; i < MF; ++i) {
            double s2 = zc[i];
#pragma unroll
            for (int j = 0; j < MF; ++j) s2 = fma(-Zc[j][i], x[j], s2);
            xn[i] = s2;
          }
          if (k + 1 < n_back) load_back(v + vstep);
#pragma unroll
          for (int i = 0; i < MF; ++i) {
            x[i] = xn[i];
            dvp[(v * D + d) * MP + 1 + i] = xn[i];
          }
        }
      }
      MTG_STAMP(9);
    }
    const bool not_spd = __any(!(pmin > 0.0));
    __syncthreads();
    MTG_STAMP(5);
    return not_spd;
  }

  // Coefficients (when out != null, S x D x N at `out`, global or LDS, 16-byte
  // aligned) and computeCost of segment-dimension sd; returns this lane's
  // share of the cost (0.5 c^T Q c summed over its (s, d)).
  __device__ double coeff_cost_sd(int sd, double* out) const {
    constexpr AInvTab<N> kA{};
    const int s = sd / D, d = sd % D;
    const double* ps = pw() + s * PWP + N;
    double e[N], f[N], h[N];
    {
      double e0[MP], e1[MP];
      lds_load(dv() + (s * D + d) * MP, e0);
      lds_load(dv() + ((s + 1) * D + d) * MP, e1);
#pragma unroll
      for (int j = 0; j < M; ++j) {
        e[j] = e0[j];
        e[M + j] = e1[j];
      }
    }
    double tp[MP];
    lds_load(ps, tp);  // T^0 .. T^(MP-1)
#pragma unroll
    for (int j = 0; j < N; ++j) f[j] = e[j] * tp[j % M];
    // Rows k < M of A(1)^-1 are diagonal (A(0) = diag(k!)).
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
      for (int i = 0; i < N; ++i) cc[i] = h[i] * ps[-i];
      double2* o2 = reinterpret_cast<double2*>(out + static_cast<int64_t>(sd) * N);
#pragma unroll
      for (int i = 0; i < N / 2; ++i) o2[i] = make_double2(cc[2 * i], cc[2 * i + 1]);
    }
    return q_form(h) * ps[1 - 2 * R];
  }

  // sum_ij w_ij h_i h_j over i, j >= r.
  __device__ static double q_form(const double (&h)[N]) {
    constexpr CostW<N, R> kW{};
    double q2 = 0.0;
#pragma unroll
    for (int i = R; i < N; ++i) {
      double t = kW.v[i][i] * h[i];
#pragma unroll
      for (int j = i + 1; j < N; ++j) t = fma(2.0 * kW.v[i][j], h[j], t);
      q2 = fma(t, h[i], q2);
    }
    return q2;
  }

  // computeCost (wave-uniform), coefficients into out when non-null.
  __device__ double coeff_cost(double* out) const {
    double acc = 0.0;
    // First pass outside any loop so the folded constants are not hoisted and
    // kept live across iterations.
    if (lane < S * D) acc = coeff_cost_sd(lane, out);
    for (int sd = lane + kWave; sd < S * D; sd += kWave) acc += coeff_cost_sd(sd, out);
    return wave_sum_dpp(acc);
  }

  // sum_d e_s^T H_s(tau) e_s with the vertex derivatives of dv held fixed:
  // the part of getCostAndGradientDerivative's J_d = d^T R d that depends on
  // T_s (nonlinear_impl:1537-1606, 2495-2584).  Called by one lane.
  __device__ double seg_energy(int s, double tau) const {
    constexpr AInvTab<N> kA{};
    const double inv = rcp64(tau);
    double tp[N], tn;  // tau^0 .. tau^(M-1); tau^(1-2r)
    tp[0] = 1.0;
#pragma unroll
    for (int j = 1; j < M; ++j) tp[j] = tp[j - 1] * tau;
    {
      const int e = 1 - 2 * R;
      const double base = e < 0 ? inv : tau;
      double p = 1.0;
#pragma unroll
      for (int q2 = 0; q2 < (e < 0 ? -e : e); ++q2) p *= base;
      tn = p;
    }
    double tot = 0.0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      double f[N], h[N];
#pragma unroll
      for (int j = 0; j < N; ++j) f[j] = dv()[((s + j / M) * D + d) * MP + j % M] * tp[j % M];
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
      tot += q_form(h);
    }
    return 2.0 * tn * tot;  // e^T H e = c^T Q c = 2 * computeCost's share
  }
};

}  // namespace stdp
}  // namespace mtg
