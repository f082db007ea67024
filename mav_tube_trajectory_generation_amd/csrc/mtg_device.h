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
//     trajectory the same uniform block structure.
//   * Block LDL^T sweep over the S+1 vertices.  Per vertex one parallel Schur
//     step (lanes over block entries) and one factor step in which lane c
//     factors the M x M block in registers and turns column c of the coupling
//     block / right-hand side into Z_v = S_v^-1 O_v, z_v = S_v^-1 r_v.  The
//     back substitution is then the affine recurrence x_v = z_v - Z_v x_{v+1}
//     (M*D lanes, one step per vertex).  Fully fixed vertices (start/end of
//     the standard pattern) skip the factorisation.
// LDS holds everything a trajectory touches (about 11 KB at S=10, N=10,
// D=3); HBM sees only the compact inputs (times, d_f) and the outputs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtg_internal.h"

// Diagnostic build only (make STAMPS=1): s_memtime stamps of workgroup 0 at
// phase boundaries into g_mtg_stamps (read by mtg_debug_stamps).  The
// shipped library never defines MTG_STAMPS.
#ifdef MTG_STAMPS
__device__ unsigned long long g_mtg_stamps[512];
#define MTG_STAMP(slot)                                                     \
  do {                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                      \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                              \
      unsigned long long t_;                                                \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      g_mtg_stamps[(slot)] = t_;                                            \
    }                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                      \
  } while (0)
// Accumulating variant: adds the cycles since `last` to slot and resets
// `last` (phase totals over loop iterations).
#define MTG_TACC(slot, last)                                                \
  do {                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                      \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                              \
      unsigned long long t_;                                                \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      atomicAdd(&g_mtg_stamps[(slot)], t_ - (last)); /* no-return: no wait */ \
      (last) = t_;                                                          \
    }                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                      \
  } while (0)
#else
#define MTG_STAMP(slot) \
  do {                  \
  } while (0)
#define MTG_TACC(slot, last) \
  do {                       \
    (void)(last);            \
  } while (0)
#endif

namespace mtg {

constexpr int kWave = 64;

// XCD-aware problem index of a one-problem-per-workgroup launch.  The
// dispatcher deals workgroups to the eight XCDs round-robin (workgroup i to
// XCD i mod 8: tools/tube_order.py fits that model), and each XCD has its
// own L2, so with b = blockIdx.x neighbouring problems, which share the cache
// lines at the edges of their input rows, land on different XCDs and each
// of them fetches those lines from HBM.  This bijection gives XCD x the
// contiguous range of problems [x q + min(x, r), ...) (q = G / 8,
// r = G mod 8), so shared lines are read once.
constexpr int kXcds = 8;
__device__ inline int64_t xcd_problem(int64_t i, int64_t G) {
  const int64_t q = G / kXcds, r = G % kXcds;
  const int64_t x = i % kXcds, k = i / kXcds;
  return x * q + (x < r ? x : r) + k;
}

// Copy NCH 16-byte pieces of a staged output from LDS to global memory, lane
// t of a group of W lanes taking pieces t, t + W, ...: consecutive lanes
// store consecutive addresses (one instruction covers W x 16 contiguous
// bytes), and four LDS reads are in flight per batch (named registers: an
// array here is promoted to LDS before the loop is unrolled).
template <int W, int NCH>
__device__ inline void copy_out16(const double2* __restrict__ src, double2* __restrict__ dst,
                                  int t) {
  constexpr int IT = (NCH + W - 1) / W;
#pragma unroll
  for (int k0 = 0; k0 < IT; k0 += 4) {
    const int c0 = t + k0 * W, c1 = c0 + W, c2 = c1 + W, c3 = c2 + W;
    double2 a0 = {}, a1 = {}, a2 = {}, a3 = {};
    if (c0 < NCH) a0 = src[c0];
    if (k0 + 1 < IT && c1 < NCH) a1 = src[c1];
    if (k0 + 2 < IT && c2 < NCH) a2 = src[c2];
    if (k0 + 3 < IT && c3 < NCH) a3 = src[c3];
    if (c0 < NCH) dst[c0] = a0;
    if (k0 + 1 < IT && c1 < NCH) dst[c1] = a1;
    if (k0 + 2 < IT && c2 < NCH) dst[c2] = a2;
    if (k0 + 3 < IT && c3 < NCH) dst[c3] = a3;
  }
}

// LDS carve-up (in doubles, then ints), identical for every kernel.
struct Layout {
  int tabH, tabA;  // H(1), A(1)^-1: N*N each
  int pw;          // S * (2N-1): T_s^e for e in [-(N-1), N-1]
  int T;           // S segment times
  int dv;          // (S+1)*M*D vertex derivatives (fixed values, then x)
  int Dt;          // (S+1)*M*M diagonal blocks -> pinned -> Schur complements
  int Ot;          // S*M*M     coupling blocks -> pinned
  int Zt;          // (S+1)*M*M Z_v of the two sweeps (see solve)
  int Tm;          // M*M       backward sweep's Schur term at the middle vertex
  int Bt;          // (S+1)*M*D right-hand sides -> z_v = S_v^-1 r_v
  int aux;         // 4*S extra (optimiser state)
  int ndouble;
  int slot;        // (S+1)*M int slots (after the doubles)
  int nint;
  __host__ __device__ size_t bytes() const { return sizeof(double) * ndouble + sizeof(int) * nint; }
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
  l.Zt = o;   o += (S + 1) * M * M;
  l.Tm = o;   o += M * M;
  l.Bt = o;   o += (S + 1) * M * D;
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
  double* sm;         // double region
  int* si;            // int region
  int lane;
  uint64_t fmask;     // fixed-pattern bits (v*M+k) when (S+1)*M <= 64
  bool use_mask;

  __device__ double* tabH() const { return sm + lay->tabH; }
  __device__ double* tabA() const { return sm + lay->tabA; }
  __device__ double* pw() const { return sm + lay->pw; }
  __device__ double* T() const { return sm + lay->T; }
  __device__ double* dv() const { return sm + lay->dv; }
  __device__ int* slot() const { return si + lay->slot; }
  __device__ int* flag() const { return si + (S + 1) * M; }

  // T_s^e, e in [-(N-1), N-1].
  __device__ double pwr(int s, int e) const { return pw()[s * PWN + e + (N - 1)]; }
  // Pattern test: SGPR bitmask when it fits (wave-uniform, no LDS load).
  __device__ bool fixed_at(int v, int k) const {
    const int idx = v * M + k;
    return use_mask ? ((fmask >> idx) & 1ull) != 0 : slot()[idx] >= 0;
  }
  __device__ bool vertex_fixed(int v) const {
    bool all = true;
#pragma unroll
    for (int k = 0; k < M; ++k) all = all && fixed_at(v, k);
    return all;
  }

  // H_s block entry: row (a_blk, j), column (b_blk, k); a_blk 0 = start
  // vertex s, 1 = end vertex s+1.
  __device__ double H(int s, int ab, int bb, int j, int k) const {
    return tabH()[(ab * M + j) * N + bb * M + k] * pwr(s, 1 - 2 * r + j + k);
  }

  // All global inputs of one trajectory in a single round of independent
  // loads (first pass of every array issued before any LDS store): tables,
  // slots, times, and d_f scattered into dv (fixed_map gives the (vertex,
  // derivative) slot of fixed index f).
  __device__ void load_inputs(const double* __restrict__ tab, const int* __restrict__ slots,
                              const int* __restrict__ fixed_map,
                              const double* __restrict__ times_b,
                              const double* __restrict__ df, int nf) {
    constexpr int NT = (2 * N * N + kWave - 1) / kWave;
    const int nslot = (S + 1) * M, ndf = D * nf;
    double rt[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int i = lane + q * kWave;
      rt[q] = i < 2 * N * N ? tab[i] : 0.0;
    }
    const int rs = lane < nslot ? slots[lane] : 0;
    const double rtime = lane < S ? times_b[lane] : 0.0;
    const double rdf = lane < ndf ? df[lane] : 0.0;
    const int rfm = lane < ndf ? fixed_map[lane % nf] : 0;
    // dv: zero everything, then scatter the fixed values (same wave, LDS
    // stores retire in order).
    for (int i = lane; i < (S + 1) * M * D; i += kWave) dv()[i] = 0.0;
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int i = lane + q * kWave;
      if (i < 2 * N * N) sm[lay->tabH + i] = rt[q];
    }
    if (lane < nslot) slot()[lane] = rs;
    if (lane < S) T()[lane] = rtime;
    if (lane < ndf) dv()[rfm * D + lane / nf] = rdf;
    // Remainders for large S (never taken at the benchmark sizes).
    for (int i = lane + kWave; i < nslot; i += kWave) slot()[i] = slots[i];
    for (int i = lane + kWave; i < S; i += kWave) T()[i] = times_b[i];
    for (int i = lane + kWave; i < ndf; i += kWave)
      dv()[fixed_map[i % nf] * D + i / nf] = df[i];
    if (lane == 0) flag()[0] = 0;
  }

  // Powers T_s^e by two multiplication chains per segment (exact integer
  // exponents; 1/T by rcp64).  Sets flag()[0] |= 1 if any time is not > 0.
  __device__ void compute_powers() {
    for (int s = lane; s < S; s += kWave) {
      const double t = T()[s];
      if (!(t > 0.0) || !(t < 1e300)) atomicOr(&flag()[0], 1);
      const double inv = rcp64(t);
      double* p = pw() + s * PWN + (N - 1);
      double up = 1.0, dn = 1.0;
      p[0] = 1.0;
#pragma unroll
      for (int e = 1; e < N; ++e) {
        up *= t;
        dn *= inv;
        p[e] = up;
        p[-e] = dn;
      }
    }
  }

  // Re-zero the free entries of dv (before a re-solve that reuses dv).
  __device__ void clear_free() {
    for (int i = lane; i < (S + 1) * M * D; i += kWave) {
      const int vk = i / D;
      if (!fixed_at(vk / M, vk % M)) dv()[i] = 0.0;
    }
  }

  __device__ double dval(int v, int k, int d) const {
    return dv()[(v * M + k) * D + d];
  }

  // Blocks of R in vertex order, b = -R_pf d_f, then pinning, in one pass:
  // lane (v, j) builds row j of D_v and O_v, column j of O_{v-1} and b_v[j]
  // in registers from rows j and M+j of H(1) (plus column M+j) and the
  // powers of segments v-1 and v, then writes the pinned rows.
  __device__ void assemble() {
    double* Dt = sm + lay->Dt;
    double* Ot = sm + lay->Ot;
    double* Bt = sm + lay->Bt;
    const double* tH = tabH();
    for (int row = lane; row < (S + 1) * M; row += kWave) {
      const int v = row / M, j = row % M;
      const double fl = v > 0 ? 1.0 : 0.0, fr = v < S ? 1.0 : 0.0;
      const int sl = v > 0 ? v - 1 : 0, sr = v < S ? v : S - 1;
      double Dr[M], Or[M], Oc[M];
#pragma unroll
      for (int k = 0; k < M; ++k) {
        const double pl = pwr(sl, 1 - 2 * r + j + k), pr = pwr(sr, 1 - 2 * r + j + k);
        Dr[k] = fl * (tH[(M + j) * N + M + k] * pl) + fr * (tH[j * N + k] * pr);  // H(v-1,1,1)+H(v,0,0)
        Or[k] = fr * (tH[j * N + M + k] * pr);                                    // H(v,0,1)[j][k]
        Oc[k] = fl * (tH[k * N + M + j] * pl);                                    // H(v-1,0,1)[k][j]
      }
      const int v0 = v > 0 ? v - 1 : 0, v2 = v < S ? v + 1 : S;
      // dv is zero at free entries: the sums run over fixed columns only.
      const bool fj = fixed_at(v, j);
#pragma unroll
      for (int d = 0; d < kMaxD; ++d) {
        if (d >= D) break;
        double b = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) {
          b = fma(Dr[k], dval(v, k, d), b);
          b = fma(Or[k], dval(v2, k, d), b);
          b = fma(Oc[k], dval(v0, k, d), b);
        }
        Bt[(v * M + j) * D + d] = fj ? dval(v, j, d) : -b;
      }
#pragma unroll
      for (int k = 0; k < M; ++k) {
        Dt[(v * M + j) * M + k] = (fj || fixed_at(v, k)) ? (j == k ? 1.0 : 0.0) : Dr[k];
        if (v < S) Ot[(v * M + j) * M + k] = (fj || fixed_at(v + 1, k)) ? 0.0 : Or[k];
      }
    }
  }

  // LDL^T of the M x M block P (row-major, lower triangle) held in registers
  // (Lr), then x <- P^-1 x.  Lr[i][k] (k < i) ends as L[i][k] * delta_k and
  // inv[k] = 1 / delta_k.  Returns false on a non-positive pivot.
  __device__ static bool ldlt(double (&Lr)[M][M], double (&inv)[M]) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < M; ++j) {
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
        Lr[i][j] = s;
      }
    }
    return ok;
  }
  __device__ static void ldlt_apply(const double (&Lr)[M][M], const double (&inv)[M],
                                    double (&x)[M]) {
#pragma unroll
    for (int i = 0; i < M; ++i) {
      double s = x[i];
#pragma unroll
      for (int k = 0; k < i; ++k) s -= (Lr[i][k] * inv[k]) * x[k];
      x[i] = s;
    }
#pragma unroll
    for (int i = M - 1; i >= 0; --i) {
      double s = x[i] * inv[i];
#pragma unroll
      for (int k = i + 1; k < M; ++k) s -= (Lr[k][i] * inv[i]) * x[k];
      x[i] = s;
    }
  }

  // Twisted block LDL^T: two sweeps run at once and meet at the middle
  // vertex mid = (S+1)/2.  Lanes 0..31 sweep forward over v = 0..mid-1,
  // lanes 32..63 backward over v = S..mid+1 (the same recurrence on the
  // reversed chain, whose couplings are the transposed blocks: the two
  // groups run one instruction stream with per-lane addresses and strides).
  // In a group, lane c < M owns column c of the coupling block, lane M + d
  // right-hand side d.  Per step each active lane reads the Schur complement
  // S_v, factors it in registers and maps its column: Z_v[:, c] =
  // S_v^-1 P[:, c] (P = coupling to the next vertex of the sweep) or
  // z_v = S_v^-1 (b_v - Q^T z_prev) (Q = coupling from the previous one;
  // z_prev stays in registers); the coupling lanes then write column c of the
  // next Schur complement, S_next[:, c] = D_next[:, c] - P^T Z_v[:, c].  The
  // middle vertex combines both sweeps; back substitution
  // x_v = z_v - Z_v x_(toward mid) runs outward from it, both halves at once.
  // Fully fixed vertices skip the factorisation.  On exit dv holds every
  // vertex derivative (fixed values untouched).  flag()[0] |= 2 on a
  // non-positive pivot.
  __device__ void solve() {
    double* Dt = sm + lay->Dt;
    double* Ot = sm + lay->Ot;
    double* Zt = sm + lay->Zt;
    double* Bt = sm + lay->Bt;
    double* Tm = sm + lay->Tm;
    constexpr int MM = M * M;
    assemble();
    for (int i = lane; i < MM; i += kWave) Tm[i] = 0.0;
    __syncthreads();
    MTG_STAMP(3);
    const int mid = (S + 1) / 2;
    const int grp = lane >> 5, gl = lane & 31;
    const bool zl = gl < M;                    // coupling-column lane
    const bool rl = gl >= M && gl < M + D;     // right-hand-side lane
    const int c = zl ? gl : 0;
    const int d = rl ? gl - M : 0;
    const int nsteps = grp == 0 ? mid : S - mid;
    const int kmax = mid > S - mid ? mid : S - mid;
    double zprev[M];
#pragma unroll
    for (int i = 0; i < M; ++i) zprev[i] = 0.0;
    bool ok = true;
    for (int k = 0; k < kmax; ++k) {
      MTG_STAMP(100 + 2 * k);
      const bool act = k < nsteps && (zl || rl);
      // Vertex of this step and its neighbours along the sweep.
      const int v = grp == 0 ? k : S - k;
      const int vn = grp == 0 ? v + 1 : v - 1;       // next (toward mid)
      const int vp = grp == 0 ? v - 1 : v + 1;       // previous
      const bool has_prev = k > 0;
      // P = coupling v -> vn, Q = coupling vp -> v, as (base, row stride,
      // column stride) views of the stored O blocks (row-major O_u = u -> u+1).
      const int pb = (grp == 0 ? v : vn) * MM, qb = (grp == 0 ? (k > 0 ? vp : 0) : v) * MM;
      const int rs = grp == 0 ? M : 1, cs = grp == 0 ? 1 : M;
      const bool fixed = act && vertex_fixed(v);
      if (act && fixed) {
        // Identity block: z_v = b_v (the fixed values), Z_v = 0, no Schur term.
        if (rl) {
#pragma unroll
          for (int i = 0; i < M; ++i) zprev[i] = Bt[(v * M + i) * D + d];
        }
        if (zl) {
#pragma unroll
          for (int i = 0; i < M; ++i) Zt[v * MM + i * M + c] = 0.0;
        }
      } else if (act) {
        double Lr[M][M], inv[M], x[M], Pc[M][M], dn[M];
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
          for (int j = 0; j <= i; ++j) Lr[i][j] = Dt[v * MM + i * M + j];
        // Coupling lanes need P (next), rhs lanes Q (previous).
        const int ob = zl ? pb : qb;
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
          for (int j = 0; j < M; ++j) Pc[i][j] = Ot[ob + i * rs + j * cs];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          x[i] = zl ? Ot[pb + i * rs + c * cs] : Bt[(v * M + i) * D + d];
          dn[i] = Dt[(vn == mid && grp == 1 ? 0 : vn * MM) + i * M + c];
        }
        // Trailing mid for the backward sweep: its term goes to Tm, not D.
        __builtin_amdgcn_sched_barrier(0);
        if (rl && has_prev) {
#pragma unroll
          for (int i = 0; i < M; ++i) {
            double s = x[i];
#pragma unroll
            for (int m = 0; m < M; ++m) s -= Pc[m][i] * zprev[m];
            x[i] = s;
          }
        }
        ok = ldlt(Lr, inv) && ok;
        ldlt_apply(Lr, inv, x);
        if (rl) {
#pragma unroll
          for (int i = 0; i < M; ++i) {
            zprev[i] = x[i];
            Bt[(v * M + i) * D + d] = x[i];
          }
        }
        if (zl) {
#pragma unroll
          for (int i = 0; i < M; ++i) Zt[v * MM + i * M + c] = x[i];
          if (!vertex_fixed(vn)) {
            // S_next[:, c] = D_next[:, c] - P^T Z_v[:, c]; the backward
            // sweep's term at the middle is kept apart in Tm.
            const bool to_tm = grp == 1 && vn == mid;
#pragma unroll
            for (int i = 0; i < M; ++i) {
              double u = 0.0;
#pragma unroll
              for (int m = 0; m < M; ++m) u += Pc[m][i] * x[m];
              if (to_tm)
                Tm[i * M + c] = u;
              else
                Dt[vn * MM + i * M + c] = dn[i] - u;
            }
          }
        }
      }
      __syncthreads();
      MTG_STAMP(101 + 2 * k);
    }
    // Middle vertex: S_mid = D_mid (with the forward term) - Tm,
    // r_mid = b_mid - O_{mid-1}^T z_{mid-1} - O_mid z'_{mid+1}.
    if (!vertex_fixed(mid) && grp == 0 && (zl || rl)) {
      double Lr[M][M], inv[M], x[M];
#pragma unroll
      for (int i = 0; i < M; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) Lr[i][j] = Dt[mid * MM + i * M + j] - Tm[i * M + j];
      if (rl) {
#pragma unroll
        for (int i = 0; i < M; ++i) {
          double s = Bt[(mid * M + i) * D + d];
          if (mid > 0) {
#pragma unroll
            for (int m = 0; m < M; ++m)
              s -= Ot[(mid - 1) * MM + m * M + i] * Bt[((mid - 1) * M + m) * D + d];
          }
          if (mid < S) {
#pragma unroll
            for (int m = 0; m < M; ++m)
              s -= Ot[mid * MM + i * M + m] * Bt[((mid + 1) * M + m) * D + d];
          }
          x[i] = s;
        }
      } else {
#pragma unroll
        for (int i = 0; i < M; ++i) x[i] = 0.0;
      }
      ok = ldlt(Lr, inv) && ok;
      ldlt_apply(Lr, inv, x);
      if (rl) {
#pragma unroll
        for (int i = 0; i < M; ++i)
          if (!fixed_at(mid, i)) dv()[(mid * M + i) * D + d] = x[i];
      }
    }
    if (!ok) atomicOr(&flag()[0], 2);
    __syncthreads();
    MTG_STAMP(4);
    // Back substitution outward from the middle, lanes (i, d) per group:
    // x_v = z_v - Z_v x_(v toward mid).
    for (int k = 0; k < kmax; ++k) {
      const int nst = grp == 0 ? mid : S - mid;
      if (k < nst && gl < M * D) {
        const int v = grp == 0 ? mid - 1 - k : mid + 1 + k;
        const int vt = grp == 0 ? v + 1 : v - 1;
        const int i = gl / D, dd = gl % D;
        if (!fixed_at(v, i)) {
          double s = Bt[(v * M + i) * D + dd];
          const double* Zv = Zt + v * MM;
#pragma unroll
          for (int m = 0; m < M; ++m) s -= Zv[i * M + m] * dval(vt, m, dd);
          dv()[(v * M + i) * D + dd] = s;
        }
      }
      __syncthreads();
    }
    MTG_STAMP(5);
  }

  // Wave-wide sum (all 64 lanes receive it).
  __device__ static double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
    return x;
  }

  // Lanes over (segment, dimension, half) with e = [x_s; x_{s+1}] in
  // registers; half h covers coefficients / rows k in [hM, hM + M):
  //   c_s[d][k] = sum_j A(1)^-1[k][j] T_s^(j mod M - k) e_j   (coefficients,
  //               linear_impl:254-275; written to `out` when kCoeffs)
  //   cost     += e_k (H_s e)_k                               (computeCost,
  //               linear_impl:113-130: 0.5 c^T Q c == 0.5 e^T H e)
  // Returns computeCost() on every lane.
  template <bool kCoeffs>
  __device__ double coeffs_and_cost(const double* __restrict__ tab,
                                    double* __restrict__ out) const {
    (void)tab;
    double acc = 0.0;
    for (int item = lane; item < 2 * S * D; item += kWave) {
      const int h = item & 1;
      const int sd = item >> 1;
      const int s = sd / D, d = sd % D;
      double e[N];
#pragma unroll
      for (int j = 0; j < N; ++j) e[j] = dval(s + j / M, j % M, d);
      const double* tH = tabH() + h * M * N;
      const double* ph = pw() + s * PWN + (N - 1) + 1 - 2 * r;  // T^(1-2r+q)
      double cs = 0.0;
      // Rolled over rows (N table values live per row, not N*M).
#pragma unroll 1
      for (int kk = 0; kk < M; ++kk) {
        double hk = 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j) hk += tH[kk * N + j] * ph[kk + (j % M)] * e[j];
        cs += hk * dval(s + h, kk, d);
      }
      acc += cs;
      if (kCoeffs) {
        // T^(l - k) for l in [0, M), k = hM + kk.
        const double* tA = tabA() + h * M * N;
        const double* pws = pw() + s * PWN + (N - 1) - h * M;
#pragma unroll 1
        for (int kk = 0; kk < M; ++kk) {
          double c = 0.0;
#pragma unroll
          for (int j = 0; j < N; ++j) c += tA[kk * N + j] * pws[(j % M) - kk] * e[j];
          out[sd * N + h * M + kk] = c;
        }
      }
    }
    return 0.5 * wave_sum(acc);
  }

  __device__ double cost(const double* __restrict__ tab) const {
    return coeffs_and_cost<false>(tab, nullptr);
  }

  // sum_d e_s^T H_s(tau) e_s for segment s at time tau (fixed e): the part of
  // getCostAndGradientDerivative's J_d that depends on T_s.
  __device__ double seg_energy_at(int s, double tau) const {
    double acc = 0.0;
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
