// mtg_linear_std.hip — batched linear solve specialised for the standard
// vertex pattern: start and end vertex fully fixed (all M = N/2 derivatives),
// every intermediate vertex fixing only its position.  This is the pattern
// of the reference's createRandomVertices / makeStartOrEnd (vertex.cpp:27-82,
// 147-153) and of BASELINE configs 1, 2, 4 and 5.  Other patterns run the
// generic kernel (mtg_device.h / mtg_kernels.hip).
//
// Same mathematics as the generic kernel (linear_impl:277-379, 254-275,
// 113-130 restated with the exact time scaling H_s(T) = T^(1-2r) S_T H(1) S_T,
// A_s^-1(T) = D_T^-1 A(1)^-1 S_T), organised for the shortest instruction
// stream on one gfx950 wave.  A single wave issues one FP64 FMA per ~4.5
// cycles with no extra dependency stall and v_rcp_f64 per 16 cycles
// (tools/ubench/fp64_latency.hip), so at B = 1024 (one wave per SIMD) the
// launch time is the wave's instruction count; every phase is written to
// minimise it:
//   * free unknowns are the MF = M-1 non-position derivatives of the S-1
//     intermediate vertices; the system is block tridiagonal with MF x MF
//     blocks (4 x 4 at N = 10 instead of the generic kernel's pinned 5 x 5);
//   * assembly: lane (v, i) builds row i of A_v = H11(v-1) + H00(v), of the
//     coupling C_v = H01(v) (and column i of C_v^T) and b_v[i] from the rows
//     k, M+k of H(1), loaded from global memory together with the inputs;
//   * twisted block LDL^T: lanes 0.. sweep forward over v = 1..m-1, lanes
//     32.. backward over v = S-1..m+1 in one instruction stream; in a chain
//     lane c < MF maps coupling column c, lane MF + d right-hand side d, all
//     through the same code (r = u - G^T w, x = S^-1 r, out = a - G^T x; the
//     data decides the role).  Every operand is a contiguous row (C_v and
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
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_device.h"
#include "mtg_internal.h"
#include "mtg_tables_gen.h"

namespace mtg {

namespace {

// One Newton step after v_rcp_f64: the seed is accurate to far more than
// the 27 bits one step needs to reach full FP64 precision.
__device__ inline double rcp64_1(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  const double e = fma(-d, r, 1.0);
  return fma(r, e, r);
}

// x = S^-1 r for a symmetric MF x MF block (lower triangle of S used) by
// LDL^T in registers.  Returns false on a non-positive pivot (the pivot is
// then replaced by 1 to keep the arithmetic finite).
template <int MF>
__device__ inline bool ldlt_solve(const double (&S)[MF][MF], const double (&r)[MF],
                                  double (&x)[MF]) {
  double Lr[MF][MF];  // Lr[i][j] = L_ij * d_j (i > j)
  double l[MF][MF];   // l[i][j]  = L_ij
  double inv[MF];
  bool ok = true;
#pragma unroll
  for (int j = 0; j < MF; ++j) {
    double dj = S[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) dj = fma(-Lr[j][k], l[j][k], dj);
    ok = ok && (dj > 0.0);
    inv[j] = rcp64_1(dj > 0.0 ? dj : 1.0);
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
  return ok;
}

// K doubles from / to LDS, 16-byte accesses for the pairs (callers keep the
// addresses of even-length rows 16-byte aligned).
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

// x + (x moved by DPP control CTRL), rows/banks masked as given; lanes with
// no source (or in disabled rows) add 0.
template <int CTRL, int RM, int BM>
__device__ inline double dpp_add(double x) {
  const long long u = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(u), CTRL, RM, BM, false);
  const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(u >> 32), CTRL, RM, BM, false);
  return x + __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) |
                                            static_cast<unsigned int>(lo));
}

// Value of lane j of this lane's quad (DPP quad_perm [j, j, j, j]).
__device__ inline double quad_bcast(double x, int j) {
  const long long u = __builtin_bit_cast(long long, x);
  int lo, hi;
  switch (j) {
    case 0:
      lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(u), 0x00, 0xf, 0xf, false);
      hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(u >> 32), 0x00, 0xf, 0xf, false);
      break;
    case 1:
      lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(u), 0x55, 0xf, 0xf, false);
      hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(u >> 32), 0x55, 0xf, 0xf, false);
      break;
    case 2:
      lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(u), 0xaa, 0xf, 0xf, false);
      hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(u >> 32), 0xaa, 0xf, 0xf, false);
      break;
    default:
      lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(u), 0xff, 0xf, 0xf, false);
      hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(u >> 32), 0xff, 0xf, 0xf, false);
      break;
  }
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) |
                                        static_cast<unsigned int>(lo));
}

// Sum over the 64 lanes (all active), returned wave-uniform: inclusive scan
// in rows of 16 (row_shr 1, 2, 4, 8), then row_bcast 15 and 31; lane 63
// holds the total.
__device__ inline double wave_sum_dpp(double x) {
  x = dpp_add<0x111, 0xf, 0xf>(x);
  x = dpp_add<0x112, 0xf, 0xf>(x);
  x = dpp_add<0x114, 0xf, 0xf>(x);
  x = dpp_add<0x118, 0xf, 0xf>(x);
  x = dpp_add<0x142, 0xa, 0xf>(x);
  x = dpp_add<0x143, 0xc, 0xf>(x);
  const long long u = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(u), 63);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(u >> 32), 63);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) |
                                        static_cast<unsigned int>(lo));
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
// even and blocks BS = MF * RS, so every row the kernel reads as a vector
// starts 16-byte aligned.
struct StdLayout {
  int pw;    // S * 2N: T_s^e at [s*2N + N + e], e in [-(N-1), N-1]
  int dv;    // (S+1) * D * MP: vertex derivatives [v][d][k] (MP = M rounded up even)
  int Sb;    // (S+1) * BS: A_v, then Schur complements, by rows
  int Cs;    // (S+1) * BS: C_v = coupling v -> v+1, [v][i][j]
  int Ct;    // (S+1) * BS: C_v^T
  int Zt;    // (S+1) * BS: Z_v^T (row c = column c of Z_v)
  int bz;    // (S+1) * D * RS: b_v, then z_v, [v][d][i]
  int Tm;    // BS: backward chain's Schur term at the middle vertex
  int junk;  // RS: sink for the rhs lanes' unused sweep output
  int n;
};

__host__ __device__ inline int even(int x) { return (x + 1) & ~1; }

__host__ __device__ inline StdLayout std_layout(int N, int S, int D) {
  const int M = N / 2, MF = M - 1, RS = even(MF), BS = MF * RS, MP = even(M);
  StdLayout l;
  int o = 0;
  l.pw = o; o += S * 2 * N;
  l.dv = o; o += (S + 1) * D * MP;
  l.Sb = o; o += (S + 1) * BS;
  l.Cs = o; o += (S + 1) * BS;
  l.Ct = o; o += (S + 1) * BS;
  l.Zt = o; o += (S + 1) * BS;
  l.bz = o; o += (S + 1) * D * RS;
  l.Tm = o; o += BS;
  l.junk = o; o += RS;
  l.n = o;
  return l;
}

}  // namespace

size_t linear_std_lds_bytes(int N, int S, int D) {
  return sizeof(double) * static_cast<size_t>(std_layout(N, S, D).n);
}

template <int N, int R, int D>
__global__ __launch_bounds__(kWave) void linear_std_kernel(
    int S, const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    const double* __restrict__ times, double* __restrict__ coeffs, double* __restrict__ cost,
    double* __restrict__ free_vals, int32_t* __restrict__ status) {
  constexpr int M = N / 2, MF = M - 1, RS = (MF + 1) & ~1, BS = MF * RS, PWP = 2 * N,
                MP = (M + 1) & ~1;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const StdLayout L = std_layout(N, S, D);
  double* pw = smem + L.pw;
  double* dv = smem + L.dv;
  double* Sb = smem + L.Sb;
  double* Cs = smem + L.Cs;
  double* Ct = smem + L.Ct;
  double* Zt = smem + L.Zt;
  double* bz = smem + L.bz;
  double* Tm = smem + L.Tm;
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int nf = 2 * M + S - 1, np = (S - 1) * MF;
  const double* tb = times + b * S;
  const double* fb = fixed_vals + b * D * nf;
  MTG_STAMP(0);

  // ---- Phase 0: inputs.  Times, fixed values and this lane's two rows of
  // H(1) for the assembly are all issued before the first use.
  const int nrows = (S - 1) * MF;
  double hk[N], hMk[N];  // rows k and M+k of H(1), k = (row mod MF) + 1
  auto load_rows = [&](int k) {
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      const double2 x = *reinterpret_cast<const double2*>(tab + k * N + j);
      const double2 y = *reinterpret_cast<const double2*>(tab + (M + k) * N + j);
      hk[j] = x.x;
      hk[j + 1] = x.y;
      hMk[j] = y.x;
      hMk[j + 1] = y.y;
    }
  };
  load_rows((lane < nrows ? lane : 0) % MF + 1);
  const double t_l = lane < S ? tb[lane] : 1.0;
  const double f_l = lane < D * nf ? fb[lane] : 0.0;
  bool bad = false;
  // Standard fixed order (linear_impl:171-252): vertex 0 derivatives
  // 0..M-1, intermediate positions, vertex S derivatives 0..M-1.
  auto put_fixed = [&](int i, double val) {
    int d = 0;  // i / nf without an integer division (D <= 4)
#pragma unroll
    for (int dd2 = 1; dd2 < D; ++dd2) d += i >= dd2 * nf ? 1 : 0;
    const int f = i - d * nf;
    int v, k;
    if (f < M) {
      v = 0; k = f;
    } else if (f < M + S - 1) {
      v = f - M + 1; k = 0;
    } else {
      v = S; k = f - (M + S - 1);
    }
    dv[(v * D + d) * MP + k] = val;
  };
  if (lane < D * nf) put_fixed(lane, f_l);
  for (int i = lane + kWave; i < D * nf; i += kWave) put_fixed(i, fb[i]);
  MTG_STAMP(7);
  // Powers T_s^e by exact multiplication chains (1/T by rcp + Newton).
  auto powers = [&](int s, double t) {
    bad = bad || !(t > 0.0) || !(t < 1e300);
    const double inv = rcp64(t);
    double* p = pw + s * PWP + N;
    double up = 1.0, dn = 1.0;
    p[0] = 1.0;
#pragma unroll
    for (int e = 1; e < N; ++e) {
      up *= t;
      dn *= inv;
      p[e] = up;
      p[-e] = dn;
    }
  };
  if (lane < S) powers(lane, t_l);
  for (int s = lane + kWave; s < S; s += kWave) powers(s, tb[s]);
  if (lane < BS) Tm[lane] = 0.0;
  const bool bad_time = __any(bad);
  __syncthreads();
  MTG_STAMP(1);

  const int64_t per = static_cast<int64_t>(S) * D * N;
  if (bad_time) {
    for (int i = lane; i < per; i += kWave) coeffs[b * per + i] = NAN;
    if (cost && lane == 0) cost[b] = NAN;
    if (status && lane == 0) status[b] = MTG_TRAJ_BAD_TIME;
    return;
  }

  // ---- Phase 1: assembly.  Lane (v, i): row i (derivative k = i+1) of
  // A_v = H11(v-1) + H00(v), C_v = H01(v) and b_v = -R_pf d_f restricted to
  // that row.  Exponent of H(a, b) at T: 1 - 2r + (a mod M) + (b mod M).
  auto assemble_row = [&](int row) {
    const int v = row / MF + 1, i = row % MF, k = i + 1;
    const double* pl = pw + (v - 1) * PWP + N + 1 - 2 * R + k;  // left segment
    const double* pr = pw + v * PWP + N + 1 - 2 * R + k;        // right segment
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
    const double fl = v == 1 ? 1.0 : 0.0, fr = v == S - 1 ? 1.0 : 0.0;
    const double cpos = fma(hMk[M], ql[0], hk[0] * qr[0]);  // p_v
    const double cprev = hMk[0] * ql[0];                     // p_{v-1}
    const double cnext = hk[M] * qr[0];                      // p_{v+1}
    double el[MF], er[MF];  // fully fixed neighbours (vertex 0 / S)
#pragma unroll
    for (int l = 1; l < M; ++l) {
      el[l - 1] = fl * (hMk[l] * ql[l]);
      er[l - 1] = fr * (hk[M + l] * qr[l]);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      double s = cpos * dv[(v * D + d) * MP];
      s = fma(cprev, dv[((v - 1) * D + d) * MP], s);
      s = fma(cnext, dv[((v + 1) * D + d) * MP], s);
#pragma unroll
      for (int l = 1; l < M; ++l) {
        s = fma(el[l - 1], dv[d * MP + l], s);
        s = fma(er[l - 1], dv[(S * D + d) * MP + l], s);
      }
      bz[(v * D + d) * RS + i] = -s;
    }
    lds_store(Sb + v * BS + i * RS, Ar);
    lds_store(Cs + v * BS + i * RS, Cr);
#pragma unroll
    for (int j = 0; j < MF; ++j) Ct[v * BS + j * RS + i] = Cr[j];
  };
  if (lane < nrows) assemble_row(lane);
  for (int row = lane + kWave; row < nrows; row += kWave) {
    load_rows(row % MF + 1);
    assemble_row(row);
  }
  __syncthreads();
  MTG_STAMP(2);

  // ---- Phase 2: twisted block LDL^T over the intermediate vertices.
  const int m = S / 2;  // middle vertex, 1 <= m <= S-1
  const int g = lane >> 5, q = lane & 31;
  const bool cpl = q < MF;  // coupling-column lane
  const bool rhs = q >= MF && q < MF + D;
  const int c = cpl ? q : 0, dd = rhs ? q - MF : 0;
  const int nst = g == 0 ? m - 1 : S - 1 - m;
  const int kmax = (m - 1) > (S - 1 - m) ? (m - 1) : (S - 1 - m);
  const int dir = g == 0 ? 1 : -1;
  const int v0 = g == 0 ? 1 : S - 1;
  // Per-lane operand rows at step 0 and their per-step strides.
  //   coupling lane c: G = P (forward C_v, backward C_{v-1}^T), u = P[:, c]
  //   (= row c of P^T), a = row c of S_next; x -> row c of Z_v^T,
  //   out -> row c of S_next (or Tm at the backward chain's last step).
  //   rhs lane d: G = Q (forward C_{v-1}, backward C_v^T), u = b_v[d];
  //   x -> z_v[d] (in place of b), out -> junk.
  const int gofs = cpl ? (g == 0 ? L.Cs + v0 * BS : L.Ct + (v0 - 1) * BS)
                       : (g == 0 ? L.Cs + (v0 - 1) * BS : L.Ct + v0 * BS);
  const int uofs = cpl ? (g == 0 ? L.Ct + v0 * BS : L.Cs + (v0 - 1) * BS) + c * RS
                       : L.bz + (v0 * D + dd) * RS;
  const int ustep = cpl ? dir * BS : dir * D * RS;
  const int aofs = L.Sb + (v0 + dir) * BS + c * RS;
  const int xofs = cpl ? L.Zt + v0 * BS + c * RS : uofs;
  const double rf = rhs ? 1.0 : 0.0;
  bool ok = true;
  double w[MF], G[MF][MF], u[MF], a[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) w[i] = 0.0;
  auto load_ops = [&](int k) {
    const double* Gp = smem + gofs + k * dir * BS;
#pragma unroll
    for (int i = 0; i < MF; ++i) lds_load(Gp + i * RS, G[i]);
    lds_load(smem + uofs + k * ustep, u);
    lds_load(smem + aofs + k * dir * BS, a);
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
        lds_load(Sb + v * BS + i * RS, row);
#pragma unroll
        for (int j = 0; j <= i; ++j) Sv[i][j] = row[j];
      }
      double rr[MF];
#pragma unroll
      for (int i = 0; i < MF; ++i) rr[i] = u[i];
      if (k > 0) {  // r = u - Q^T z_prev (w = 0 on coupling lanes)
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int j = 0; j < MF; ++j) rr[i] = fma(-G[j][i], w[j], rr[i]);
      }
      double x[MF];
      ok = ldlt_solve<MF>(Sv, rr, x) && ok;
      // The backward chain's last step stores its term alone (into Tm).
      const bool to_tm = cpl && g == 1 && k == nst - 1;
      const double af = to_tm ? 0.0 : 1.0;
      double out[MF];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        double s = a[i] * af;
#pragma unroll
        for (int j = 0; j < MF; ++j) s = fma(-G[j][i], x[j], s);
        out[i] = s;
      }
      const int xo = xofs + k * (cpl ? dir * BS : ustep);
      int oo = cpl ? aofs + k * dir * BS : L.junk;
      if (to_tm) oo = L.Tm + c * RS;
      lds_store(smem + xo, x);
      lds_store(smem + oo, out);
#pragma unroll
      for (int i = 0; i < MF; ++i) w[i] = x[i] * rf;
      if (k + 1 < nst) load_ops(k + 1);
    }
    __syncthreads();
  }
  MTG_STAMP(3);

  // ---- Phase 3: middle vertex (solved redundantly by both halves) and back
  // substitution outward from it, one lane per (half, dimension):
  //   S_m = (A_m - forward term) + Tm,  r_m = b_m - C_{m-1}^T z_{m-1} - C_m z'_{m+1},
  //   x_v = z_v - Z_v x_(toward m).
  // Lanes: for MF <= 4 a quad per (half g, dimension d), lane = g*32 + 4d + i
  // owning row i (the middle block is solved redundantly by all of them, so
  // no exchange precedes the back substitution, whose x_next rows are
  // broadcast inside the quad by DPP quad_perm); for MF = 5 one lane per
  // (g, d) holding all rows.
  constexpr bool kQuad = MF <= 4;
  const int pd = kQuad ? (q >> 2) : q;
  const int pi = kQuad ? (q & 3) : 0;
  const bool p_act = kQuad ? (pd < D && pi < MF) : (q < D);
  if (p_act) {
    const int d = pd;
    double Sv[MF][MF], rr[MF], x[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      double row[MF], tm[MF];
      lds_load(Sb + m * BS + i * RS, row);
      lds_load(Tm + i * RS, tm);
#pragma unroll
      for (int j = 0; j <= i; ++j) Sv[i][j] = row[j] + tm[j];
    }
    lds_load(bz + (m * D + d) * RS, rr);
    if (m >= 2) {
      double z[MF];
      lds_load(bz + ((m - 1) * D + d) * RS, z);
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        double row[MF];
        lds_load(Ct + (m - 1) * BS + i * RS, row);
#pragma unroll
        for (int j = 0; j < MF; ++j) rr[i] = fma(-row[j], z[j], rr[i]);
      }
    }
    if (m <= S - 2) {
      double z[MF];
      lds_load(bz + ((m + 1) * D + d) * RS, z);
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        double row[MF];
        lds_load(Cs + m * BS + i * RS, row);
#pragma unroll
        for (int j = 0; j < MF; ++j) rr[i] = fma(-row[j], z[j], rr[i]);
      }
    }
    ok = ldlt_solve<MF>(Sv, rr, x) && ok;
    MTG_STAMP(4);
    const int n_back = g == 0 ? m - 1 : S - 1 - m;
    const int vstep = g == 0 ? -1 : 1;
    if constexpr (kQuad) {
      double xi = x[0];  // own row of x_m
#pragma unroll
      for (int i = 1; i < MF; ++i) xi = pi == i ? x[i] : xi;
      if (g == 0) dv[(m * D + d) * MP + 1 + pi] = xi;
      double zr[MF], zz = 0.0;  // row pi of Z_v and z_v[pi][d] of the next step
      auto load_b = [&](int vv) {
#pragma unroll
        for (int c2 = 0; c2 < MF; ++c2) zr[c2] = Zt[vv * BS + c2 * RS + pi];
        zz = bz[(vv * D + d) * RS + pi];
      };
      int v = m + vstep;
      if (n_back > 0) load_b(v);
      for (int k = 0; k < n_back; ++k, v += vstep) {
        double xb[MF];
#pragma unroll
        for (int j = 0; j < MF; ++j) xb[j] = quad_bcast(xi, j);
        double s2 = zz;
#pragma unroll
        for (int j = 0; j < MF; ++j) s2 = fma(-zr[j], xb[j], s2);
        if (k + 1 < n_back) load_b(v + vstep);
        xi = s2;
        dv[(v * D + d) * MP + 1 + pi] = s2;
      }
    } else {
      if (g == 0) {
#pragma unroll
        for (int i = 0; i < MF; ++i) dv[(m * D + d) * MP + 1 + i] = x[i];
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
          dv[(v * D + d) * MP + 1 + i] = xn[i];
        }
      }
    }
  }
  const bool not_spd = __any(!ok);
  __syncthreads();
  MTG_STAMP(5);

  // ---- Phase 4: coefficients and cost, lane (s, d).
  constexpr CostW<N, R> kW{};
  constexpr AInvTab<N> kA{};
  double acc = 0.0;
  auto coeff_cost = [&](int sd) {
    const int s = sd / D, d = sd % D;
    const double* ps = pw + s * PWP + N;
    double e[N], f[N], h[N];
    {
      double e0[MP], e1[MP];
      lds_load(dv + (s * D + d) * MP, e0);
      lds_load(dv + ((s + 1) * D + d) * MP, e1);
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
    double cc[N];
#pragma unroll
    for (int i = 0; i < N; ++i) cc[i] = h[i] * ps[-i];
    double2* out = reinterpret_cast<double2*>(coeffs + b * per + static_cast<int64_t>(sd) * N);
#pragma unroll
    for (int i = 0; i < N / 2; ++i) out[i] = make_double2(cc[2 * i], cc[2 * i + 1]);
    double q2 = 0.0;
#pragma unroll
    for (int i = R; i < N; ++i) {
      double t = kW.v[i][i] * h[i];
#pragma unroll
      for (int j = i + 1; j < N; ++j) t = fma(2.0 * kW.v[i][j], h[j], t);
      q2 = fma(t, h[i], q2);
    }
    acc = fma(q2, ps[1 - 2 * R], acc);
  };
  if (lane < S * D) coeff_cost(lane);
  for (int sd = lane + kWave; sd < S * D; sd += kWave) coeff_cost(sd);
  const double J = wave_sum_dpp(acc);
  if (cost && lane == 0) cost[b] = J;
  if (free_vals) {
    for (int i = lane; i < D * np; i += kWave) {
      const int d = i / np, p = i % np;
      const int v = p / MF + 1, kk = p % MF + 1;
      free_vals[b * D * np + i] = dv[(v * D + d) * MP + kk];
    }
  }
  if (status && lane == 0) status[b] = not_spd ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK;
  MTG_STAMP(6);
}

template <int N, int R, int D>
static hipError_t launch_std_nrd(int S, int64_t B, const double* tab, const double* df,
                                 const double* times, double* coeffs, double* cost,
                                 double* free_vals, int32_t* status, hipStream_t st) {
  const size_t lds = linear_std_lds_bytes(N, S, D);
  hipLaunchKernelGGL((linear_std_kernel<N, R, D>), dim3(static_cast<unsigned>(B)), dim3(kWave),
                     lds, st, S, tab, df, times, coeffs, cost, free_vals, status);
  return hipGetLastError();
}

template <int N, int R>
static hipError_t launch_std_nr(int D, int S, int64_t B, const double* tab, const double* df,
                                const double* times, double* coeffs, double* cost,
                                double* free_vals, int32_t* status, hipStream_t st) {
  switch (D) {
    case 1: return launch_std_nrd<N, R, 1>(S, B, tab, df, times, coeffs, cost, free_vals, status, st);
    case 2: return launch_std_nrd<N, R, 2>(S, B, tab, df, times, coeffs, cost, free_vals, status, st);
    case 3: return launch_std_nrd<N, R, 3>(S, B, tab, df, times, coeffs, cost, free_vals, status, st);
    case 4: return launch_std_nrd<N, R, 4>(S, B, tab, df, times, coeffs, cost, free_vals, status, st);
    default: return hipErrorInvalidValue;
  }
}

template <int N>
static hipError_t launch_std_n(int r, int D, int S, int64_t B, const double* tab,
                               const double* df, const double* times, double* coeffs,
                               double* cost, double* free_vals, int32_t* status,
                               hipStream_t st) {
#define MTG_STD_R(RR)                                                                  \
  case RR:                                                                            \
    if constexpr (RR < N / 2)                                                         \
      return launch_std_nr<N, RR>(D, S, B, tab, df, times, coeffs, cost, free_vals,   \
                                  status, st);                                        \
    return hipErrorInvalidValue;
  switch (r) {
    MTG_STD_R(0)
    MTG_STD_R(1)
    MTG_STD_R(2)
    MTG_STD_R(3)
    MTG_STD_R(4)
    MTG_STD_R(5)
    default: return hipErrorInvalidValue;
  }
#undef MTG_STD_R
}

hipError_t launch_linear_solve_std(const PlanDev& pl, int64_t B, const double* df,
                                   const double* times, double* coeffs, double* cost,
                                   double* free_vals, int32_t* status, hipStream_t st) {
  switch (pl.N) {
    case 4: return launch_std_n<4>(pl.r, pl.D, pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 6: return launch_std_n<6>(pl.r, pl.D, pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 8: return launch_std_n<8>(pl.r, pl.D, pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 10: return launch_std_n<10>(pl.r, pl.D, pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 12: return launch_std_n<12>(pl.r, pl.D, pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg

#ifdef MTG_STAMPS
// Each HIP translation unit is its own code object: this kernel's stamps.
extern "C" int mtg_debug_stamps_std(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mtg_stamps),
                             sizeof(unsigned long long) * n) == hipSuccess ? 0 : -3;
}
#endif
