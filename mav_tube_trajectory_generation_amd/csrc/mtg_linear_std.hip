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
// (tools/ubench/fp64_latency.hip), so the launch time at B = 1024 (one wave
// per SIMD) is the wave's instruction count, and this kernel is written to
// minimise it:
//   * free unknowns are the MF = M-1 non-position derivatives of the S-1
//     intermediate vertices; the system is block tridiagonal with MF x MF
//     blocks (4 x 4 at N = 10 instead of the generic kernel's pinned 5 x 5);
//   * assembly: lane (v, i) builds row i of A_v = H11(v-1) + H00(v), of the
//     coupling C_v = H01(v) and b_v[i] from the rows k, M+k of H(1) (loaded
//     straight from global memory with the inputs) and the powers of T;
//   * twisted block LDL^T: lanes 0.. sweep forward over v = 1..m-1, lanes
//     32.. backward over v = S-1..m+1, one instruction stream with per-lane
//     addresses; in a chain lane c < MF maps coupling column c, lane MF + d
//     right-hand side d, all through the same code (data decides the role:
//     r = u - G^T w, x = S^-1 r, out = a - G^T x); next-step operands are
//     prefetched before the barrier, so only the Schur complement read is
//     exposed;
//   * back substitution: one lane per (half, dimension) holds x in registers;
//   * coefficients and cost: lane (s, d), with f_j = e_j T^(j mod M) so that
//     cost = T^(1-2r) f^T H(1) f and c_k = T^-k (A(1)^-1 f)_k; the table
//     reads are wave-uniform (scalar loads).
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_device.h"
#include "mtg_internal.h"

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

// LDS carve-up in doubles (all offsets even: 16-byte aligned).
struct StdLayout {
  int pw;  // S * (2N-1): T_s^e, e in [-(N-1), N-1]
  int dv;  // (S+1) * M * D: vertex derivatives [v][k][d]
  int Sb;  // (S+1) * MF*MF: A_v, then Schur complements [v][i][j]
  int Cs;  // (S+1) * MF*MF: C_v = coupling v -> v+1 [v][i][j]
  int Zs;  // (S+1) * MF*MF: Z_v [v][i][c]
  int bz;  // (S+1) * MF * D: b_v, then z_v [v][i][d]
  int Tm;  // MF*MF: backward chain's Schur term at the middle vertex
  int n;
};

__host__ __device__ inline int even(int x) { return (x + 1) & ~1; }

__host__ __device__ inline StdLayout std_layout(int N, int S, int D) {
  const int M = N / 2, MF = M - 1, MM = MF * MF;
  StdLayout l;
  int o = 0;
  l.pw = o; o += even(S * (2 * N - 1));
  l.dv = o; o += even((S + 1) * M * D);
  l.Sb = o; o += even((S + 1) * MM);
  l.Cs = o; o += even((S + 1) * MM);
  l.Zs = o; o += even((S + 1) * MM);
  l.bz = o; o += even((S + 1) * MF * D);
  l.Tm = o; o += even(MM);
  l.n = o;
  return l;
}

}  // namespace

size_t linear_std_lds_bytes(int N, int S, int D) {
  return sizeof(double) * static_cast<size_t>(std_layout(N, S, D).n);
}

template <int N, int D>
__global__ __launch_bounds__(kWave) void linear_std_kernel(
    int S, int r, const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    const double* __restrict__ times, double* __restrict__ coeffs, double* __restrict__ cost,
    double* __restrict__ free_vals, int32_t* __restrict__ status) {
  constexpr int M = N / 2, MF = M - 1, MM = MF * MF, PWN = 2 * N - 1;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const StdLayout L = std_layout(N, S, D);
  double* pw = smem + L.pw;
  double* dv = smem + L.dv;
  double* Sb = smem + L.Sb;
  double* Cs = smem + L.Cs;
  double* Zs = smem + L.Zs;
  double* bz = smem + L.bz;
  double* Tm = smem + L.Tm;
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int nf = 2 * M + S - 1, np = (S - 1) * MF;
  const double* tb = times + b * S;
  const double* fb = fixed_vals + b * D * nf;
  const double* tH = tab;
  const double* tA = tab + N * N;

  // ---- Phase 0: inputs.  Times, fixed values and this lane's two rows of
  // H(1) for the assembly are all issued before the first use.
  const int nrows = (S - 1) * MF;
  const int arow_i = (lane < nrows ? lane : 0) % MF;
  double hk[N], hMk[N];  // rows k and M+k of H(1), k = arow_i + 1
#pragma unroll
  for (int j = 0; j < N; ++j) {
    hk[j] = tH[(arow_i + 1) * N + j];
    hMk[j] = tH[(M + arow_i + 1) * N + j];
  }
  const double t_l = lane < S ? tb[lane] : 1.0;
  bool bad = false;
  for (int i = lane; i < D * nf; i += kWave) {
    const int d = i / nf, f = i % nf;
    // Standard fixed order (linear_impl:171-252): vertex 0 derivatives
    // 0..M-1, intermediate positions, vertex S derivatives 0..M-1.
    int v, k;
    if (f < M) {
      v = 0; k = f;
    } else if (f < M + S - 1) {
      v = f - M + 1; k = 0;
    } else {
      v = S; k = f - (M + S - 1);
    }
    dv[(v * M + k) * D + d] = fb[i];
  }
  // Powers T_s^e by exact multiplication chains (1/T by rcp + Newton).
  for (int s = lane; s < S; s += kWave) {
    const double t = s == lane ? t_l : tb[s];
    bad = bad || !(t > 0.0) || !(t < 1e300);
    const double inv = rcp64(t);
    double* p = pw + s * PWN + (N - 1);
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
  for (int i = lane; i < MM; i += kWave) Tm[i] = 0.0;
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
  for (int row = lane; row < nrows; row += kWave) {
    const int v = row / MF + 1, i = row % MF, k = i + 1;
    if (row >= kWave) {  // rows beyond the first pass (S > 17): reload
#pragma unroll
      for (int j = 0; j < N; ++j) {
        hk[j] = tH[k * N + j];
        hMk[j] = tH[(M + k) * N + j];
      }
    }
    const double* pl = pw + (v - 1) * PWN + (N - 1) + 1 - 2 * r + k;  // left segment
    const double* pr = pw + v * PWN + (N - 1) + 1 - 2 * r + k;        // right segment
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
#pragma unroll
    for (int d = 0; d < D; ++d) {
      double s = cpos * dv[(v * M) * D + d];
      s = fma(cprev, dv[((v - 1) * M) * D + d], s);
      s = fma(cnext, dv[((v + 1) * M) * D + d], s);
      double e0 = 0.0, eS = 0.0;  // fully fixed neighbours (vertex 0 / S)
#pragma unroll
      for (int l = 1; l < M; ++l) {
        e0 = fma(hMk[l] * ql[l], dv[l * D + d], e0);
        eS = fma(hk[M + l] * qr[l], dv[(S * M + l) * D + d], eS);
      }
      s = fma(fl, e0, s);
      s = fma(fr, eS, s);
      bz[(v * MF + i) * D + d] = -s;
    }
#pragma unroll
    for (int j = 0; j < MF; ++j) {
      Sb[v * MM + i * MF + j] = Ar[j];
      Cs[v * MM + i * MF + j] = Cr[j];
    }
  }
  __syncthreads();
  MTG_STAMP(2);

  // ---- Phase 2: twisted block LDL^T over the intermediate vertices.
  const int m = S / 2;                 // middle vertex, 1 <= m <= S-1
  const int g = lane >> 5, q = lane & 31;
  const bool cpl = q < MF;             // coupling-column lane
  const bool rhs = q >= MF && q < MF + D;
  const int c = cpl ? q : 0, dd = rhs ? q - MF : 0;
  const int nst = g == 0 ? m - 1 : S - 1 - m;
  const int kmax = (m - 1) > (S - 1 - m) ? (m - 1) : (S - 1 - m);
  bool ok = true;
  double w[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) w[i] = 0.0;
  // Per-step operands of lane: G (P for coupling lanes, Q for rhs lanes, as
  // a strided view of C), u (P[:, c] or b_v[:, d]) and a (S_next[:, c]).
  double G[MF][MF], u[MF], a[MF];
  auto load_ops = [&](int k) {
    const int v = g == 0 ? 1 + k : S - 1 - k;
    const int vn = g == 0 ? v + 1 : v - 1;
    // forward: P = C_v, Q = C_{v-1};  backward: P = C_{v-1}^T, Q = C_v^T.
    int gb = g == 0 ? (cpl ? v : v - 1) : (cpl ? v - 1 : v);
    gb = gb < 0 ? 0 : gb;
    const int rs = g == 0 ? MF : 1, cs = g == 0 ? 1 : MF;
    const double* Gp = Cs + gb * MM;
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < MF; ++j) G[i][j] = Gp[i * rs + j * cs];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      u[i] = cpl ? Gp[i * rs + c * cs] : bz[(v * MF + i) * D + dd];
      const bool to_tm = g == 1 && vn == m;
      a[i] = to_tm ? 0.0 : Sb[vn * MM + i * MF + c];
    }
  };
  const bool lane_act = cpl || rhs;
  if (lane_act && nst > 0) load_ops(0);
  for (int k = 0; k < kmax; ++k) {
    MTG_STAMP(100 + 2 * k);
    if (lane_act && k < nst) {
      const int v = g == 0 ? 1 + k : S - 1 - k;
      const int vn = g == 0 ? v + 1 : v - 1;
      double Sv[MF][MF];
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) Sv[i][j] = Sb[v * MM + i * MF + j];
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
      double out[MF];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        double s = a[i];
#pragma unroll
        for (int j = 0; j < MF; ++j) s = fma(-G[j][i], x[j], s);
        out[i] = s;
      }
      if (cpl) {
        const bool to_tm = g == 1 && vn == m;
        double* dst = to_tm ? Tm : Sb + vn * MM;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          Zs[v * MM + i * MF + c] = x[i];
          dst[i * MF + c] = out[i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          bz[(v * MF + i) * D + dd] = x[i];
          w[i] = x[i];
        }
      }
      if (k + 1 < nst) load_ops(k + 1);
    }
    __syncthreads();
  }
  MTG_STAMP(3);
  // Middle vertex: S_m = (A_m - forward term) + Tm (= - backward term),
  // r_m = b_m - C_{m-1}^T z_{m-1} - C_m z'_{m+1}.
  if (g == 0 && rhs) {
    double Sv[MF][MF], rr[MF], x[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
#pragma unroll
      for (int j = 0; j <= i; ++j) Sv[i][j] = Sb[m * MM + i * MF + j] + Tm[i * MF + j];
      rr[i] = bz[(m * MF + i) * D + dd];
    }
    if (m - 1 >= 1) {
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < MF; ++j)
          rr[i] = fma(-Cs[(m - 1) * MM + j * MF + i], bz[((m - 1) * MF + j) * D + dd], rr[i]);
    }
    if (m + 1 <= S - 1) {
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < MF; ++j)
          rr[i] = fma(-Cs[m * MM + i * MF + j], bz[((m + 1) * MF + j) * D + dd], rr[i]);
    }
    ok = ldlt_solve<MF>(Sv, rr, x) && ok;
#pragma unroll
    for (int i = 0; i < MF; ++i) dv[(m * M + 1 + i) * D + dd] = x[i];
  }
  const bool not_spd = __any(!ok);
  __syncthreads();
  MTG_STAMP(4);

  // ---- Phase 3: back substitution outward from the middle, one lane per
  // (half, dimension): x_v = z_v - Z_v x_(toward m).
  if (q < D) {
    double x[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) x[i] = dv[(m * M + 1 + i) * D + q];
    const int n_back = g == 0 ? m - 1 : S - 1 - m;
    for (int k = 0; k < n_back; ++k) {
      const int v = g == 0 ? m - 1 - k : m + 1 + k;
      double xn[MF];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        double s = bz[(v * MF + i) * D + q];
#pragma unroll
        for (int j = 0; j < MF; ++j) s = fma(-Zs[v * MM + i * MF + j], x[j], s);
        xn[i] = s;
      }
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        x[i] = xn[i];
        dv[(v * M + 1 + i) * D + q] = xn[i];
      }
    }
  }
  __syncthreads();
  MTG_STAMP(5);

  // ---- Phase 4: coefficients and cost, lane (s, d).
  double acc = 0.0;
  auto coeff_cost = [&](int sd) {
    const int s = sd / D, d = sd % D;
    const double* ps = pw + s * PWN + (N - 1);
    double e[N], f[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      e[j] = dv[((s + j / M) * M + j % M) * D + d];
      f[j] = e[j] * ps[j % M];
    }
    // cost: 0.5 T^(1-2r) f^T H(1) f (0.5 applied after the reduction)
    double cs = 0.0;
#pragma unroll
    for (int a2 = 0; a2 < N; ++a2) {
      double h = tH[a2 * N + a2] * f[a2];
#pragma unroll
      for (int b2 = a2 + 1; b2 < N; ++b2) h = fma(2.0 * tH[a2 * N + b2], f[b2], h);
      cs = fma(h, f[a2], cs);
    }
    acc = fma(cs, ps[1 - 2 * r], acc);
    double* out = coeffs + b * per + static_cast<int64_t>(sd) * N;
    // Rows k < M of A(1)^-1 are diagonal (A(0) = diag(k!)).
#pragma unroll
    for (int k = 0; k < M; ++k) out[k] = tA[k * N + k] * e[k];
#pragma unroll
    for (int k = M; k < N; ++k) {
      double cc = 0.0;
#pragma unroll
      for (int j = 0; j < N; ++j) cc = fma(tA[k * N + j], f[j], cc);
      out[k] = cc * ps[-k];
    }
  };
  // First pass outside any loop so the wave-uniform table reads are not
  // hoisted and kept live across iterations (SGPR pressure).
  if (lane < S * D) coeff_cost(lane);
  for (int sd = lane + kWave; sd < S * D; sd += kWave) coeff_cost(sd);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, kWave);
  if (cost && lane == 0) cost[b] = 0.5 * acc;
  if (free_vals) {
    for (int i = lane; i < D * np; i += kWave) {
      const int d = i / np, p = i % np;
      const int v = p / MF + 1, kk = p % MF + 1;
      free_vals[b * D * np + i] = dv[(v * M + kk) * D + d];
    }
  }
  if (status && lane == 0) status[b] = not_spd ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK;
  MTG_STAMP(6);
}

template <int N, int D>
static hipError_t launch_std_nd(int S, int r, int64_t B, const double* tab, const double* df,
                                const double* times, double* coeffs, double* cost,
                                double* free_vals, int32_t* status, hipStream_t st) {
  const size_t lds = linear_std_lds_bytes(N, S, D);
  hipLaunchKernelGGL((linear_std_kernel<N, D>), dim3(static_cast<unsigned>(B)), dim3(kWave),
                     lds, st, S, r, tab, df, times, coeffs, cost, free_vals, status);
  return hipGetLastError();
}

template <int N>
static hipError_t launch_std_n(int D, int S, int r, int64_t B, const double* tab,
                               const double* df, const double* times, double* coeffs,
                               double* cost, double* free_vals, int32_t* status,
                               hipStream_t st) {
  switch (D) {
    case 1: return launch_std_nd<N, 1>(S, r, B, tab, df, times, coeffs, cost, free_vals, status, st);
    case 2: return launch_std_nd<N, 2>(S, r, B, tab, df, times, coeffs, cost, free_vals, status, st);
    case 3: return launch_std_nd<N, 3>(S, r, B, tab, df, times, coeffs, cost, free_vals, status, st);
    case 4: return launch_std_nd<N, 4>(S, r, B, tab, df, times, coeffs, cost, free_vals, status, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_linear_solve_std(const PlanDev& pl, int64_t B, const double* df,
                                   const double* times, double* coeffs, double* cost,
                                   double* free_vals, int32_t* status, hipStream_t st) {
  switch (pl.N) {
    case 4: return launch_std_n<4>(pl.D, pl.S, pl.r, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 6: return launch_std_n<6>(pl.D, pl.S, pl.r, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 8: return launch_std_n<8>(pl.D, pl.S, pl.r, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 10: return launch_std_n<10>(pl.D, pl.S, pl.r, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 12: return launch_std_n<12>(pl.D, pl.S, pl.r, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
