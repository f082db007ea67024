// mtg_tube_device.h — per-trajectory tube QCQP (PolynomialOptimizationConstrained,
// qcqp_impl) on one 64-lane workgroup, all state in LDS.
//
// Problem (qcqp_impl:476-788): free variables are every
// derivative 0..M-1 of every intermediate vertex in all 3 dimensions,
// objective x^T R_pp x + 2 d_f^T R_fp x, and per segment i the constraints
//   sphere  (i < S-1)     ||c_{i,N-1} - p_{i+1}||^2 - r2_i^2        <= 0
//   tube    j = 1..N-2    ||A_i c_ij + b_i||^2 - r1_i^2             <= 0
//   ends    j = 1..N-2    n_i.(p_s - c_ij) <= 0,  n_i.(c_ij - p_e) <= 0
// with c_ij the Bezier control points of the segment (qcqp_impl:267-474).
//
// MI355X formulation.  Control point j < M of segment i depends only on the
// start vertex i (row j of B_ul^-1), j >= M only on the end vertex i+1 (row
// j-M of B_lr^-1): every constraint touches ONE vertex's 3M variables, so its
// gradient is w (3-vector) (x) beta (M-vector) and its Hessian G (x) beta
// beta^T.  The Newton/KKT matrix is therefore block tridiagonal with 3M x 3M
// blocks (vertex coupling only through R_pp, which is the same M x M block in
// each dimension).  A primal-dual Mehrotra interior-point method (the
// oracle's algorithm, oracle/mtg_oracle.cpp TubeProblem::solveIPM) runs per
// trajectory: per iteration one block LDL^T factorisation (explicit unit
// L^-1 per block so the two solves are mat-vecs) and two solves.  State is
// sized to 40 KB of LDS at S = 10, N = 10, so 4 trajectories share a CU.
#pragma once
#include "mtg_device.h"

namespace mtg {

constexpr int kTubeD = 3;

// LDS per trajectory (doubles).  Sized for 4 workgroups per CU at the
// reference's S = 10, N = 10 (40 KB): the constant tables stay in global
// memory (L1/L2-resident), Bezier beta rows are derived from B_ul^-1, P is
// stored as its symmetric half, the constraint values and complementarity
// targets are recomputed where used, the step's control points share the
// dual-residual scratch, L_a^-1 is kept as a packed lower triangle whose
// diagonal holds 1 / pivot, and W_a = L_a^-1 C_a only for the block the
// factorisation is on (the solves apply C_a^T L_a^-T / L_a^-1 C_a instead).
struct TubeLayout {
  int bul;                // S*M*M  B_ul^-1 per segment (zero-snapped)
  int pw;                 // S*(2N-1) powers of the current times (overlays Li:
                          // setup and output only)
  int T;                  // S
  int geo;                // S*kGeo tube geometry per segment
  int fixv;               // 2*3*M start/end derivatives [end][d][m]
  int pos;                // (S+1)*3
  int Pd, Po, q;          // nv*M(M+1)/2 (packed symmetric), (nv-1)*M*M, nv*3M
  int x, dx, rd, rhs;     // nv*3M each (rhs at least 64)
  int cp, acc;            // S*N*3 each; acc also holds the step's control points
  int s, lam, ds, dl;     // ncon each
  int Li;                 // nv*BS(BS+1)/2 L_a^-1 packed by rows, diagonal = 1/pivot
  int W;                  // BS*BS  W_a of the current block, row-major
  int Wb;                 // BS*BS  V_a of the backward sweep's current block: ds/dl
                          // (dead during the factorisation) when they are large
                          // enough, else its own slot
  int Gc;                 // S*N*6  per control point: sum lam Hess + lam/s w w^T (sym)
  int red;                // 4: cross-wave reductions
  int ndouble;
  size_t bytes() const { return sizeof(double) * ndouble; }
};

constexpr int kGeo = 19;  // n[3] LL[9] L[3] mu n.ps n.pe r2^2

__host__ __device__ inline int tube_ncon(int N, int S) { return (S - 1) + 3 * S * (N - 2); }

__host__ __device__ inline TubeLayout make_tube_layout(int N, int S) {
  const int M = N / 2, BS = 3 * M, nv = S - 1, nc = tube_ncon(N, S);
  const int tri = BS * (BS + 1) / 2;
  TubeLayout l;
  int o = 0;
  l.bul = o;  o += S * M * M;
  l.T = o;    o += S;
  l.geo = o;  o += S * kGeo;
  l.fixv = o; o += 2 * 3 * M;
  l.pos = o;  o += (S + 1) * 3;
  l.Pd = o;   o += nv * M * (M + 1) / 2;
  l.Po = o;   o += (nv > 1 ? nv - 1 : 1) * M * M;
  l.q = o;    o += nv * BS;
  l.x = o;    o += nv * BS;
  l.dx = o;   o += nv * BS;
  l.rd = o;   o += nv * BS;
  l.rhs = o;  o += nv * BS > kWave ? nv * BS : kWave;  // also factor()'s dummy store slots
  l.cp = o;   o += S * N * 3;
  l.acc = o;  o += S * N * 3;
  l.s = o;    o += nc;
  l.lam = o;  o += nc;
  l.ds = o;   o += nc;
  l.dl = o;   o += nc;
  l.Li = o;
  l.pw = o;
  o += (nv * tri > S * (2 * N - 1) ? nv * tri : S * (2 * N - 1));
  l.W = o;    o += BS * BS;
  l.Gc = o;   o += S * N * 6;
  l.red = o;  o += 4;
  if (2 * nc >= BS * BS) {
    l.Wb = l.ds;  // ds, dl adjacent
  } else {
    l.Wb = o;
    o += BS * BS;
  }
  l.ndouble = o;
  return l;
}

template <int N>
struct Tube {
  static constexpr int M = N / 2;
  static constexpr int BS = 3 * M;
  static constexpr int PWN = 2 * N - 1;
  static constexpr int kTri = BS * (BS + 1) / 2;
  int S, r, nv, nc;
  const TubeLayout* L;
  double* sm;
  int lane;                          // lane in its wave
  const double* __restrict__ gtab;
  int tid, nthr, wv;                 // thread, threads (64 or 128), wave
  int redp = 0;                      // block_red's slot pair (alternates)
  // With two waves per trajectory the data-parallel phases use both; the
  // block LDL^T and the block solves run on wave 0 (wave 1 meets the same
  // barriers with nothing to do).  // plan table: H(1) N*N, A(1)^-1 N*N, C^-1 M*M (global)

  __device__ static int tri(int i, int k) { return i * (i + 1) / 2 + k; }  // k <= i
  __device__ double pd(int a, int j, int k) const {  // symmetric P block a
    return sm[L->Pd + a * (M * (M + 1) / 2) + (j >= k ? tri(j, k) : tri(k, j))];
  }
  __device__ static int gsym(int a, int e) {  // packed symmetric 3 x 3
    const int lo = a < e ? a : e, hi = a < e ? e : a;
    return lo == 0 ? hi : (lo == 1 ? 2 + hi : 5);
  }

  __device__ double* at(int off) const { return sm + off; }
  __device__ double pwr(int s, int e) const { return sm[L->pw + s * PWN + e + (N - 1)]; }

  // Control point (i, j) -> vertex it depends on.
  __device__ static int cp_vertex(int i, int j) { return j < M ? i : i + 1; }
  // beta_ij[m]: row j of B_ul^-1 (j < M) or row j-M of
  // B_lr^-1 = rowreverse(B_ul^-1) diag((-1)^m) (qcqp_impl:309-317).
  __device__ double beta_raw(int i, int j, int m) const {
    const double* b = sm + L->bul + i * M * M;
    if (j < M) return b[j * M + m];
    const double v = b[(M - 1 - (j - M)) * M + m];
    return (m & 1) ? -v : v;
  }
  __device__ double beta(int i, int j, int m) const { return beta_raw(i, j, m); }
  // Derivative m of vertex u in dimension d (fixed at the ends).
  __device__ double xval(const double* xv, int u, int d, int m) const {
    if (u == 0) return sm[L->fixv + (0 * 3 + d) * M + m];
    if (u == S) return sm[L->fixv + (1 * 3 + d) * M + m];
    return xv[((u - 1) * 3 + d) * M + m];
  }

  // Constraint index layout per segment (qcqp_impl:321-355):
  // [sphere if i < S-1] [tube j=1..N-2] [end j=1..N-2: side 0, side 1].
  __device__ int seg_base(int i) const { return i * (3 * N - 5); }
  __device__ int sphere_idx(int i) const { return seg_base(i); }
  __device__ int tube_idx(int i, int j) const {
    return seg_base(i) + (i < S - 1 ? 1 : 0) + (j - 1);
  }
  __device__ int end_idx(int i, int j, int side) const {
    return seg_base(i) + (i < S - 1 ? 1 : 0) + (N - 2) + 2 * (j - 1) + side;
  }
  // Inverse: constraint k -> (segment, control point, type 0 sphere / 1 tube
  // / 2 end side 0 / 3 end side 1).
  __device__ void con_of(int k, int* i, int* j, int* type) const {
    int seg = k / (3 * N - 5);
    if (seg > S - 1) seg = S - 1;
    int o = k - seg_base(seg);
    const int sp = seg < S - 1 ? 1 : 0;
    *i = seg;
    if (sp && o == 0) {
      *j = N - 1;
      *type = 0;
      return;
    }
    o -= sp;
    if (o < N - 2) {
      *j = o + 1;
      *type = 1;
      return;
    }
    o -= N - 2;
    *j = o / 2 + 1;
    *type = 2 + (o & 1);
  }

  // ------------------------------------------------------------------ setup
  // Loads inputs, builds B_ul^-1 (zero-snapped), tube geometry, P and q.
  // Times are those of problem b; the geometry (positions, fixed values,
  // control-point times, radii) that of trajectory bin (a trajectory's
  // several evaluation points share it).
  __device__ void setup(const double* __restrict__ tab, int64_t b, int64_t bin,
                        const double* __restrict__ positions,
                        const double* __restrict__ fixed_vals,
                        const double* __restrict__ times_cp,
                        const double* __restrict__ times,
                        const double* __restrict__ radii, int* bad) {
    const int NN = N * N;
    for (int i = tid; i < S; i += nthr) sm[L->T + i] = times[b * S + i];
    for (int i = tid; i < (S + 1) * 3; i += nthr) sm[L->pos + i] = positions[bin * (S + 1) * 3 + i];
    for (int i = tid; i < 3 * N; i += nthr) {
      // fixed_vals[d][end*M + m] -> fixv[end][d][m]
      const int d = i / N, e = (i % N) / M, m = i % M;
      sm[L->fixv + (e * 3 + d) * M + m] = fixed_vals[bin * 3 * N + i];
    }
    if (tid == 0) *bad = 0;
    __syncthreads();
    // B_ul^-1(T_cp) = C^-1 diag(T^l), snapped |x| < 1e-5 (qcqp_impl:299-307).
    for (int idx = tid; idx < S * M * M; idx += nthr) {
      const int i = idx / (M * M), k = (idx / M) % M, l = idx % M;
      const double tc = times_cp[bin * S + i];
      if (!(tc > 0.0)) atomicOr(bad, 1);
      double p = 1.0;
      for (int q = 0; q < l; ++q) p *= tc;
      double v = gtab[2 * NN + k * M + l] * p;
      if (v > -0.00001 && v < 0.00001) v = 0.0;
      sm[L->bul + idx] = v;
    }
    // Powers of the current times (H, A^-1, cost).
    if (!compute_powers()) atomicOr(bad, 1);
    // Tube geometry per segment (qcqp_impl:369-474).
    for (int i = tid; i < S; i += nthr) {
      const double* p0 = sm + L->pos + i * 3;
      const double* p1 = p0 + 3;
      double n[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
      const double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
      for (int k = 0; k < 3; ++k) n[k] /= nn;
      double A[9] = {1 - n[0] * n[0], -n[0] * n[1], -n[0] * n[2],
                     -n[0] * n[1], 1 - n[1] * n[1], -n[1] * n[2],
                     -n[0] * n[2], -n[1] * n[2], 1 - n[2] * n[2]};
      for (int k = 0; k < 9; ++k)
        if (A[k] > -0.000001 && A[k] < 0.000001) A[k] = 0.0;
      double bb[3] = {(n[0] * n[0] - 1) * p0[0] + n[0] * n[1] * p0[1] + n[0] * n[2] * p0[2],
                      n[0] * n[1] * p0[0] + (n[1] * n[1] - 1) * p0[1] + n[1] * n[2] * p0[2],
                      n[0] * n[2] * p0[0] + n[1] * n[2] * p0[1] + (n[2] * n[2] - 1) * p0[2]};
      for (int k = 0; k < 3; ++k)
        if (bb[k] > -0.000001 && bb[k] < 0.000001) bb[k] = 0.0;
      double* G = sm + L->geo + i * kGeo;
      for (int k = 0; k < 3; ++k) G[k] = n[k];
      for (int a = 0; a < 3; ++a)
        for (int c = 0; c < 3; ++c) {
          double s = 0.0;
          for (int k = 0; k < 3; ++k) s += A[k * 3 + a] * A[k * 3 + c];
          G[3 + a * 3 + c] = s;  // LL = A^T A
        }
      for (int c = 0; c < 3; ++c) {
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += bb[k] * A[k * 3 + c];
        G[12 + c] = 2.0 * s;  // L = 2 b^T A
      }
      const double r1 = radii[(bin * S + i) * 2 + 0];
      const double r2 = radii[(bin * S + i) * 2 + 1];
      G[15] = bb[0] * bb[0] + bb[1] * bb[1] + bb[2] * bb[2] - r1 * r1;  // mu
      const double rs = (i == 0) ? radii[(bin * S + 0) * 2 + 0] : radii[(bin * S + i - 1) * 2 + 1];
      double nps = 0.0, npe = 0.0;
      for (int k = 0; k < 3; ++k) {
        nps += n[k] * (p0[k] - n[k] * rs);
        npe += n[k] * (p1[k] + n[k] * r2);
      }
      G[16] = nps;
      G[17] = npe;
      G[18] = r2 * r2;
    }
    __syncthreads();
    // P = 2 R_pp (identical M x M blocks per dimension, symmetric half) and
    // q = 2 R_pf d_f.
    constexpr int MT = M * (M + 1) / 2;
    for (int idx = tid; idx < nv * MT; idx += nthr) {
      const int a = idx / MT, t2 = idx % MT;
      int j = 0;
      while (tri(j + 1, 0) <= t2) ++j;
      const int k = t2 - tri(j, 0);
      const int u = a + 1;  // vertex
      sm[L->Pd + idx] = 2.0 * (Hb(u - 1, 1, 1, j, k) + Hb(u, 0, 0, j, k));
    }
    for (int idx = tid; idx < (nv - 1) * M * M; idx += nthr) {
      const int a = idx / (M * M), j = (idx / M) % M, k = idx % M;
      sm[L->Po + idx] = 2.0 * Hb(a + 1, 0, 1, j, k);  // vertex a+1 -> a+2
    }
    for (int idx = tid; idx < nv * BS; idx += nthr) {
      const int a = idx / BS, d = (idx / M) % 3, j = idx % M;
      const int u = a + 1;
      double v = 0.0;
      if (u == 1)
        for (int k = 0; k < M; ++k) v += Hb(0, 1, 0, j, k) * sm[L->fixv + (0 * 3 + d) * M + k];
      if (u == S - 1)
        for (int k = 0; k < M; ++k) v += Hb(S - 1, 0, 1, j, k) * sm[L->fixv + (1 * 3 + d) * M + k];
      sm[L->q + idx] = 2.0 * v;
    }
    __syncthreads();
  }

  __device__ double Hb(int s, int ab, int bb, int j, int k) const {
    return gtab[(ab * M + j) * N + bb * M + k] * pwr(s, 1 - 2 * r + j + k);
  }

  // Powers T_s^e, e in [-(N-1), N-1], of the current times into pw (which
  // overlays the factor storage: call before the IPM and again for the
  // outputs).  Returns false if a time is not a valid segment time.
  __device__ bool compute_powers() {
    bool ok = true;
    for (int idx = tid; idx < S * PWN; idx += nthr) {
      const int s = idx / PWN;
      const int e = idx % PWN - (N - 1);
      const double t = sm[L->T + s];
      if (!(t > 0.0) || !(t < 1e300)) ok = false;
      const double base = e < 0 ? 1.0 / t : t;
      const int n = e < 0 ? -e : e;
      double p = 1.0;
      for (int q = 0; q < n; ++q) p *= base;
      sm[L->pw + idx] = p;
    }
    return ok;
  }

  // --------------------------------------------------------- control points
  // One lane per control point (i, j): its beta row is formed once and used
  // for the three dimensions (same products and summation order as one
  // lane per (i, j, d)).
  __device__ void control_points(const double* xv, int out) {
    for (int cpi = tid; cpi < S * N; cpi += nthr) {
      const int i = cpi / N, j = cpi % N;
      const int u = cp_vertex(i, j);
      double bt[M];
#pragma unroll
      for (int m = 0; m < M; ++m) bt[m] = beta(i, j, m);
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        double c = 0.0;
#pragma unroll
        for (int m = 0; m < M; ++m) c += bt[m] * xval(xv, u, d, m);
        sm[out + cpi * 3 + d] = c;
      }
    }
  }
  // Same, for a step direction (fixed vertices contribute zero).
  __device__ void control_point_steps(const double* dxv, int out) {
    for (int cpi = tid; cpi < S * N; cpi += nthr) {
      const int i = cpi / N, j = cpi % N;
      const int u = cp_vertex(i, j);
      const bool fr = u > 0 && u < S;
      const double* xu = dxv + ((fr ? u : 1) - 1) * 3 * M;
      double bt[M];
#pragma unroll
      for (int m = 0; m < M; ++m) bt[m] = beta(i, j, m);
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        double c = 0.0;
        if (fr) {
#pragma unroll
          for (int m = 0; m < M; ++m) c += bt[m] * xu[d * M + m];
        }
        sm[out + cpi * 3 + d] = c;
      }
    }
  }

  // Residual g_k and gradient w_k (w.r.t. the control point) of constraint k
  // at control points `cpo`.
  __device__ double con_eval(int k, int cpo, double w[3]) const {
    int i, j, type;
    con_of(k, &i, &j, &type);
    const double* c = sm + cpo + (i * N + j) * 3;
    const double* G = sm + L->geo + i * kGeo;
    if (type == 0) {  // sphere around vertex i+1 (qcqp_impl:357-365)
      const double* p = sm + L->pos + (i + 1) * 3;
      double g = -G[18];
      for (int d = 0; d < 3; ++d) {
        const double e = c[d] - p[d];
        g += e * e;
        w[d] = 2.0 * e;
      }
      return g;
    }
    if (type == 1) {  // tube (qcqp_impl:369-429): c^T LL c + L c + mu
      double g = G[15];
      for (int a = 0; a < 3; ++a) {
        double llc = 0.0;
        for (int e = 0; e < 3; ++e) llc += G[3 + a * 3 + e] * c[e];
        g += c[a] * llc + G[12 + a] * c[a];
        w[a] = 2.0 * llc + G[12 + a];
      }
      return g;
    }
    // end caps (qcqp_impl:431-474)
    const double sgn = type == 2 ? -1.0 : 1.0;
    double nc = 0.0;
    for (int d = 0; d < 3; ++d) {
      nc += G[d] * c[d];
      w[d] = sgn * G[d];
    }
    return type == 2 ? (G[16] - nc) : (nc - G[17]);
  }

  // Every constraint on control point (i, j) at control points `cpo`, in
  // con_at's slots: slot 0 the tube (1 <= j <= N-2) or the sphere (j = N-1,
  // i < S-1), slots 1 and 2 the end caps (1 <= j <= N-2); k[t] = -1 marks an
  // absent slot.  con_eval's arithmetic without its per-constraint decode and
  // type branches (round 5): the tube, sphere and cap formulas run on every
  // lane and slot 0 selects, so a wave whose lanes hold different j does not
  // serialise the types.  h0 = 1 selects slot 0's Hessian factor 2 I
  // (sphere) over 2 LL (tube); the caps' is 0.
  __device__ void cp_cons(int i, int j, int cpo, int (&k)[3], double (&g)[3],
                          double (&w)[3][3], bool& sph) const {
    const double* cv = sm + cpo + (i * N + j) * 3;
    const double* G = sm + L->geo + i * kGeo;
    const bool mid = j >= 1 && j <= N - 2;
    sph = j == N - 1 && i < S - 1;
    const int eb = seg_base(i) + (i < S - 1 ? 1 : 0);
    k[0] = mid ? eb + (j - 1) : (sph ? seg_base(i) : -1);
    k[1] = mid ? eb + (N - 2) + 2 * (j - 1) : -1;
    k[2] = mid ? eb + (N - 2) + 2 * (j - 1) + 1 : -1;
    const double c[3] = {cv[0], cv[1], cv[2]};
    double gt = G[15], wt[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {  // tube (qcqp_impl:369-429)
      double llc = 0.0;
#pragma unroll
      for (int e = 0; e < 3; ++e) llc += G[3 + a * 3 + e] * c[e];
      gt += c[a] * llc + G[12 + a] * c[a];
      wt[a] = 2.0 * llc + G[12 + a];
    }
    const double* p = sm + L->pos + (i + 1) * 3;  // sphere (qcqp_impl:357-365)
    double gs = -G[18], ws[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const double e = c[d] - p[d];
      gs += e * e;
      ws[d] = 2.0 * e;
    }
    g[0] = sph ? gs : gt;
    double nc = 0.0;  // end caps (qcqp_impl:431-474)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      w[0][d] = sph ? ws[d] : wt[d];
      nc += G[d] * c[d];
      w[1][d] = -1.0 * G[d];
      w[2][d] = 1.0 * G[d];
    }
    g[1] = G[16] - nc;
    g[2] = nc - G[17];
  }

  // Hessian factor of constraint type (w.r.t. the control point): 2 I, 2 LL, 0.
  __device__ double con_hess(int type, int i, int a, int e) const {
    if (type == 0) return a == e ? 2.0 : 0.0;
    if (type == 1) return 2.0 * sm[L->geo + i * kGeo + 3 + a * 3 + e];
    return 0.0;
  }

  // Constraint slot t (0..2) acting on control point (i, j): returns its
  // index or -1.  Slots: sphere on j = N-1 (i < S-1); tube / end side 0 /
  // end side 1 on j = 1..N-2.  (Fixed-slot form: no runtime-indexed arrays,
  // which hipcc would place in scratch.)
  __device__ int con_at(int i, int j, int t) const {
    if (j == N - 1) return (t == 0 && i < S - 1) ? sphere_idx(i) : -1;
    if (j < 1 || j > N - 2) return -1;
    return t == 0 ? tube_idx(i, j) : end_idx(i, j, t - 1);
  }

  // P x + q for vertex block entry idx (a, d, m).
  __device__ double Pxq(const double* xv, int idx) const {
    const int a = idx / BS, d = (idx / M) % 3, m = idx % M;
    double v = sm[L->q + idx];
    for (int k = 0; k < M; ++k) {
      v += pd(a, m, k) * xv[(a * 3 + d) * M + k];
      if (a > 0) v += sm[L->Po + (a - 1) * M * M + k * M + m] * xv[((a - 1) * 3 + d) * M + k];
      if (a < nv - 1) v += sm[L->Po + a * M * M + m * M + k] * xv[((a + 1) * 3 + d) * M + k];
    }
    return v;
  }

  // Sum over the control points of vertex u=a+1 of beta[m] * acc[cp][d]
  // (the a_k-weighted sums of the dual residual / right-hand side).
  __device__ double gather_cp(int acc_off, int a, int d, int m) const {
    const int u = a + 1;
    double v = 0.0;
    for (int j = M; j < N; ++j) v += beta(u - 1, j, m) * sm[acc_off + ((u - 1) * N + j) * 3 + d];
    for (int j = 0; j < M; ++j) v += beta(u, j, m) * sm[acc_off + (u * N + j) * 3 + d];
    return v;
  }

  // --------------------------------------------------------- KKT assembly
  // Per control point: G = sum_k lam_k Hess_k + (lam_k / s_k) w_k w_k^T over
  // the (at most 3) constraints acting on it (ipm's residual pass).  The
  // diagonal KKT block of vertex a is K_a = I_3 (x) Pd_a + sum_cp G_cp (x)
  // beta_cp beta_cp^T; its columns are built in registers by factor().

  // 1 if x == 0 else 0 (integer arithmetic, see is_zero).
  __device__ static int izero(int x) { return ((x | -x) >> 31) + 1; }
  // 1.0 if x == 0 else 0.0, by integer arithmetic: a compare would yield a
  // lane mask (SGPR pair) that the compiler hoists and keeps live.
  __device__ static double is_zero(int x) {
    return static_cast<double>(((x | -x) >> 31) + 1);
  }

  // 64-bit lane broadcast (uniform source lane).
  __device__ static double bcast(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(b & 0xffffffffLL), src);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), src);
    return __longlong_as_double((static_cast<long long>(hi) << 32) |
                                (static_cast<unsigned int>(lo)));
  }

  // ----------------------------------------------------- lane organisation
  // For BS <= 16 the wave is 4 rows of 16 lanes: lane (g, c) = 16 g + c.
  // Dot products and the S_a update are split over the rows (every row takes
  // every 4th term) and summed with the gfx950 cross-row swaps; in the
  // elimination row g holds role g (0 = S_a, 1 = identity, 2 = C_a, 3 idle).
  // For BS > 16 (N = 12) a single group: roles at lanes 0, BS, 2BS.
  static constexpr int kNG = BS <= 16 ? 4 : 1;
  __device__ int grp() const { return kNG == 4 ? lane >> 4 : 0; }
  __device__ int col_of() const { return kNG == 4 ? (lane & 15) : lane % BS; }
  __device__ int role_of() const {
    const int c = kNG == 4 ? (lane & 15) : lane % BS;
    const int r = kNG == 4 ? (lane >> 4) : lane / BS;
    return (c >= BS || r > 2) ? 3 : r;
  }

  __device__ static double join(unsigned lo, unsigned hi) {
    return __longlong_as_double((static_cast<long long>(hi) << 32) | lo);
  }
  // x + x(lane ^ 32) and x + x(lane ^ 16): v_permlane{32,16}_swap with the
  // value as both operands leaves {x(lane), x(partner)} in the two results.
  __device__ static double xsum32(double x) {
    const long long b = __double_as_longlong(x);
    const unsigned lo = static_cast<unsigned>(b), hi = static_cast<unsigned>(b >> 32);
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return join(l[0], h[0]) + join(l[1], h[1]);
  }
  __device__ static double xsum16(double x) {
    const long long b = __double_as_longlong(x);
    const unsigned lo = static_cast<unsigned>(b), hi = static_cast<unsigned>(b >> 32);
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return join(l[0], h[0]) + join(l[1], h[1]);
  }
  // Sum over the kNG rows (the result is in every row).  Call with all 64
  // lanes active.
  __device__ static double rows_sum(double x) {
    if constexpr (kNG == 4) return xsum16(xsum32(x));
    return x;
  }

  // --------------------------------------------------------- factorisation
  // Twisted block LDL^T of the block-tridiagonal KKT matrix.  With two waves,
  // wave 0 eliminates blocks 0 .. m-1 forward while wave 1 eliminates
  // nv-1 .. m+1 backward, then wave 0 the middle block m = nv / 2 with both
  // Schur terms (one wave: m = nv - 1, a plain forward sweep):
  //   forward   S_a = K_a - W_{a-1}^T D_{a-1}^-1 W_{a-1},  W_a = L_a^-1 C_a,
  //   backward  S_a = K_a - V_{a+1}^T D_{a+1}^-1 V_{a+1},  V_a = L_a^-1 C_{a-1}^T,
  //   middle    S_m = K_m - W_{m-1}^T D^-1 W_{m-1} - V_{m+1}^T D^-1 V_{m+1},
  // C_a = I_3 (x) Po_a coupling block a to a+1, S_a = L_a D_a L_a^T.
  // The constraint and Schur terms of S_a are accumulated with the rows
  // sharing the sums (control points q = g + 4k, W rows t = g + 4k), then
  // the elimination runs on [S_a | I | C] held column-per-lane in registers;
  // the pivot column is broadcast with v_readlane, so it needs no LDS traffic
  // and no barrier inside.  Afterwards the identity lanes hold L_a^-1 (unit
  // lower) and the coupling lanes W_a / V_a; the pivots are D_a.  S_a is SPD
  // (no pivoting); a non-positive pivot sets *fail.  W is kept for the block
  // being eliminated only, V likewise in Wb (normally the ds / dl buffers,
  // dead from the step update to the next direction).
  __device__ int mid() const { return nthr > kWave ? nv / 2 : nv - 1; }

  // reg > 0: the retry after a non-positive pivot (ipm()): every block's
  // S_a lanes scale their diagonal entry by 1 + reg (|S_ii| reg added), a
  // diagonal regularisation of the block elimination (the oracle adds
  // reg K_ii to its dense K; both steps converge to the same optimum).
  __device__ void factor(int* fail, bool with_constraints, double reg = 0.0) {
    const double* Gcp = sm + L->Gc;
    int bad = 0;
    unsigned long long tf = 0;
    MTG_TACC(511, tf);
    const int g = grp();
    const int cc0 = col_of() < BS ? col_of() : BS - 1;  // clamped on pad lanes
    const int role0 = role_of();
    // Per-lane target of the unused stores (rhs is dead during factor():
    // written by direction() / the start system afterwards).
    const int dummy = L->rhs + lane;
    const int m = mid(), nb = nv - 1 - m;
    const bool bw = wv == 1;  // wave-uniform
    for (int st = 0; st <= m; ++st) {
      // The middle step reads wave 1's last V and L^-1 block: the one
      // barrier of the sweep (workgroup-uniform condition).
      if (st == m) __syncthreads();
      // This wave's block: wave 0 a = st (the middle at st = m), wave 1
      // a = nv - 1 - st while st < nb.
      const bool act = bw ? st < nb : true;
      const int a = bw ? nv - 1 - st : st;
      const bool midb = !bw && st == m;
      const bool sf = !bw && a > 0;                         // W_{a-1} term
      const bool sb = bw ? st > 0 : (midb && m < nv - 1);   // V_{a+1} term
      const int u = a + 1;  // vertex
      double col[BS], acc[BS];
      // Opaque per iteration: keeps the compiler from hoisting the 0/1
      // factors below out of the loop as live lane masks (SGPR pressure).
      int cc = cc0;
      asm volatile("" : "+v"(cc));
      const int d2 = cc / M, m2 = cc % M;
      const int role = (role0 == 2 && midb) ? 3 : role0;
      // Roles enter as exact 0/1 factors (VGPR values: no lane masks kept
      // live); loads are unconditional with clamped indices.
      const double r0 = is_zero(role), r1 = is_zero(role - 1), r2 = is_zero(role - 2);
      double dpiv = 1.0;
      if (act) {  // ---- assemble and eliminate block a
      {
        // Coupling columns: C_a = I_3 (x) Po_a (forward), C_{a-1}^T (backward).
        const int pb = bw ? (a > 0 ? a - 1 : 0) : (a < nv - 1 ? a : 0);
        const double* Po = sm + L->Po + pb * M * M;
        const int pt = bw ? 1 : M, ps = bw ? M : 1;
        double ind[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) ind[d] = is_zero(d - d2);
#pragma unroll
        for (int mm = 0; mm < M; ++mm) {
          const double v = pd(a, mm, m2) * r0 + Po[mm * pt + m2 * ps] * r2;
#pragma unroll
          for (int d = 0; d < 3; ++d) col[d * M + mm] = v * ind[d];
        }
#pragma unroll
        for (int i = 0; i < BS; ++i) col[i] += r1 * is_zero(i - cc);
#pragma unroll
        for (int i = 0; i < BS; ++i) acc[i] = 0.0;
      }
      MTG_TACC(220, tf);
      if (with_constraints) {
        // This row's control points of vertex u (q < M: segment u-1,
        // j = q + M, rows of B_lr^-1; q >= M: segment u, j = q - M):
        // acc += G[d][d2] beta[m] beta[m2].
#pragma unroll
        for (int k = 0; k < (N + kNG - 1) / kNG; ++k) {
          const int q0 = g + kNG * k;
          const double wq = static_cast<double>(q0 < N);
          const int q = q0 < N ? q0 : N - 1;
          const bool lo = q < M;
          const int seg = lo ? u - 1 : u;
          const double sg = lo ? -1.0 : 1.0;  // B_lr^-1 = rowreverse(B_ul^-1) diag((-1)^m)
          const double* bro = sm + L->bul + seg * M * M + (lo ? M - 1 - q : q - M) * M;
          const int cpi = seg * N + (lo ? q + M : q - M);
          double bt[M];
#pragma unroll
          for (int mm = 0; mm < M; ++mm) bt[mm] = (mm & 1) ? sg * bro[mm] : bro[mm];
          const double bm = ((m2 & 1) ? sg * bro[m2] : bro[m2]) * wq;
#pragma unroll
          for (int d = 0; d < 3; ++d) {
            const double gd = Gcp[cpi * 6 + gsym(d, d2)] * bm;
#pragma unroll
            for (int mm = 0; mm < M; ++mm) acc[d * M + mm] = fma(gd, bt[mm], acc[d * M + mm]);
          }
        }
      }
      MTG_TACC(221, tf);
      // acc -= sum_t X[t][:] dinv[t] X[t][c] over this row's t, X = W_{a-1}
      // or V_{a+1} with dinv on the diagonal of the neighbour's packed L^-1.
      // Row t + kNG is loaded while row t is applied (sched barriers keep
      // the loads ahead: otherwise they are issued one pair at a time).
      auto schur = [&](const double* Wp, const double* Lp) {
        constexpr int KT = (BS + kNG - 1) / kNG;
        double wr[BS], wn[BS], wc, dt, wcn = 0.0, dtn = 0.0;
        auto row = [&](int k, double* w, double* c, double* d) {
          const int t0 = g + kNG * k;
          const int t = t0 < BS ? t0 : BS - 1;
#pragma unroll
          for (int i = 0; i < BS; ++i) w[i] = Wp[t * BS + i];
          *c = Wp[t * BS + cc];
          *d = Lp[tri(t, t)] * static_cast<double>(t0 < BS);
        };
        row(0, wr, &wc, &dt);
#pragma unroll
        for (int k = 0; k < KT; ++k) {
          if (k + 1 < KT) row(k + 1, wn, &wcn, &dtn);
          __builtin_amdgcn_sched_barrier(0);
          const double w = wc * dt;
#pragma unroll
          for (int i = 0; i < BS; ++i) acc[i] = fma(-wr[i], w, acc[i]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < BS; ++i) wr[i] = wn[i];
          wc = wcn;
          dt = dtn;
        }
      };
      if (sf) schur(sm + L->W, sm + L->Li + (a - 1) * kTri);
      if (sb) schur(sm + L->Wb, sm + L->Li + (a + 1) * kTri);
#pragma unroll
      for (int i = 0; i < BS; ++i) col[i] = fma(rows_sum(acc[i]), r0, col[i]);
      if (reg > 0.0) {  // workgroup-uniform: the retry only
#pragma unroll
        for (int i = 0; i < BS; ++i) col[i] = fma(reg * r0 * is_zero(i - cc), fabs(col[i]), col[i]);
      }
      // Forward elimination (below the pivot) on all columns at once; the
      // pivot column is broadcast with v_readlane.
      MTG_TACC(222, tf);
#pragma unroll
      for (int j = 0; j < BS; ++j) {
        const double piv = bcast(col[j], j);
        dpiv = lane == j ? piv : dpiv;  // lane j: its own pivot
        if (j == BS - 1) break;
        const double f = col[j] * rcp64(piv > 0.0 ? piv : 1.0);
        // All broadcasts of the step first, then the updates.
        double pc[BS];
#pragma unroll
        for (int i = j + 1; i < BS; ++i) pc[i] = bcast(col[i], j);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = j + 1; i < BS; ++i) col[i] = fma(-pc[i], f, col[i]);
      }
      bad |= __ballot(lane < BS && !(dpiv > 0.0)) != 0;
      MTG_TACC(223, tf);
      }  // ---- act
      // S_a lanes store 1 / pivot on the diagonal of the packed L_a^-1, the
      // identity lanes its strictly lower columns, the coupling lanes W_a or
      // V_a (replacing the previous block's, which every lane of the wave has
      // read by the barrier).  Offsets are selected per lane with integer
      // masks (no branches), unused stores go to a per-lane dummy slot.
      // No barrier: a wave's blocks are its own until the middle step (its
      // W / V reads of this step are issued before these stores, and LDS
      // operations of a wave complete in issue order).
      asm volatile("" ::: "memory");
      if (act) {
        const int li = L->Li + a * kTri;
        const int wo = bw ? L->Wb : L->W;
        const int s0 = -izero(role), s1 = -izero(role - 1), s2 = -izero(role - 2);
        sm[((li + tri(cc, cc)) & s0) | (dummy & ~s0)] = rcp64(dpiv > 0.0 ? dpiv : 1.0);
#pragma unroll
        for (int i = 0; i < BS; ++i) {
          const int a1 = s1 & ((cc - i) >> 31);  // identity lane, i > cc
          const int o = ((li + tri(i, cc)) & a1) | ((wo + i * BS + cc) & s2) |
                        (dummy & ~(a1 | s2));
          sm[o] = col[i];
        }
      }
      asm volatile("" ::: "memory");
      MTG_TACC(224, tf);
    }
    if (bad && lane == 0) *fail = 1;
  }

  // Solve K out = rhs with the twisted factors (rhs overwritten by y).
  // Row i of a block belongs to lanes (g, i) of every row g, which share its
  // dot products; the vectors of the recurrence stay in registers (lane k
  // holds entry k) and move between lanes with __shfl.  W and V are not
  // stored; the coupling is applied as C_a = I_3 (x) Po_a next to the
  // packed L^-1.  Outer blocks (wave 0 forward from block 0, wave 1 backward
  // from block nv-1), with p the previous block of the wave:
  //   y_a = L_a^-1 (b_a - X_a L_p^-T D_p^-1 y_p),  X_a = C_{a-1}^T / C_a,
  // the middle block with both neighbours' terms and x_m = L_m^-T D_m^-1 y_m,
  // then outward from the middle, with n the block towards it:
  //   x_a = L_a^-T D_a^-1 (y_a - L_a^-1 Y_a x_n),    Y_a = C_a / C_{a-1}^T.
  // Triangular sums run over the full row with the out-of-triangle terms
  // weighted by exact 0 (the unit diagonal by exact 1).
  __device__ void solve(int rhs_off, int out_off) {
    double* y = sm + rhs_off;
    double* xo = sm + out_off;
    const int g = grp();
    const int i = col_of() < BS ? col_of() : BS - 1;
    const bool wr = kNG == 4 ? (g == 0 && col_of() < BS) : lane < BS;
    const int di = i / M, mi = i % M;
    constexpr int KS = (BS + kNG - 1) / kNG;
    // L^-1 row i (k < i) / column i (k > i) coefficient of this lane's k-th
    // term, and the term's index.
    auto kidx = [&](int kk) {
      const int k0 = g + kNG * kk;
      return k0 < BS ? k0 : BS - 1;
    };
    auto lrow = [&](const double* Lb, int kk) {  // (L^-1)[i][k], unit diagonal
      const int k0 = g + kNG * kk, k = kidx(kk);
      const int kx = k < i ? k : i;
      return fma(Lb[tri(i, kx)], static_cast<double>(k < i && k0 < BS), is_zero(k0 - i));
    };
    auto lcol = [&](const double* Lb, int kk) {  // (L^-1)[k][i], unit diagonal
      const int k0 = g + kNG * kk, k = kidx(kk);
      const int kx = k > i ? k : i;
      return fma(Lb[tri(kx, i)], static_cast<double>(k > i && k0 < BS), is_zero(k0 - i));
    };
    // (X L_p^-T uu)_i with uu = D_p^-1 y_p (lane k holds entry k), X given
    // by its Po block: X[(d, mi), (d, mm)] = Po[mm * pt + mi * ps].
    auto term = [&](double uu, const double* Lp, const double* Po, int pt, int ps) {
      double v = 0.0;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) v = fma(lcol(Lp, kk), __shfl(uu, kidx(kk)), v);
      v = rows_sum(v);
      double s = 0.0;
#pragma unroll
      for (int mm = 0; mm < M; ++mm) s = fma(Po[mm * pt + mi * ps], __shfl(v, di * M + mm), s);
      return s;
    };
    const int m = mid(), nb = nv - 1 - m;
    const bool bw = wv == 1;  // wave-uniform
    const int nf = bw ? nb : m;  // this wave's outer blocks
    double u = 0.0;              // D_p^-1 y_p, entry i
    for (int k = 0; k < nf; ++k) {
      const int a = bw ? nv - 1 - k : k;
      const double* Li = sm + L->Li + a * kTri;
      double t = y[a * BS + i];
      if (k > 0)  // forward: C_{a-1}^T (Po_{a-1} transposed); backward: C_a
        t -= bw ? term(u, Li + kTri, sm + L->Po + a * M * M, 1, M)
                : term(u, Li - kTri, sm + L->Po + (a - 1) * M * M, M, 1);
      double z = 0.0;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) z = fma(lrow(Li, kk), __shfl(t, kidx(kk)), z);
      z = rows_sum(z);
      u = z * Li[tri(i, i)];
      if (wr) y[a * BS + i] = z;
    }
    __syncthreads();
    double xn = 0.0;  // x of the block towards the middle, entry i
    if (!bw) {        // the middle block
      const double* Li = sm + L->Li + m * kTri;
      double t = y[m * BS + i];
      if (m > 0) t -= term(u, Li - kTri, sm + L->Po + (m - 1) * M * M, M, 1);
      if (m < nv - 1) {
        const double ub = y[(m + 1) * BS + i] * Li[kTri + tri(i, i)];
        t -= term(ub, Li + kTri, sm + L->Po + m * M * M, 1, M);
      }
      double z = 0.0;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) z = fma(lrow(Li, kk), __shfl(t, kidx(kk)), z);
      z = rows_sum(z) * Li[tri(i, i)];
      double x = 0.0;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) x = fma(lcol(Li, kk), __shfl(z, kidx(kk)), x);
      x = rows_sum(x);
      xn = x;
      if (wr) xo[m * BS + i] = x;
    }
    __syncthreads();
    if (bw) xn = xo[m * BS + i];
    for (int k = nf - 1; k >= 0; --k) {
      const int a = bw ? nv - 1 - k : k;
      const double* Li = sm + L->Li + a * kTri;
      double t = y[a * BS + i];
      // c = C_a x_{a+1} (forward blocks) or C_{a-1}^T x_{a-1} (backward);
      // t -= (L_a^-1 c)_i.
      const double* Po = sm + L->Po + (bw ? a - 1 : a) * M * M;
      const int pt = bw ? M : 1, ps = bw ? 1 : M;
      double c = 0.0;
#pragma unroll
      for (int mm = 0; mm < M; ++mm) c = fma(Po[mm * pt + mi * ps], __shfl(xn, di * M + mm), c);
      double s = 0.0;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) s = fma(lrow(Li, kk), __shfl(c, kidx(kk)), s);
      t -= rows_sum(s);
      t *= Li[tri(i, i)];
      double x = 0.0;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) x = fma(lcol(Li, kk), __shfl(t, kidx(kk)), x);
      x = rows_sum(x);
      xn = x;
      if (wr) xo[a * BS + i] = x;
    }
    __syncthreads();
  }

  // x op (x moved by DPP control CTRL); lanes with no source, or in rows
  // RM leaves out, take their own value (op(x, x) = x).
  template <int CTRL, int RM, bool kMax>
  __device__ static double dpp_op(double x) {
    const long long u = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_update_dpp(static_cast<int>(u), static_cast<int>(u), CTRL, RM,
                                               0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(static_cast<int>(u >> 32),
                                               static_cast<int>(u >> 32), CTRL, RM, 0xf, false);
    const double y = __builtin_bit_cast(
        double, (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
    return kMax ? fmax(x, y) : fmin(x, y);
  }
  // Wave maximum / minimum in every lane: DPP scans in rows of 16, the row
  // broadcasts, then lane 63's value (VALU moves instead of the six LDS
  // permutes of a shuffle butterfly; max and min do not depend on the order).
  template <bool kMax>
  __device__ static double wave_ext(double x) {
    x = dpp_op<0x111, 0xf, kMax>(x);
    x = dpp_op<0x112, 0xf, kMax>(x);
    x = dpp_op<0x114, 0xf, kMax>(x);
    x = dpp_op<0x118, 0xf, kMax>(x);
    x = dpp_op<0x142, 0xa, kMax>(x);
    x = dpp_op<0x143, 0xc, kMax>(x);
    const long long u = __builtin_bit_cast(long long, x);
    return __builtin_bit_cast(
        double, (static_cast<long long>(__builtin_amdgcn_readlane(static_cast<int>(u >> 32), 63))
                 << 32) |
                    static_cast<unsigned int>(__builtin_amdgcn_readlane(static_cast<int>(u), 63)));
  }
  __device__ static double wave_max(double x) { return wave_ext<true>(x); }
  __device__ static double wave_min(double x) { return wave_ext<false>(x); }
  __device__ static double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
    return x;
  }
  // Workgroup reductions (one or two waves); every thread calls them.
  template <int kOp>  // 0 max, 1 min, 2 sum
  __device__ double block_red(double x) {
    x = kOp == 0 ? wave_max(x) : kOp == 1 ? wave_min(x) : wave_sum(x);
    if (nthr == kWave) return x;
    // Consecutive reductions alternate between two slot pairs, so one
    // barrier suffices: a wave that writes a pair again has passed the next
    // reduction's barrier, which the other wave reaches only after reading.
    const int p = L->red + 2 * redp;
    redp ^= 1;
    if (lane == 0) sm[p + wv] = x;
    __syncthreads();
    const double a = sm[p], c = sm[p + 1];
    return kOp == 0 ? fmax(a, c) : kOp == 1 ? fmin(a, c) : a + c;
  }
  __device__ double block_max(double x) { return block_red<0>(x); }
  __device__ double block_min(double x) { return block_red<1>(x); }
  __device__ double block_sum(double x) { return block_red<2>(x); }

  // Complementarity target: affine rc = s lam; corrector
  // rc = s lam + ds_aff dl_aff - sigma mu (ds, dl still hold the affine step).
  template <bool kCorr>
  __device__ double rc_of(int k, double smu) const {
    const double v = sm[L->s + k] * sm[L->lam + k];
    return kCorr ? v + sm[L->ds + k] * sm[L->dl + k] - smu : v;
  }

  // Newton direction for the complementarity target rc_of<kCorr>:
  // rhs = -rd - sum a_k (lam rp - rc)/s, solve, then dl, ds.  Expects cp, rd
  // valid and the factorisation done.  The step's control points go to acc.
  template <bool kCorr>
  __device__ void direction(double smu) {
    // Per control point: Psi[d] = sum_k w_k[d] (lam_k rp_k - rc_k) / s_k.
    // The constraint values and gradients are re-evaluated here rather than
    // cached from the predictor: a 4*ncon cache (round 5) grew the layout
    // 39.2 -> 40.5 KB and measured 8.09 -> 9.65 ms at config 3.
    for (int cpi = tid; cpi < S * N; cpi += nthr) {
      const int i = cpi / N, j = cpi % N;
      double P3[3] = {0.0, 0.0, 0.0};
      int kk[3];
      double gg[3], ww[3][3];
      bool sph;
      cp_cons(i, j, L->cp, kk, gg, ww, sph);
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int k = kk[t];
        if (k < 0) continue;
        const double lam = sm[L->lam + k], s = sm[L->s + k];
        const double rp = gg[t] + s;
        const double coef = (lam * rp - rc_of<kCorr>(k, smu)) / s;
        for (int d = 0; d < 3; ++d) P3[d] += ww[t][d] * coef;
      }
      for (int d = 0; d < 3; ++d) sm[L->acc + cpi * 3 + d] = P3[d];
    }
    __syncthreads();
    for (int idx = tid; idx < nv * BS; idx += nthr) {
      const int a = idx / BS, d = (idx / M) % 3, m = idx % M;
      sm[L->rhs + idx] = -sm[L->rd + idx] - gather_cp(L->acc, a, d, m);
    }
    __syncthreads();
    unsigned long long tl = 0;
    MTG_TACC(511, tl);
    solve(L->rhs, L->dx);
    MTG_TACC(210, tl);
    control_point_steps(sm + L->dx, L->acc);
    __syncthreads();
    // dl, ds per control point (its constraints' (g, w) evaluated once).
    for (int cpi = tid; cpi < S * N; cpi += nthr) {
      const int i = cpi / N, j = cpi % N;
      int kk[3];
      double gg[3], ww[3][3];
      bool sph;
      cp_cons(i, j, L->cp, kk, gg, ww, sph);
      const double* dc = sm + L->acc + cpi * 3;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int k = kk[t];
        if (k < 0) continue;
        const double adx = ww[t][0] * dc[0] + ww[t][1] * dc[1] + ww[t][2] * dc[2];
        const double lam = sm[L->lam + k], s = sm[L->s + k];
        const double rp = gg[t] + s;
        const double rc = rc_of<kCorr>(k, smu);
        const double dl = (lam / s) * (adx + rp) - rc / s;
        sm[L->dl + k] = dl;
        sm[L->ds + k] = (-rc - s * dl) / lam;
      }
    }
    __syncthreads();
  }

  __device__ double max_step() {
    double alpha = 1.0;
    for (int k = tid; k < nc; k += nthr) {
      const double ds = sm[L->ds + k], dl = sm[L->dl + k];
      if (ds < 0) alpha = fmin(alpha, -sm[L->s + k] / ds);
      if (dl < 0) alpha = fmin(alpha, -sm[L->lam + k] / dl);
    }
    return block_min(alpha);
  }

  // Full IPM (oracle TubeProblem::solveIPM).  Returns iterations; *status
  // 0 converged, 1 iteration cap, 2 numerical breakdown away from the
  // optimum, 3 near-optimal; *bad bit 2 set for a non-positive pivot of the
  // start system.  Safeguard (same in the oracle): when the KKT
  // factorisation or the step breaks down, stop at the current iterate and
  // report it near-optimal if every residual is within 1e3 * tol (status 3);
  // with the dual residual within 1e5 * tol instead, not converged
  // (status 1).
#ifndef MTG_TUBE_FLOOR  // A/B builds only (tools/build_variant.sh -DMTG_TUBE_FLOOR=...)
#define MTG_TUBE_FLOOR 2e-2
#endif
  static constexpr double kComplFloor = MTG_TUBE_FLOOR;
  static constexpr double kKktReg = 1e-10;
  // Warm start (ws != nullptr: the trajectory's previous solve, x then s
  // then lam in this kernel's own layouts): x as it was, s and lam floored
  // at kWarmFloor so the iterate is interior again.  Used by the LN_SBPLX
  // time optimiser over the QCQP objective between consecutive evaluations
  // of one trajectory (the constraints do not change: the control-point
  // maps stay at T0); the oracle does the same.  Converges to the same
  // optimum in about half the iterations (55 -> 30 per evaluation).
  static constexpr double kWarmFloor = 1e-2;
  // Cold-start multipliers: at least kLamStart |q|_inf (the oracle's value;
  // with the slack scale of ipm() and kComplFloor 30.8 -> 22.9 iterations
  // on the 4096 C3 problems).
  static constexpr double kLamStart = 30.0;
  __device__ void warm_start(const double* __restrict__ ws) {
    for (int idx = tid; idx < nv * BS; idx += nthr) sm[L->x + idx] = ws[idx];
    for (int k = tid; k < nc; k += nthr) {
      sm[L->s + k] = fmax(ws[nv * BS + k], kWarmFloor);
      sm[L->lam + k] = fmax(ws[nv * BS + nc + k], kWarmFloor);
    }
    __syncthreads();
  }
  // The state a later warm start reads (after ipm(), usable statuses only).
  __device__ void save_state(double* __restrict__ ws) const {
    for (int idx = tid; idx < nv * BS; idx += nthr) ws[idx] = sm[L->x + idx];
    for (int k = tid; k < nc; k += nthr) {
      ws[nv * BS + k] = sm[L->s + k];
      ws[nv * BS + nc + k] = sm[L->lam + k];
    }
  }

  __device__ int ipm(double tol, int max_iter, int* status, int* bad,
                     const double* __restrict__ ws = nullptr) {
    int* fail = bad + 1;
    if (tid == 0) *fail = 0;
    double qn = 0.0;
    for (int idx = tid; idx < nv * BS; idx += nthr) qn = fmax(qn, fabs(sm[L->q + idx]));
    qn = block_max(qn);
    __syncthreads();
    if (ws) {
      warm_start(ws);
    } else {
    // Unconstrained start: P x = -q.  Where P is numerically singular (long
    // segments: with T = 20 s a vertex's position barely changes the snap
    // cost, T^-7, and P's equilibrated spectrum reaches -1e-12) the start is
    // the tube axis instead: every intermediate vertex at its position, its
    // higher derivatives zero, so every control point sits on the vertex,
    // strictly inside its tubes and sphere (the oracle's rule).  The
    // constrained Newton systems add the constraints' curvature.
    factor(fail, false);
    __syncthreads();
    if (*fail) {
      for (int idx = tid; idx < nv * BS; idx += nthr) {
        const int a = idx / BS, d = (idx / M) % 3, m = idx % M;
        sm[L->x + idx] = m == 0 ? sm[L->pos + (a + 1) * 3 + d] : 0.0;
      }
      __syncthreads();
    } else {
      for (int idx = tid; idx < nv * BS; idx += nthr) sm[L->rhs + idx] = -sm[L->q + idx];
      __syncthreads();
      solve(L->rhs, L->x);
    }
    control_points(sm + L->x, L->cp);
    // Start scaled to the problem (the oracle's rule): slacks at least the
    // square of the largest vertex coordinate (the constraints are in squared
    // lengths), multipliers at least kLamStart |q|_inf.
    double pm = 1.0;
    for (int i = tid; i < (S + 1) * 3; i += nthr) pm = fmax(pm, fabs(sm[L->pos + i]));
    pm = block_max(pm);
    __syncthreads();
    const double s_start = pm * pm, lam_start = fmax(1.0, kLamStart * qn);
    for (int k = tid; k < nc; k += nthr) {
      double w[3];
      const double g = con_eval(k, L->cp, w);
      sm[L->s + k] = fmax(-g, s_start);
      sm[L->lam + k] = lam_start;
    }
    }  // cold start
    __syncthreads();
    int it = 0;
    *status = 1;
    unsigned long long tl = 0;
    MTG_TACC(511, tl);
    for (it = 0; it < max_iter; ++it) {
      // Residuals at the current point.  One pass over the control points
      // evaluates each constraint once (round 5; three passes evaluated it
      // three times): the primal residual and mu, the dual residual weights
      // Omega[cp][d] = sum_k lam_k w_k[d], and the KKT blocks' constraint
      // terms G_cp = sum_k lam_k Hess_k + (lam_k / s_k) w_k w_k^T (formerly
      // assemble_g after the convergence test; unused on the last
      // iteration).  Every constraint acts on exactly one control point.
      control_points(sm + L->x, L->cp);
      __syncthreads();
      double rpn = 0.0, mu = 0.0;
      for (int cpi = tid; cpi < S * N; cpi += nthr) {
        const int i = cpi / N, j = cpi % N;
        double O3[3] = {0.0, 0.0, 0.0};
        double G[9];
#pragma unroll
        for (int e = 0; e < 9; ++e) G[e] = 0.0;
        int kk[3];
        double gg[3], ww[3][3];
        bool sph;
        cp_cons(i, j, L->cp, kk, gg, ww, sph);
        const double* LL = sm + L->geo + i * kGeo + 3;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const int k = kk[t];
          if (k < 0) continue;
          const double s = sm[L->s + k], lam = sm[L->lam + k];
          rpn = fmax(rpn, fabs(gg[t] + s));
          mu += s * lam;
          for (int d = 0; d < 3; ++d) O3[d] += lam * ww[t][d];
          const double ws = lam / s;
#pragma unroll
          for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int e = 0; e < 3; ++e) {
              // con_hess: 2 I (sphere), 2 LL (tube), 0 (caps)
              const double h = t > 0 ? 0.0 : (sph ? (a == e ? 2.0 : 0.0) : 2.0 * LL[a * 3 + e]);
              G[a * 3 + e] += lam * h + ws * ww[t][a] * ww[t][e];
            }
        }
        for (int d = 0; d < 3; ++d) sm[L->acc + cpi * 3 + d] = O3[d];
        for (int a = 0; a < 3; ++a)
          for (int e = a; e < 3; ++e) sm[L->Gc + cpi * 6 + gsym(a, e)] = G[a * 3 + e];
      }
      rpn = block_max(rpn);
      mu = block_sum(mu) / nc;
      __syncthreads();
      double rdn = 0.0;
      for (int idx = tid; idx < nv * BS; idx += nthr) {
        const int a = idx / BS, d = (idx / M) % 3, m = idx % M;
        const double v = Pxq(sm + L->x, idx) + gather_cp(L->acc, a, d, m);
        sm[L->rd + idx] = v;
        rdn = fmax(rdn, fabs(v));
      }
      rdn = block_max(rdn);
      __syncthreads();
      if (rdn <= tol * (1.0 + qn) && rpn <= tol && mu <= tol) {
        *status = 0;
        break;
      }
      const bool near = rdn <= 1e3 * tol * (1.0 + qn) && rpn <= 1e3 * tol && mu <= 1e3 * tol;
      const double infeas = fmax(rdn / (1.0 + qn), rpn);
      // Stalled dual residual (lam / s ~ 1e12 on active constraints): not
      // converged, value usable (same tiers in the oracle).
      const bool stalled = rdn <= 1e5 * tol * (1.0 + qn) && rpn <= 1e3 * tol && mu <= 1e3 * tol;
      const int brk = near ? 3 : (stalled ? 1 : 2);
      MTG_TACC(200, tl);
      MTG_TACC(201, tl);
      // A non-positive pivot (lam / s ~ 1e12 on active constraints swamps
      // the rest of K in rounding) away from the optimum (brk == 2) is
      // retried once with a diagonal regularisation (kKktReg); the
      // regularised Newton step still converges to the same optimum, where
      // stopping left 16 % of the points of the time optimiser's box
      // [0.1, 2 T0] without a value.  Near the optimum (brk 1 or 3) the
      // iterate is kept, as before: going on regularised only stalls the dual
      // residual to the iteration cap (the oracle's rule).  One call site,
      // so the factorisation is instantiated once.
      for (double reg = 0.0;; reg = kKktReg) {
        if (tid == 0) *fail = 0;
        __syncthreads();
        factor(fail, true, reg);
        __syncthreads();
        if (!*fail || reg > 0.0 || brk != 2) break;
      }
      MTG_TACC(202, tl);
      if (*fail) {
        *status = brk;
        break;
      }
      // Affine (predictor) direction: rc = s * lam.
      direction<false>(0.0);
      MTG_TACC(203, tl);
      const double a_aff = max_step();
      double mua = 0.0;
      for (int k = tid; k < nc; k += nthr)
        mua += (sm[L->s + k] + a_aff * sm[L->ds + k]) * (sm[L->lam + k] + a_aff * sm[L->dl + k]);
      mua = block_sum(mua) / nc;
      const double ratio = mua / mu;
      // Mehrotra's sigma, with the complementarity target kept at or above
      // kComplFloor x the relative infeasibility (the oracle's rule): mu
      // running ahead of the dual residual sends lam / s on the active
      // constraints past 1e12, where the condensed KKT matrix loses its
      // null-space part to rounding, the dual residual stalls and the
      // factorisation breaks down.  kComplFloor = 2e-2 with the scaled start
      // (1e-2 with unit starts, round 5; the oracle's values).
      double sigma = ratio * ratio * ratio;
      {
        const double floor_mu = fmin(mu, kComplFloor * infeas);
        if (sigma * mu < floor_mu) sigma = floor_mu / mu;
      }
      __syncthreads();
      // Corrector: rc = s lam + ds_aff dl_aff - sigma mu.
      MTG_TACC(204, tl);
      direction<true>(sigma * mu);
      MTG_TACC(205, tl);
      const double alpha = fmin(1.0, 0.99 * max_step());
      double dxn = 0.0;
      for (int idx = tid; idx < nv * BS; idx += nthr) dxn = fmax(dxn, fabs(sm[L->dx + idx]));
      dxn = block_max(dxn);
      if (!(alpha > 0.0) || !(dxn < 1e300) || !(sigma < 1e300)) {
        *status = brk;
        break;
      }
      for (int idx = tid; idx < nv * BS; idx += nthr) sm[L->x + idx] += alpha * sm[L->dx + idx];
      for (int k = tid; k < nc; k += nthr) {
        sm[L->s + k] += alpha * sm[L->ds + k];
        sm[L->lam + k] += alpha * sm[L->dl + k];
      }
      __syncthreads();
      MTG_TACC(206, tl);
    }
    return it;
  }
};

}  // namespace mtg
