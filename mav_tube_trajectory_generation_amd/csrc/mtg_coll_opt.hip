// mtg_coll_opt.hip — the collision-driven objectives of
// PolynomialOptimizationNonLinear and a batched device optimiser over them:
// the reference demo's path (src/main.cpp:77, 104-105).
//   mode 0  objectiveFunctionFreeConstraintsAndCollision (nonlinear_impl:
//           1115-1272) over x = d_p, driver optimizeFreeConstraintsAnd
//           Collision (:495-607);
//   mode 1  objectiveFunctionFreeConstraintsAndCollisionAndTime (:1274-1535)
//           over x = [T; d_p], driver optimizeFreeConstraintsAndCollisionAnd
//           Time (:708-845).
// See include/mtg_hip.h (mtg_coll_cost / mtg_coll_optimize) for the exact
// objective, including the reference quirks it reproduces.
//
// One objective evaluation of a batch is a short chain of launches, each
// shaped for its work:
//   prep   one wave per trajectory (generic per-trajectory state,
//          mtg_device.h): times, coefficients A^-1(T) M d, J_d = 2 computeCost
//          and its gradient 2 (R_pf d_f + R_pp d_p) (no R assembled), J_t and
//          the d-fixed time differences of J_d (seg_energy_at, only segment n
//          changes);
//   walk   one 256-thread workgroup per (trajectory, walk): the collision
//          walk at T and, for the time gradient, at every perturbed T
//          (mtg_collision_device.h); the gradient walk maps dJ_c/dc to the
//          free derivatives;
//   soft   (soft constraints only) one wave per (trajectory, perturbation)
//          builds the coefficients of x +- h e_i (only the one or two
//          segments touching the perturbed vertex are recomputed), then the
//          batched extremum search of mtg_extrema.hip forms every soft cost;
//   combine one wave per trajectory: weights, the collision raise rule and
//          the gradient; in the optimiser also one step of the L-BFGS state
//          machine, which places the next evaluation point.
// The optimiser enqueues max_evals such rounds.  Every kernel first reads
// the trajectory's `done` flag, so finished trajectories cost one load per
// launch and nothing synchronises with the host.  All scratch lives in the
// caller's workspace.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_collision_device.h"
#include "mtg_free_device.h"
#include "mtg_internal.h"

namespace mtg {

namespace {

constexpr double kLowerT = 0.1;  // the clamp of getCostAndGradientTime (:2529-2530)
constexpr int kMaxLbfgsMemory = 16;
constexpr double kArmijo = 1e-4;

struct CollDims {
  int mode, S, D, np;
  int nfr;   // D * np free variables
  int nv;    // variables per trajectory (mode 1: S + nfr)
  int off;   // offset of d_p in x (mode 1: S)
  int P;     // collision walks per trajectory (1, or 1 + S / 1 + 2S for the time gradient)
  int Q;     // soft-cost problems per trajectory (0 without soft constraints)
  int central_t, central_sc;
  int m;     // L-BFGS memory
};

CollDims coll_dims(const PlanDev& pl, int mode, const mtg_coll_params& p) {
  CollDims c{};
  c.mode = mode;
  c.S = pl.S;
  c.D = pl.D;
  c.np = pl.np;
  c.nfr = pl.D * pl.np;
  c.off = mode ? pl.S : 0;
  c.nv = c.off + c.nfr;
  c.central_t = !p.simple_numgrad_time;
  c.central_sc = mode == 0 || !p.simple_numgrad_constraints;
  c.P = mode ? (c.central_t ? 1 + 2 * pl.S : 1 + pl.S) : 1;
  c.Q = p.n_soft > 0 ? (c.central_sc ? 1 + 2 * c.nfr : 1 + c.nfr) : 0;
  c.m = p.lbfgs_memory;
  return c;
}

struct CollWs {
  double* xt;      // B x nv   evaluation point (optimiser)
  double* T;       // B x S    its segment times
  double* coeffs;  // B x S x D x N
  double* Jd;      // B        J_d (unweighted)
  double* Jt;      // B        sum T
  double* gd;      // B x nfr  dJ_d / dd_p
  double* dJd;     // B x S    dJ_d / dT_n (d held)
  double* Jc;      // B x P    J_c of every walk
  int32_t* coll;   // B x P
  double* gc;      // B x nfr  dJ_c / dd_p of the walk at T
  double* softc;   // B x Q x S x D x N
  double* softT;   // B x Q x S
  double* softJ;   // B x Q
  double* softm;   // B x Q x n_soft (per-constraint launches)
  int32_t* st;     // B        MTG_TRAJ_* of the evaluation point
  int32_t* done;   // B        (optimiser) trajectory finished
  // L-BFGS state (optimiser).
  double *x, *g, *G, *dir, *Sh, *Yh, *rho, *f, *alpha, *Jref0, *Jlast, *terms, *tterms, *step0;
  int32_t *hist, *evals, *result, *phase;
};

struct Carver {
  char* base;
  size_t off = 0;
  template <typename T>
  T* take(int64_t n) {
    off = (off + 255) & ~size_t(255);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += sizeof(T) * static_cast<size_t>(n > 0 ? n : 1);
    return p;
  }
};

size_t carve(void* base, const CollDims& c, int N, int64_t B, int n_soft, bool opt, CollWs* w) {
  Carver k{static_cast<char*>(base)};
  const int S = c.S, D = c.D;
  *w = CollWs{};
  w->xt = k.take<double>(B * c.nv);
  w->T = k.take<double>(B * S);
  w->coeffs = k.take<double>(B * S * D * N);
  w->Jd = k.take<double>(B);
  w->Jt = k.take<double>(B);
  w->gd = k.take<double>(B * c.nfr);
  w->dJd = k.take<double>(B * S);
  w->Jc = k.take<double>(B * c.P);
  w->coll = k.take<int32_t>(B * c.P);
  w->gc = k.take<double>(B * c.nfr);
  if (c.Q > 0) {
    w->softc = k.take<double>(B * c.Q * S * D * N);
    w->softT = k.take<double>(B * c.Q * S);
    w->softJ = k.take<double>(B * c.Q);
    w->softm = k.take<double>(B * c.Q * n_soft);
  }
  w->st = k.take<int32_t>(B);
  if (opt) {
    w->done = k.take<int32_t>(B);
    w->x = k.take<double>(B * c.nv);
    w->g = k.take<double>(B * c.nv);
    w->G = k.take<double>(B * c.nv);
    w->dir = k.take<double>(B * c.nv);
    w->Sh = k.take<double>(B * c.m * c.nv);
    w->Yh = k.take<double>(B * c.m * c.nv);
    w->rho = k.take<double>(B * c.m);
    w->f = k.take<double>(B);
    w->alpha = k.take<double>(B);
    w->Jref0 = k.take<double>(B);
    w->Jlast = k.take<double>(B);
    w->terms = k.take<double>(B * 4);
    w->tterms = k.take<double>(B * 4);
    w->step0 = k.take<double>(B);
    w->hist = k.take<int32_t>(B * 2);
    w->evals = k.take<int32_t>(B);
    w->result = k.take<int32_t>(B);
    w->phase = k.take<int32_t>(B);
  }
  return k.off + 256;
}

__device__ inline bool skipped(const CollWs& w, int64_t b) { return w.done && w.done[b]; }

// Segment time n of the time-gradient walk q (q = 0: T itself): central
// differences lower / raise T_n by h (q = 1 + 2n / 2 + 2n), forward
// differences raise it (q = 1 + n); both clamp at 0.1 (:2529-2530, 2622-2623).
__device__ inline double walk_time(const CollDims& cd, const double* T, int q, int i, double h) {
  const double t = T[i];
  if (q == 0) return t;
  const int n = cd.central_t ? (q - 1) >> 1 : q - 1;
  if (i != n) return t;
  const bool up = !cd.central_t || ((q - 1) & 1);
  return t <= kLowerT ? kLowerT : (up ? t + h : t - h);
}

// ---------------------------------------------------------------------------
// prep: coefficients, J_d and its gradient, J_t and dJ_d/dT (d held).
template <int N>
__global__ __launch_bounds__(kWave) void coll_prep_kernel(PlanDev pl, CollDims cd,
                                                          const double* __restrict__ fixed_vals,
                                                          const double* __restrict__ times_in,
                                                          const double* __restrict__ xsrc,
                                                          double inc, CollWs w) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int64_t b = blockIdx.x;
  if (skipped(w, b)) return;
  const int S = pl.S, D = pl.D, nf = pl.nf, np = pl.np;
  const Layout lay = make_layout(N, S, D);
  const FreeLds fl = free_lds(N, S, D, np, false);
  Traj<N> t{S, D, pl.r, &lay, smem, reinterpret_cast<int*>(smem + lay.ndouble),
            static_cast<int>(threadIdx.x), pl.fmask, pl.use_mask != 0};
  const double* xb = xsrc + b * cd.nv;
  const double* tb = cd.mode ? xb : times_in + b * S;
  const bool bad = free_setup(t, pl, fixed_vals + b * D * nf, xb + cd.off, tb);
  for (int i = t.lane; i < S; i += kWave) w.T[b * S + i] = t.T()[i];
  double Jd = NAN, Jt = NAN;
  if (!bad) {
    // J_d = sum_dim d^T R d = c^T Q c = 2 computeCost() (:1537-1606).
    Jd = 2.0 * t.template coeffs_and_cost<true>(pl.tab, w.coeffs + b * S * D * N);
    double* gv = lds_at<double>(smem, fl.gv);
    free_rd(t, gv);
    for (int i = t.lane; i < D * np; i += kWave)
      w.gd[b * cd.nfr + i] = 2.0 * gv[pl.free_map[i % np] * D + i / np];
    if (cd.mode == 1) {
      double tot = 0.0;
      for (int i = 0; i < S; ++i) tot += t.T()[i];  // computeTotalTrajectoryTime (:2768-2774)
      Jt = tot;
      // getCostAndGradientTime: J_d at T_n +- h with d held (updateSegmentTimes
      // then getCostAndGradientDerivative, :2532-2537); only segment n's
      // energy changes.
      for (int n = 0; n < S; ++n) {
        const double Tn = t.T()[n];
        const double hi = Tn <= kLowerT ? kLowerT : Tn + inc;
        const double e_hi = t.seg_energy_at(n, hi);
        double dj;
        if (cd.central_t) {
          const double lo = Tn <= kLowerT ? kLowerT : Tn - inc;
          dj = (e_hi - t.seg_energy_at(n, lo)) / (2.0 * inc);
        } else {
          dj = (e_hi - t.seg_energy_at(n, Tn)) / inc;
        }
        if (t.lane == 0) w.dJd[b * S + n] = dj;
      }
    }
  }
  if (t.lane == 0) {
    w.Jd[b] = Jd;
    w.Jt[b] = Jt;
    w.st[b] = bad ? MTG_TRAJ_BAD_TIME : MTG_TRAJ_OK;
  }
}

// walk: J_c of walk q of trajectory b; q = 0 also the gradient.
template <int N>
__global__ __launch_bounds__(kCollBlock) void coll_walk_kernel(
    PlanDev pl, CollDims cd, const float* __restrict__ occ, int nx, int ny, int nz,
    const uint16_t* __restrict__ field, mtg_collision_params cp, double inc, CollWs w) {
  constexpr int D = 3;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int S = pl.S;
  const int64_t prob = blockIdx.x;
  const int64_t b = prob / cd.P;
  const int q = static_cast<int>(prob - b * cd.P);
  const int tid = threadIdx.x;
  if (skipped(w, b)) return;
  if (w.st[b] != MTG_TRAJ_OK) {
    if (tid == 0) {
      w.Jc[prob] = NAN;
      w.coll[prob] = 0;
    }
    if (q == 0)
      for (int i = tid; i < cd.nfr; i += static_cast<int>(blockDim.x)) w.gc[b * cd.nfr + i] = NAN;
    return;
  }
  double* c_s = sm;               // S x D x N
  double* T_s = c_s + S * D * N;  // S (walk times)
  double* g_s = T_s + S;          // S x D x N
  double* scratch = g_s + S * D * N;
  const bool grad = q == 0;
  for (int i = tid; i < S * D * N; i += static_cast<int>(blockDim.x)) {
    c_s[i] = w.coeffs[b * S * D * N + i];
    if (grad) g_s[i] = 0.0;
  }
  for (int i = tid; i < S; i += static_cast<int>(blockDim.x)) T_s[i] = walk_time(cd, w.T + b * S, q, i, inc);
  __syncthreads();
  double J;
  bool hit;
  collision_walk<N>(S, c_s, T_s, occ, nx, ny, nz, cp, grad, g_s, scratch, &J, &hit, field);
  if (tid == 0) {
    w.Jc[prob] = J;
    w.coll[prob] = hit ? 1 : 0;
  }
  if (grad)  // T_s is T itself for q = 0
    for (int i = tid; i < cd.nfr; i += static_cast<int>(blockDim.x))
      w.gc[b * cd.nfr + i] =
          coll_grad_free<N>(S, D, pl.np, pl.tab + N * N, pl.free_map, T_s, g_s, i);
}

// soft points: coefficients of problem q of trajectory b.  q = 0 is x itself;
// q > 0 perturbs free variable i = (q-1)/2 by -h / +h (central) or i = q-1 by
// +h (forward) as setFreeConstraints(free_constraints -+ increment) does
// (:2396-2416, 2469-2479): only the segments meeting at the perturbed vertex
// change, and they are recomputed as c = A^-1(T) [d(s); d(s+1)] from the
// perturbed endpoint derivatives.
template <int N>
__global__ __launch_bounds__(kWave) void coll_soft_points_kernel(
    PlanDev pl, CollDims cd, const double* __restrict__ fixed_vals,
    const double* __restrict__ xsrc, double h, CollWs w) {
  constexpr int M = N / 2;
  const int S = pl.S, D = pl.D, per = S * D * N;
  const int64_t prob = blockIdx.x;
  const int64_t b = prob / cd.Q;
  const int q = static_cast<int>(prob - b * cd.Q);
  const int lane = threadIdx.x;
  if (skipped(w, b)) return;
  double* dst = w.softc + prob * per;
  if (w.st[b] != MTG_TRAJ_OK) {  // keep the search on finite data; J is NaN anyway
    for (int i = lane; i < per; i += kWave) dst[i] = 0.0;
    for (int i = lane; i < S; i += kWave) w.softT[prob * S + i] = 1.0;
    return;
  }
  for (int i = lane; i < per; i += kWave) dst[i] = w.coeffs[b * per + i];
  for (int i = lane; i < S; i += kWave) w.softT[prob * S + i] = w.T[b * S + i];
  if (q == 0) return;
  __syncthreads();
  const int iv = cd.central_sc ? (q - 1) >> 1 : q - 1;
  const double sgn = (!cd.central_sc || ((q - 1) & 1)) ? 1.0 : -1.0;
  const int k = iv / pl.np, pidx = iv % pl.np;
  const int slot = pl.free_map[pidx], v = slot / M, j = slot % M;
  const double* xb = xsrc + b * cd.nv + cd.off;
  const double xp = xb[iv];
  const double xpert = sgn > 0.0 ? xp + h : xp - h;
  // Lanes 0..N-1: segment v (v = its start vertex); lanes 32..32+N-1:
  // segment v-1 (v = its end vertex).
  const int half = lane >> 5, a = lane & 31;
  const int s = v - half;
  if (a >= N || s < 0 || s >= S) return;
  double e[N];
#pragma unroll
  for (int jj = 0; jj < N; ++jj) {
    const int vv = s + jj / M, kk = jj % M;
    const int sl = pl.slots[vv * M + kk];
    double val = sl >= 0 ? fixed_vals[(b * D + k) * pl.nf + sl] : xb[k * pl.np + (-sl - 1)];
    if (vv == v && kk == j) val = xpert;
    e[jj] = val;
  }
  // c_a = sum_jj A(1)^-1[a][jj] T^(jj mod M - a) e_jj (Traj::coeffs_and_cost),
  // the powers by the multiplication chains of Traj::compute_powers.
  const double T = w.T[b * S + s];
  const double inv = rcp64(T);
  const double* tA = pl.tab + N * N;  // A(1)^-1
  double c = 0.0;
#pragma unroll
  for (int jj = 0; jj < N; ++jj) {
    const int ex = (jj % M) - a;
    const double base = ex >= 0 ? T : inv;
    double pw = 1.0;
    for (int z = 0; z < (ex >= 0 ? ex : -ex); ++z) pw *= base;
    c += tA[a * N + jj] * pw * e[jj];
  }
  dst[(s * D + k) * N + a] = c;
}

// NLopt's relstop (vold -> vnew within reltol or abstol; util/stop.c).
__device__ inline bool relstop(double vold, double vnew, double reltol, double abstol) {
  if (vold == vnew) return true;
  const double d = fabs(vnew - vold);
  return d < abstol || d < reltol * (fabs(vnew) + fabs(vold)) * 0.5;
}

__device__ inline double wave_sum64(double x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
  return x;
}
__device__ inline double wave_max64(double x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x = fmax(x, __shfl_xor(x, off, kWave));
  return x;
}

struct CombineOut {
  const double* raise_ref;
  double* cost;
  double* grad;
  double* terms;
  int32_t* collision;
  int32_t* status;
  // Optimiser only (nullable): B x max_evals x nv, row k = the point of the
  // (k+1)-th counted evaluation (all_trajectories_, nonlinear_impl:1244,1482).
  double* x_history;
};

struct Bounds {
  const double* lo;
  const double* hi;
};

// Projected L-BFGS direction at (x, g) of trajectory b into w.dir: two-loop
// recursion over the stored pairs on the free variables (a variable at a
// bound whose gradient pushes outward is held).  Returns max |q| (0: the
// projected gradient vanishes).
__device__ double lbfgs_direction(const CollDims& cd, const CollWs& w, const Bounds& bd, int64_t b,
                                  int lane, bool reset) {
  const int nv = cd.nv, m = cd.m;
  double* x = w.x + b * nv;
  double* g = w.g + b * nv;
  double* d = w.dir + b * nv;
  int32_t* hist = w.hist + b * 2;
  if (reset) {
    if (lane == 0) hist[0] = hist[1] = 0;
    __syncthreads();
  }
  const int cnt = hist[0], head = hist[1];
  auto held = [&](int i) {
    const double lo = bd.lo ? bd.lo[b * nv + i] : -HUGE_VAL;
    const double hi = bd.hi ? bd.hi[b * nv + i] : HUGE_VAL;
    return (x[i] <= lo && g[i] > 0.0) || (x[i] >= hi && g[i] < 0.0);
  };
  double qmax = 0.0;
  for (int i = lane; i < nv; i += kWave) {
    const double qi = held(i) ? 0.0 : g[i];
    d[i] = qi;  // q, then r
    qmax = fmax(qmax, fabs(qi));
  }
  qmax = wave_max64(qmax);
  if (!(qmax > 0.0)) return qmax;
  double a[kMaxLbfgsMemory];
  const double* Sh = w.Sh + b * m * nv;
  const double* Yh = w.Yh + b * m * nv;
  const double* rho = w.rho + b * m;
  __syncthreads();
  for (int c = 0; c < cnt; ++c) {  // newest to oldest
    const int k = (head - 1 - c + m) % m;
    double sq = 0.0;
    for (int i = lane; i < nv; i += kWave) sq += Sh[k * nv + i] * d[i];
    const double ak = rho[k] * wave_sum64(sq);
#pragma unroll
    for (int z = 0; z < kMaxLbfgsMemory; ++z)
      if (z == c) a[z] = ak;
    for (int i = lane; i < nv; i += kWave) d[i] -= ak * Yh[k * nv + i];
  }
  double gamma;
  if (cnt > 0) {
    const int k = (head - 1 + m) % m;
    double sy = 0.0, yy = 0.0;
    for (int i = lane; i < nv; i += kWave) {
      sy += Sh[k * nv + i] * Yh[k * nv + i];
      yy += Yh[k * nv + i] * Yh[k * nv + i];
    }
    gamma = wave_sum64(sy) / wave_sum64(yy);
  } else {
    const double step = w.step0[b];
    gamma = (step > 0.0 ? step : 1.0) / qmax;
  }
  for (int i = lane; i < nv; i += kWave) d[i] *= gamma;
  for (int c = cnt - 1; c >= 0; --c) {  // oldest to newest
    const int k = (head - 1 - c + m) % m;
    double yr = 0.0;
    for (int i = lane; i < nv; i += kWave) yr += Yh[k * nv + i] * d[i];
    const double beta = rho[k] * wave_sum64(yr);
    double ak = 0.0;
#pragma unroll
    for (int z = 0; z < kMaxLbfgsMemory; ++z)
      if (z == c) ak = a[z];
    for (int i = lane; i < nv; i += kWave) d[i] += (ak - beta) * Sh[k * nv + i];
  }
  double gp = 0.0;
  for (int i = lane; i < nv; i += kWave) {
    d[i] = held(i) ? 0.0 : -d[i];
    gp += g[i] * d[i];
  }
  gp = wave_sum64(gp);
  if (!(gp < 0.0)) {  // not a descent direction: restart from steepest descent
    if (lane == 0) hist[0] = hist[1] = 0;
    const double step = w.step0[b];
    const double g0 = (step > 0.0 ? step : 1.0) / qmax;
    for (int i = lane; i < nv; i += kWave) d[i] = held(i) ? 0.0 : -g0 * g[i];
  }
  __syncthreads();
  return qmax;
}

// combine: J and its gradient at the evaluation point; with kOpt also one
// step of the L-BFGS state machine.
template <bool kOpt>
__global__ __launch_bounds__(kWave) void coll_combine_kernel(CollDims cd, mtg_coll_params p,
                                                             int max_evals, Bounds bd, CollWs w,
                                                             CombineOut o) {
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  if (skipped(w, b)) return;
  const int S = cd.S, P = cd.P, Q = cd.Q, nv = cd.nv, off = cd.off, nfr = cd.nfr;
  const int st = w.st[b];
  const bool bad = st != MTG_TRAJ_OK;
  const bool coll = !bad && w.coll[b * P] != 0;
  const double Jc0 = bad ? NAN : w.Jc[b * P];
  double Jd = 0.0, Jt = 0.0, Jsc = 0.0;
  if (bad) {
    Jd = Jt = Jsc = NAN;
  } else if (!coll) {  // :1171-1178, 1355-1386
    Jd = w.Jd[b];
    if (cd.mode == 1) Jt = w.Jt[b];
    if (Q > 0) Jsc = w.softJ[b * Q];
  }
  const double ct = p.w_d * Jd, ctm = p.w_t * Jt, csc = p.w_sc * Jsc;
  double cc = p.w_c * Jc0;
  const double total = ct + cc + ctm + csc;
  if (p.is_collision_safe && coll) {  // :1207-1226, 1432-1452
    double ref;
    if constexpr (kOpt)
      ref = p.is_coll_raise_first_iter ? w.Jref0[b] : w.Jlast[b];
    else
      ref = o.raise_ref ? o.raise_ref[b] : 0.0;
    cc = ref - (total - cc) + p.add_coll_raise;
  }
  const double J = ct + cc + ctm + csc;
  const double h = p.coll.map_resolution, inc = p.increment_time;
  double* G = kOpt ? w.G + b * nv : (o.grad ? o.grad + b * nv : nullptr);
  if (G) {
    for (int i = lane; i < nv; i += kWave) {
      double gi;
      if (i < off) {  // getCostAndGradientTime (:2565-2571, 2638-2644)
        const int n = i;
        if (bad) {
          gi = NAN;
        } else if (coll) {
          gi = 0.0;
        } else {
          const double dJc = cd.central_t
                                 ? (w.Jc[b * P + 2 + 2 * n] - w.Jc[b * P + 1 + 2 * n]) / (2.0 * inc)
                                 : (w.Jc[b * P + 1 + n] - Jc0) / inc;
          gi = p.w_d * w.dJd[b * S + n] + p.w_c * dJc + p.w_sc * 0.0 + p.w_t * 1.0;
        }
      } else {  // :1263-1268, 1525-1531
        const int k = i - off;
        double gdd = 0.0, gsc = 0.0;
        if (bad) {
          gdd = NAN;
        } else if (!coll) {
          gdd = w.gd[b * nfr + k];
          if (Q > 0)
            gsc = cd.central_sc ? (w.softJ[b * Q + 2 + 2 * k] - w.softJ[b * Q + 1 + 2 * k]) /
                                      (2.0 * h)
                                : (w.softJ[b * Q + 1 + k] - w.softJ[b * Q]) / h;
        }
        gi = p.w_d * gdd + p.w_c * w.gc[b * nfr + k] + p.w_sc * gsc;
      }
      G[i] = gi;
    }
  }
  if constexpr (!kOpt) {
    if (lane == 0) {
      if (o.cost) o.cost[b] = J;
      if (o.terms) {
        o.terms[b * 4 + 0] = ct;
        o.terms[b * 4 + 1] = cc;
        o.terms[b * 4 + 2] = ctm;
        o.terms[b * 4 + 3] = csc;
      }
      if (o.collision) o.collision[b] = coll ? 1 : 0;
      if (o.status) o.status[b] = st;
    }
    return;
  } else {
    __syncthreads();
    // ---- L-BFGS state machine (one counted evaluation per round).
    const int m = cd.m;
    double* x = w.x + b * nv;
    double* g = w.g + b * nv;
    double* xt = w.xt + b * nv;
    double* d = w.dir + b * nv;
    const int phase = w.phase[b];
    const int evals = w.evals[b] + 1;
    double f = w.f[b], alpha = w.alpha[b];
    int result = 0;  // 0: continue
    bool place = false;
    if (o.x_history) {  // the evaluated point, before the state machine moves xt
      double* hrow = o.x_history + (b * max_evals + (evals - 1)) * nv;
      for (int i = lane; i < nv; i += kWave) hrow[i] = xt[i];
    }
    if (lane == 0) {
      if (phase == 0) w.Jref0[b] = J;  // total_cost_iter0_ (:1253-1257)
      w.Jlast[b] = J;                  // optimization_info_ of this evaluation
      w.evals[b] = evals;
      w.tterms[b * 4 + 0] = ct;
      w.tterms[b * 4 + 1] = cc;
      w.tterms[b * 4 + 2] = ctm;
      w.tterms[b * 4 + 3] = csc;
    }
    auto accept_point = [&]() {
      for (int i = lane; i < nv; i += kWave) {
        x[i] = xt[i];
        g[i] = G[i];
      }
      if (lane == 0) {
        w.f[b] = J;
        for (int z = 0; z < 4; ++z) w.terms[b * 4 + z] = w.tterms[b * 4 + z];
      }
      f = J;
      __syncthreads();
    };
    if (phase == 0) {
      if (!std::isfinite(J)) {
        result = -1;  // FAILURE
        if (lane == 0) w.f[b] = J;
      } else {
        accept_point();
        if (!(lbfgs_direction(cd, w, bd, b, lane, true) > 0.0)) result = 1;  // SUCCESS
        alpha = 1.0;
        place = true;
      }
      if (lane == 0) w.phase[b] = 1;
    } else {
      double dd = 0.0;
      for (int i = lane; i < nv; i += kWave) dd += g[i] * (xt[i] - x[i]);
      dd = wave_sum64(dd);
      if (std::isfinite(J) && J < f && J <= f + kArmijo * dd) {
        // Accept: store the pair, test NLopt's ftol / xtol, new direction.
        double sy = 0.0, ss = 0.0, yy = 0.0;
        bool xstop = true;
        for (int i = lane; i < nv; i += kWave) {
          const double s = xt[i] - x[i], y = G[i] - g[i];
          sy += s * y;
          ss += s * s;
          yy += y * y;
          xstop = xstop && relstop(x[i], xt[i], p.x_rel, p.x_abs);
        }
        sy = wave_sum64(sy);
        ss = wave_sum64(ss);
        yy = wave_sum64(yy);
        xstop = __all(xstop);
        const bool fstop = relstop(f, J, p.f_rel, p.f_abs);
        if (sy > 1e-12 * sqrt(ss * yy)) {
          int32_t* hist = w.hist + b * 2;
          const int head = hist[1], cnt = hist[0];
          for (int i = lane; i < nv; i += kWave) {
            w.Sh[(b * m + head) * nv + i] = xt[i] - x[i];
            w.Yh[(b * m + head) * nv + i] = G[i] - g[i];
          }
          __syncthreads();
          if (lane == 0) {
            w.rho[b * m + head] = 1.0 / sy;
            hist[1] = (head + 1) % m;
            hist[0] = cnt < m ? cnt + 1 : m;
          }
          __syncthreads();
        }
        accept_point();
        if (fstop) {
          result = 3;  // FTOL_REACHED
        } else if (xstop) {
          result = 4;  // XTOL_REACHED
        } else {
          if (!(lbfgs_direction(cd, w, bd, b, lane, false) > 0.0)) result = 1;
          alpha = 1.0;
          place = true;
        }
      } else {
        // Backtrack: minimiser of the quadratic through f, the slope dd and
        // J, kept in [0.1, 0.5] alpha.
        double an = 0.5 * alpha;
        const double den = 2.0 * (J - f - dd);
        if (std::isfinite(J) && den > 0.0)
          an = fmin(fmax(-dd * alpha / den, 0.1 * alpha), 0.5 * alpha);
        alpha = an;
        place = true;
        if (alpha < 1e-10) {
          if (w.hist[b * 2] > 0) {  // drop the curvature pairs, steepest descent
            if (!(lbfgs_direction(cd, w, bd, b, lane, true) > 0.0)) result = 1;
            alpha = 1.0;
          } else {
            result = 4;
            place = false;
          }
        }
      }
    }
    if (result == 0 && evals >= max_evals) result = 5;  // MAXEVAL_REACHED
    if (result == 0 && place) {
      bool moved = false;
      for (int i = lane; i < nv; i += kWave) {
        double v = x[i] + alpha * d[i];
        if (bd.lo) v = fmax(v, bd.lo[b * nv + i]);
        if (bd.hi) v = fmin(v, bd.hi[b * nv + i]);
        xt[i] = v;
        moved = moved || v != x[i];
      }
      if (!__any(moved)) result = 4;
    }
    if (lane == 0) {
      w.alpha[b] = alpha;
      if (result != 0) {
        w.result[b] = result;
        w.done[b] = 1;
      }
    }
  }
}

// Optimiser start: x0 clamped into the bounds, state reset.
__global__ void coll_opt_init_kernel(int64_t B, int nv, const double* __restrict__ x0,
                                     const double* __restrict__ step, Bounds bd, CollWs w) {
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  double smax = 0.0;
  for (int i = lane; i < nv; i += kWave) {
    double v = x0[b * nv + i];
    if (bd.lo) v = fmax(v, bd.lo[b * nv + i]);
    if (bd.hi) v = fmin(v, bd.hi[b * nv + i]);
    w.xt[b * nv + i] = v;
    w.x[b * nv + i] = v;
    const double s = step ? step[b * nv + i] : 0.1 * fabs(x0[b * nv + i]);  // initial_stepsize_rel
    smax = fmax(smax, fabs(s));
  }
  smax = wave_max64(smax);
  if (lane == 0) {
    w.step0[b] = smax;
    w.done[b] = 0;
    w.phase[b] = 0;
    w.evals[b] = 0;
    w.result[b] = 5;
    w.hist[b * 2] = w.hist[b * 2 + 1] = 0;
    w.alpha[b] = 1.0;
    w.f[b] = NAN;
    w.Jref0[b] = 0.0;  // total_cost_iter0_{} (polynomial_optimization_nonlinear.h:672)
    w.Jlast[b] = 0.0;  // OptimizationInfo() zeros
    for (int z = 0; z < 4; ++z) w.terms[b * 4 + z] = NAN;
    w.st[b] = MTG_TRAJ_OK;
  }
}

__global__ void coll_opt_final_kernel(int64_t B, int nv, CollWs w, double* __restrict__ x_io,
                                      double* __restrict__ cost, int32_t* __restrict__ evals,
                                      int32_t* __restrict__ result, int32_t* __restrict__ status,
                                      double* __restrict__ terms) {
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const bool ok = w.phase[b] != 0 && std::isfinite(w.f[b]);
  for (int i = lane; i < nv; i += kWave)
    if (ok) x_io[b * nv + i] = w.x[b * nv + i];
  if (lane == 0) {
    if (cost) cost[b] = w.f[b];
    if (evals) evals[b] = w.evals[b];
    if (result) result[b] = w.result[b];
    if (status) status[b] = w.st[b] != MTG_TRAJ_OK && !ok ? w.st[b] : MTG_TRAJ_OK;
    if (terms)
      for (int z = 0; z < 4; ++z) terms[b * 4 + z] = w.terms[b * 4 + z];
  }
}

unsigned grid1(int64_t n) { return static_cast<unsigned>(n); }

template <typename K>
hipError_t prepare(K kernel, size_t bytes) {
  if (bytes > 65536)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               static_cast<int>(bytes));
  return hipSuccess;
}

// One objective evaluation of the batch at xsrc (B x nv) up to the combine.
template <int N>
hipError_t evaluate_n(const PlanDev& pl, const CollDims& cd, int64_t B, const double* df,
                      const double* xsrc, const double* times, const float* occ, int nx, int ny,
                      int nz, const uint16_t* field, const mtg_coll_params& p, const CollWs& w,
                      hipStream_t st) {
  const size_t lds_prep = free_lds(N, pl.S, pl.D, pl.np, false).bytes;
  hipError_t e = prepare(coll_prep_kernel<N>, lds_prep);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(coll_prep_kernel<N>, dim3(grid1(B)), dim3(kWave), lds_prep, st, pl, cd, df,
                     times, xsrc, p.increment_time, w);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const size_t lds_walk = collision_lds_bytes(N, pl.S);
  // With the near field one thread walks alone: one wave per walk.
  hipLaunchKernelGGL(coll_walk_kernel<N>, dim3(grid1(B * cd.P)),
                     dim3(field ? kWave : kCollBlock), lds_walk, st, pl, cd, occ, nx, ny, nz,
                     field, p.coll, p.increment_time, w);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (cd.Q > 0) {
    hipLaunchKernelGGL(coll_soft_points_kernel<N>, dim3(grid1(B * cd.Q)), dim3(kWave), 0, st, pl,
                       cd, df, xsrc, p.coll.map_resolution, w);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    SoftSpec spec{};
    spec.n = p.n_soft;
    for (int c = 0; c < p.n_soft; ++c) {
      spec.derivative[c] = p.soft_derivative[c];
      spec.limit[c] = p.soft_limit[c];
    }
    spec.weight = p.soft_weight;
    spec.maximum_cost = p.soft_maximum_cost;
    spec.skip = w.done;
    spec.skip_rep = cd.Q;
    e = launch_soft_cost_any(N, pl.D, pl.S, B * cd.Q, w.softc, w.softT, spec, w.softm, w.softJ,
                             st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

#define MTG_COLL_DISPATCH(FN, ...)        \
  switch (pl.N) {                         \
    case 4: e = FN<4>(__VA_ARGS__); break;   \
    case 6: e = FN<6>(__VA_ARGS__); break;   \
    case 8: e = FN<8>(__VA_ARGS__); break;   \
    case 10: e = FN<10>(__VA_ARGS__); break; \
    case 12: e = FN<12>(__VA_ARGS__); break; \
    default: e = hipErrorInvalidValue;    \
  }

size_t coll_workspace_bytes(const PlanDev& pl, int64_t B, int mode, const mtg_coll_params& p,
                            bool optimiser) {
  const CollDims cd = coll_dims(pl, mode, p);
  CollWs w;
  return carve(nullptr, cd, pl.N, B, p.n_soft, optimiser, &w);
}

int64_t coll_problems(const PlanDev& pl, int64_t B, int mode, const mtg_coll_params& p) {
  const CollDims cd = coll_dims(pl, mode, p);
  return B * (cd.P > cd.Q ? cd.P : cd.Q);
}

int coll_cost(const PlanDev& pl, int64_t B, int mode, const double* df, const double* x,
              const double* times, const float* occ, int nx, int ny, int nz,
              const uint16_t* field, const mtg_coll_params& p, const double* raise_ref, double* cost, double* grad,
              double* terms, int32_t* collision, int32_t* status, void* workspace,
              size_t workspace_bytes, hipStream_t st) {
  const CollDims cd = coll_dims(pl, mode, p);
  if (coll_workspace_bytes(pl, B, mode, p, false) > workspace_bytes) return MTG_ERR_INVALID_ARG;
  CollWs w;
  carve(workspace, cd, pl.N, B, p.n_soft, false, &w);
  hipError_t e;
  MTG_COLL_DISPATCH(evaluate_n, pl, cd, B, df, x, times, occ, nx, ny, nz, field, p, w, st)
  if (e != hipSuccess) return MTG_ERR_HIP;
  const CombineOut o{raise_ref, cost, grad, terms, collision, status, nullptr};
  hipLaunchKernelGGL(coll_combine_kernel<false>, dim3(grid1(B)), dim3(kWave), 0, st, cd, p, 0,
                     Bounds{nullptr, nullptr}, w, o);
  return hipGetLastError() == hipSuccess ? MTG_OK : MTG_ERR_HIP;
}

int coll_optimize(const PlanDev& pl, int64_t B, int mode, const double* df, double* x_io,
                  const double* times, const double* lower, const double* upper,
                  const double* initial_step, const float* occ, int nx, int ny, int nz,
                  const uint16_t* field, const mtg_coll_params& p, int max_evals, double* cost, int32_t* evals,
                  int32_t* result, int32_t* status, double* terms, double* x_history,
                  void* workspace, size_t workspace_bytes, hipStream_t st) {
  const CollDims cd = coll_dims(pl, mode, p);
  if (coll_workspace_bytes(pl, B, mode, p, true) > workspace_bytes) return MTG_ERR_INVALID_ARG;
  CollWs w;
  carve(workspace, cd, pl.N, B, p.n_soft, true, &w);
  const Bounds bd{lower, upper};
  hipLaunchKernelGGL(coll_opt_init_kernel, dim3(grid1(B)), dim3(kWave), 0, st, B, cd.nv, x_io,
                     initial_step, bd, w);
  if (hipGetLastError() != hipSuccess) return MTG_ERR_HIP;
  CombineOut hist{};
  hist.x_history = x_history;
  for (int round = 0; round < max_evals; ++round) {
    hipError_t e;
    MTG_COLL_DISPATCH(evaluate_n, pl, cd, B, df, w.xt, times, occ, nx, ny, nz, field, p, w, st)
    if (e != hipSuccess) return MTG_ERR_HIP;
    hipLaunchKernelGGL(coll_combine_kernel<true>, dim3(grid1(B)), dim3(kWave), 0, st, cd, p,
                       max_evals, bd, w, hist);
    if (hipGetLastError() != hipSuccess) return MTG_ERR_HIP;
  }
  hipLaunchKernelGGL(coll_opt_final_kernel, dim3(grid1(B)), dim3(kWave), 0, st, B, cd.nv, w,
                     x_io, cost, evals, result, status, terms);
  return hipGetLastError() == hipSuccess ? MTG_OK : MTG_ERR_HIP;
}

}  // namespace mtg
