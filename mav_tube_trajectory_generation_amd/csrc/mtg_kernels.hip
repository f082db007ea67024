// mtg_kernels.hip — gfx950 kernels of the linear-solve and time-allocation
// hot path.  One 64-lane workgroup per trajectory; all per-trajectory state in
// LDS (mtg_device.h).  Launchers at the bottom are called by mtg_host.cpp.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_device.h"
#include "mtg_extrema_device.h"
#include "mtg_internal.h"
#include "mtg_sbplx_device.h"

namespace mtg {

// ---------------------------------------------------------------------------
// Batched linear solve (setupFromVertices' per-trajectory part +
// solveLinear + computeCost, linear_impl:277-379, 113-130).
template <int N>
__global__ __launch_bounds__(kWave) void linear_solve_kernel(
    PlanDev pl, const double* __restrict__ fixed_vals, const double* __restrict__ times,
    double* __restrict__ coeffs, double* __restrict__ cost, double* __restrict__ free_vals,
    int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int S = pl.S, D = pl.D, nf = pl.nf, np = pl.np;
  const Layout lay = make_layout(N, S, D);
  Traj<N> t{S, D, pl.r, &lay, smem, reinterpret_cast<int*>(smem + lay.ndouble),
            static_cast<int>(threadIdx.x), pl.fmask, pl.use_mask != 0};
  const int64_t b = blockIdx.x;
  MTG_STAMP(0);
  t.load_inputs(pl.tab, pl.slots, pl.fixed_map, times + b * S, fixed_vals + b * D * nf, nf);
  __syncthreads();
  MTG_STAMP(1);
  t.compute_powers();
  __syncthreads();
  MTG_STAMP(2);
  const int bad_time = t.flag()[0] & 1;
  if (!bad_time) t.solve();
  const int fl = t.flag()[0];
  const int st = (fl & 1) ? MTG_TRAJ_BAD_TIME : ((fl & 2) ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK);
  const int64_t per = static_cast<int64_t>(S) * D * N;
  if (bad_time) {
    for (int i = t.lane; i < per; i += kWave) coeffs[b * per + i] = NAN;
    if (free_vals)  // as every linear kernel: NaN free values on a bad time
      for (int i = t.lane; i < D * np; i += kWave) free_vals[b * D * np + i] = NAN;
    if (cost && t.lane == 0) cost[b] = NAN;
  } else {
    const double J = t.template coeffs_and_cost<true>(pl.tab, coeffs + b * per);
    if (cost && t.lane == 0) cost[b] = J;
    if (free_vals) {
      const int M = N / 2;
      for (int i = t.lane; i < (S + 1) * M * D; i += kWave) {
        const int sl = t.slot()[i / D];
        if (sl < 0) free_vals[b * D * np + (i % D) * np + (-sl - 1)] = t.dv()[i];
      }
    }
  }
  if (status && t.lane == 0) status[b] = st;
  MTG_STAMP(6);
}

// ---------------------------------------------------------------------------
// Coefficients and cost from given fixed and free derivatives, no solve
// (setFreeConstraints -> updateSegmentsFromCompactConstraints, linear_impl:
// 254-275, 497-506, and computeCost, :113-130).
template <int N>
__global__ __launch_bounds__(kWave) void coeffs_from_constraints_kernel(
    PlanDev pl, const double* __restrict__ fixed_vals, const double* __restrict__ free_vals,
    const double* __restrict__ times, double* __restrict__ coeffs, double* __restrict__ cost,
    int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int S = pl.S, D = pl.D, nf = pl.nf, np = pl.np;
  const Layout lay = make_layout(N, S, D);
  Traj<N> t{S, D, pl.r, &lay, smem, reinterpret_cast<int*>(smem + lay.ndouble),
            static_cast<int>(threadIdx.x), pl.fmask, pl.use_mask != 0};
  const int64_t b = blockIdx.x;
  t.load_inputs(pl.tab, pl.slots, pl.fixed_map, times + b * S, fixed_vals + b * D * nf, nf);
  for (int i = t.lane; i < D * np; i += kWave)
    t.dv()[pl.free_map[i % np] * D + i / np] = free_vals[b * D * np + i];
  __syncthreads();
  t.compute_powers();
  __syncthreads();
  const int bad_time = t.flag()[0] & 1;
  const int64_t per = static_cast<int64_t>(S) * D * N;
  if (bad_time) {
    for (int i = t.lane; i < per; i += kWave) coeffs[b * per + i] = NAN;
    if (cost && t.lane == 0) cost[b] = NAN;
  } else {
    const double J = t.template coeffs_and_cost<true>(pl.tab, coeffs + b * per);
    if (cost && t.lane == 0) cost[b] = J;
  }
  if (status && t.lane == 0) status[b] = bad_time ? MTG_TRAJ_BAD_TIME : MTG_TRAJ_OK;
}

// ---------------------------------------------------------------------------
// Per-segment matrices Q, A, A^-1, H for a batch of times (accessor parity:
// linear_impl:101-111, 132-169, 557-573, 318).  One thread per entry.
__device__ inline double falling(int n, int i) {  // base(n, i) = i!/(i-n)!
  if (i < n) return 0.0;
  double p = 1.0;
  for (int m = 0; m < n; ++m) p *= static_cast<double>(i - m);
  return p;
}

__device__ inline double ipow(double t, int e) {
  const double base = e < 0 ? 1.0 / t : t;
  const int n = e < 0 ? -e : e;
  double p = 1.0;
  for (int q = 0; q < n; ++q) p *= base;
  return p;
}

__global__ void segment_matrices_kernel(int N, int r, int64_t n,
                                        const double* __restrict__ tab,
                                        const double* __restrict__ times,
                                        double* Q, double* A, double* Ainv,
                                        double* H) {
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int NN = N * N;
  if (gid >= n * NN) return;
  const int64_t s = gid / NN;
  const int e = static_cast<int>(gid % NN);
  const int a = e / N, c = e % N;
  const int M = N / 2;
  const double T = times[s];
  if (Q) {
    double q = 0.0;
    if (a >= r && c >= r) {
      const int ex = a + c - 2 * r + 1;
      q = falling(r, a) * falling(r, c) * ipow(T, ex) * 2.0 / ex;
    }
    Q[gid] = q;
  }
  if (A) {
    const int l = a % M;
    double v;
    if (a < M)
      v = (c == l) ? falling(l, l) : 0.0;
    else
      v = c >= l ? falling(l, c) * ipow(T, c - l) : 0.0;
    A[gid] = v;
  }
  if (Ainv) Ainv[gid] = tab[NN + e] * ipow(T, (c % M) - a);
  if (H) H[gid] = tab[e] * ipow(T, 1 - 2 * r + (a % M) + (c % M));
}

// ---------------------------------------------------------------------------
// Time-allocation objective J(T) = computeCost() + time_penalty (sum T)^2
// (objectiveFunctionTime, nonlinear_impl:877-945) with optional gradient.
template <int N, bool kSoft>
__device__ double objective_at(Traj<N>& t, const double* __restrict__ tab,
                               const mtg_time_params& p, double* cbuf, double* viol) {
  *viol = 0.0;
  // Assumes T() holds the times; recomputes powers and re-solves.
  __syncthreads();
  t.compute_powers();
  __syncthreads();
  t.clear_free();
  __syncthreads();
  t.solve();
  double J;
  if constexpr (kSoft) {
    J = t.template coeffs_and_cost<true>(tab, cbuf);  // coefficients into LDS
  } else {
    J = t.cost(tab);
  }
  double tot = 0.0;
  for (int i = 0; i < t.S; ++i) tot += t.T()[i];  // nonlinear_impl:2768-2774
  J += tot * tot * p.time_penalty;
  if constexpr (kSoft) {
    // evaluateMaximumMagnitudeAsSoftConstraint (nonlinear_impl:2735-2766):
    // one extremum search per constraint over the wave, from one call site.
    __syncthreads();
    double soft = 0.0;
    for (int c = 0; c < p.n_soft; ++c) {
      int K = 0;
      double lim = 1.0;
#pragma unroll
      for (int cc = 0; cc < kMaxSoftConstraints; ++cc)  // compile-time indices
        if (cc == c) {
          K = p.soft_derivative[cc];
          lim = p.soft_limit[cc];
        }
      const double m = ext_trajectory_max_wave_k<N>(K, cbuf, t.T(), t.S, t.D, t.lane);
      if (p.hard_constraints) {  // evaluateMaximumMagnitudeConstraint (:2687-2733)
        *viol = fmax(*viol, m - lim - p.hard_tolerance);
      } else {
        const double relative_violation = (m - lim) / lim;
        soft += fmin(p.soft_maximum_cost, exp(relative_violation * p.soft_weight));
      }
    }
    J += soft;
  }
  __syncthreads();
  return J;
}

// LDS for the soft-constraint objective's coefficients, after the layout.
__host__ __device__ inline size_t soft_cbuf_offset(const Layout& lay) {
  return (lay.bytes() + 15) / 16 * 16;
}
// The optimiser's LN_SBPLX state (mtg_sbplx_device.h) after everything else.
__host__ __device__ inline size_t sbplx_state_offset(const Layout& lay, int S, int D, int N,
                                                     bool soft) {
  const size_t end = soft ? soft_cbuf_offset(lay) + sizeof(double) * S * D * N : lay.bytes();
  return (end + 15) / 16 * 16;
}

// The reference's getCostAndGradientTime (grad_mode 1): with d held at the
// base solution (dv), J_d(T') differs from J_d(T) only in segment n's block
// (nonlinear_impl:2495-2584).  No re-solve.  Gradient written to g (LDS).
template <int N>
__device__ void gradient_fixed_d(Traj<N>& t, const mtg_time_params& p, double* g) {
  const double inc = p.increment;
  for (int n = 0; n < t.S; ++n) {
    const double Tn = t.T()[n];
    const double ts = Tn <= 0.1 ? 0.1 : Tn - inc;  // nonlinear_impl:2529-2530
    const double tb = Tn <= 0.1 ? 0.1 : Tn + inc;
    const double qs = t.seg_energy_at(n, ts);
    const double qb = t.seg_energy_at(n, tb);
    if (t.lane == 0) g[n] = p.w_d * (qb - qs) / (2.0 * inc) + p.w_t * 1.0;
  }
  __syncthreads();
}

// Central-difference point of gradient step gi (0 .. 2S-1) around base
// times Tb: segment n = gi / 2 at T_n - inc (even gi) or T_n + inc (odd),
// both clamped to 0.1 when T_n <= 0.1 (nonlinear_impl:2529-2530).
template <int N>
__device__ void set_fd_point(Traj<N>& t, const double* Tb, int gi, double inc) {
  const int n = gi >> 1;
  if (t.lane == 0) {
    for (int i = 0; i < t.S; ++i) t.T()[i] = Tb[i];
    const double Tn = Tb[n];
    t.T()[n] = Tn <= 0.1 ? 0.1 : ((gi & 1) ? Tn + inc : Tn - inc);
  }
  __syncthreads();
}

// Every objective evaluation of the two kernels below goes through ONE call
// site of objective_at (a loop over evaluation points), so the solver body
// is instantiated once per kernel and stays within the register file.
template <int N, bool kSoft>
__global__ __launch_bounds__(kWave) void time_cost_kernel(
    PlanDev pl, const double* __restrict__ fixed_vals, const double* __restrict__ times,
    mtg_time_params p, double* __restrict__ cost, double* __restrict__ grad,
    int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int S = pl.S, D = pl.D, nf = pl.nf;
  const double* tab = pl.tab;
  const Layout lay = make_layout(N, S, D);
  Traj<N> t{S, D, pl.r, &lay, smem, reinterpret_cast<int*>(smem + lay.ndouble),
            static_cast<int>(threadIdx.x), pl.fmask, pl.use_mask != 0};
  const int64_t b = blockIdx.x;
  double* cbuf = reinterpret_cast<double*>(reinterpret_cast<char*>(smem) + soft_cbuf_offset(lay));
  double* g = smem + lay.aux;   // gradient
  double* Tb = g + S;           // base times
  t.load_inputs(pl.tab, pl.slots, pl.fixed_map, times + b * S, fixed_vals + b * D * nf, nf);
  for (int i = t.lane; i < S; i += kWave) Tb[i] = times[b * S + i];
  const bool fd = grad && p.grad_mode == 2;
  const int nevals = 1 + (fd ? 2 * S : 0);
  double J0 = 0.0, Jlo = 0.0;
  int fl = 0;
  for (int e = 0; e < nevals; ++e) {
    if (e > 0) set_fd_point(t, Tb, e - 1, p.increment);
    double viol;
    const double J = objective_at<N, kSoft>(t, tab, p, cbuf, &viol);
    if (e == 0) {
      J0 = J;
      fl = t.flag()[0];
      if (fl & 1) break;
    } else if ((e - 1) & 1) {
      if (t.lane == 0) g[(e - 1) >> 1] = (J - Jlo) / (2.0 * p.increment);
    } else {
      Jlo = J;
    }
  }
  __syncthreads();
  if (grad && p.grad_mode == 1 && !(fl & 1)) gradient_fixed_d(t, p, g);
  const int fl2 = t.flag()[0];
  if (t.lane == 0) {
    if (cost) cost[b] = (fl & 1) ? NAN : J0;
    if (status)
      status[b] = (fl2 & 1) ? MTG_TRAJ_BAD_TIME
                            : ((fl2 & 2) ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK);
  }
  if (grad && p.grad_mode != 0)
    for (int i = t.lane; i < S; i += kWave) grad[b * S + i] = (fl & 1) ? NAN : g[i];
}

// ---------------------------------------------------------------------------
// Batched segment-time optimisation (optimizeTime, nonlinear_impl:332-397):
// bounds [0.1, 2 T0]; projected, scaled steepest descent on the grad_mode 2
// gradient with an expand/backtrack step rule; `max_evals` objective
// evaluations (NLopt maxeval semantics, nonlinear_impl:101; gradient
// evaluations are not counted).  Written as a state machine with one
// objective evaluation per loop trip.
template <int N, bool kSoft>
__global__ __launch_bounds__(kWave) void time_optimize_kernel(
    PlanDev pl, const double* __restrict__ fixed_vals, double* __restrict__ times_io,
    mtg_time_params p, int max_evals, double* __restrict__ cost,
    int32_t* __restrict__ evals_out, int32_t* __restrict__ solves_out,
    int32_t* __restrict__ result_out, int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int S = pl.S, D = pl.D, nf = pl.nf;
  const double* tab = pl.tab;
  const Layout lay = make_layout(N, S, D);
  Traj<N> t{S, D, pl.r, &lay, smem, reinterpret_cast<int*>(smem + lay.ndouble),
            static_cast<int>(threadIdx.x), pl.fmask, pl.use_mask != 0};
  const int64_t b = blockIdx.x;
  double* cbuf = reinterpret_cast<double*>(reinterpret_cast<char*>(smem) + soft_cbuf_offset(lay));
  double* Tcur = smem + lay.aux;   // accepted times
  double* T0 = Tcur + S;           // initial times (bounds)
  double* g = T0 + S;              // gradient at Tcur
  double* gv = g + S;              // gradient of the violation (hard constraints)
  t.load_inputs(pl.tab, pl.slots, pl.fixed_map, times_io + b * S, fixed_vals + b * D * nf, nf);
  for (int i = t.lane; i < S; i += kWave) {
    const double v = times_io[b * S + i];
    Tcur[i] = v;
    T0[i] = v;
  }
  constexpr double kLower = 0.1;  // kOptimizationTimeLowerBound (:370)
  enum { kBase, kGrad, kTrial, kDone };
  int phase = kBase, gi = 0, evals = 0, nsolve = 0, res = 0;
  double f = 0.0, fv = 0.0, Jlo = 0.0, vlo = 0.0;
  double alpha = 0.1;  // initial_stepsize_rel (polynomial_optimization_nonlinear.h:55)
  int fl = 0;
  // LN_SBPLX (optimizer 1): the machine picks every point, lane 0 advances it
  const bool sb = p.optimizer == 1;
  auto* sbs = reinterpret_cast<sbplx::State*>(reinterpret_cast<char*>(smem) +
                                              sbplx_state_offset(lay, S, D, N, kSoft));
  sbplx::Machine mach{sbs};
  if (sb) {
    __syncthreads();
    if (t.lane == 0)
      mach.init(S, t.T(), p.initial_stepsize_rel > 0.0 ? p.initial_stepsize_rel : 0.1,
                max_evals, p.f_rel, p.f_abs);
    __syncthreads();
    if (sbs->done) phase = kDone;  // start outside the bounds (NLopt: FAILURE)
  }
  while (phase != kDone) {
    double viol;
    const double J = objective_at<N, kSoft>(t, tab, p, cbuf, &viol);  // at T()
    ++nsolve;
    if (sb) {
      if (t.flag()[0] & 1) break;
      __syncthreads();
      if (t.lane == 0) mach.resume(J, t.T());
      __syncthreads();
      if (sbs->done) break;
      continue;
    }
    if (phase == kBase) {
      f = J;
      fv = viol;
      evals = 1;
      fl = t.flag()[0];
      if (fl & 1) break;
      phase = kGrad;
      gi = 0;
    } else if (phase == kGrad) {
      if (gi & 1) {
        if (t.lane == 0) {
          g[gi >> 1] = (J - Jlo) / (2.0 * p.increment);
          gv[gi >> 1] = (viol - vlo) / (2.0 * p.increment);
        }
      } else {
        Jlo = J;
        vlo = viol;
      }
      if (++gi == 2 * S) phase = kTrial;
    } else {  // trial point
      ++evals;
      // Feasibility first (hard constraints; viol is 0 otherwise).
      if (viol == 0.0 ? (fv > 0.0 || J < f) : viol < fv) {
        f = J;
        fv = viol;
        if (t.lane == 0)
          for (int i = 0; i < S; ++i) Tcur[i] = t.T()[i];
        alpha = fmin(alpha * 1.5, 1.0);
        phase = kGrad;
        gi = 0;
      } else {
        alpha *= 0.5;
      }
    }
    __syncthreads();
    // Next evaluation point.
    if (phase == kGrad) {
      set_fd_point(t, Tcur, gi, p.increment);
    } else if (phase == kTrial) {
      if (!(evals < max_evals && alpha > 1e-9)) break;
      // Scaled direction -g_n T0_n, normalised so the largest relative move
      // is alpha; from an infeasible incumbent (hard constraints) the
      // direction descends the violation instead.
      const double* dir = fv > 0.0 ? gv : g;
      double gmax = 0.0;
      for (int i = 0; i < S; ++i) gmax = fmax(gmax, fabs(dir[i] * T0[i]));
      if (!(gmax > 0.0)) break;
      int moved = 0;
      for (int i = 0; i < S; ++i) {
        const double step = alpha * T0[i] * (dir[i] * T0[i]) / gmax;
        double tn = Tcur[i] - step;
        tn = fmin(fmax(tn, kLower), 2.0 * T0[i]);
        if (tn != Tcur[i]) moved = 1;
        if (t.lane == 0) t.T()[i] = tn;
      }
      __syncthreads();
      if (!moved) break;
    }
  }
  fl = t.flag()[0];
  __syncthreads();
  if (sb) {  // NLopt's x and opt_f: the best point and its value
    for (int i = t.lane; i < S; i += kWave) Tcur[i] = sbplx::best_x(sbs)[i];
    f = sbs->minf;
    evals = sbs->nevals;
    res = sbs->result;
    __syncthreads();
  } else {
    res = evals >= max_evals ? sbplx::kMaxEval : sbplx::kXtol;
  }
  for (int i = t.lane; i < S; i += kWave) times_io[b * S + i] = Tcur[i];
  if (t.lane == 0) {
    if (cost) cost[b] = (fl & 1) ? NAN : f;
    if (evals_out) evals_out[b] = evals;
    if (solves_out) solves_out[b] = nsolve;
    if (result_out) result_out[b] = res;
    if (status)
      status[b] = (fl & 1) ? MTG_TRAJ_BAD_TIME
                           : ((fl & 2) ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK);
  }
}

// ---------------------------------------------------------------------------
// Launchers.
namespace {
template <typename K>
hipError_t prepare_lds(K kernel, size_t bytes) {
  if (bytes > 65536)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               static_cast<int>(bytes));
  return hipSuccess;
}
}  // namespace

template <int N>
static hipError_t launch_linear_n(const PlanDev& pl, int64_t B, const double* df,
                                  const double* times, double* coeffs, double* cost,
                                  double* free_vals, int32_t* status, hipStream_t st) {
  const size_t bytes = make_layout(N, pl.S, pl.D).bytes();
  hipError_t e = prepare_lds(linear_solve_kernel<N>, bytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(linear_solve_kernel<N>, dim3(static_cast<unsigned>(B)), dim3(kWave),
                     bytes, st, pl, df, times, coeffs, cost, free_vals, status);
  return hipGetLastError();
}

template <int N>
static hipError_t launch_coeffs_n(const PlanDev& pl, int64_t B, const double* df,
                                  const double* dp, const double* times, double* coeffs,
                                  double* cost, int32_t* status, hipStream_t st) {
  const size_t bytes = make_layout(N, pl.S, pl.D).bytes();
  hipError_t e = prepare_lds(coeffs_from_constraints_kernel<N>, bytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(coeffs_from_constraints_kernel<N>, dim3(static_cast<unsigned>(B)),
                     dim3(kWave), bytes, st, pl, df, dp, times, coeffs, cost, status);
  return hipGetLastError();
}

template <int N>
static hipError_t launch_time_cost_n(const PlanDev& pl, int64_t B, const double* df,
                                     const double* times, const mtg_time_params& p,
                                     double* cost, double* grad, int32_t* status,
                                     hipStream_t st) {
  const Layout lay = make_layout(N, pl.S, pl.D);
  if (p.n_soft > 0) {
    const size_t bytes = soft_cbuf_offset(lay) + sizeof(double) * pl.S * pl.D * N;
    hipError_t e = prepare_lds(time_cost_kernel<N, true>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_cost_kernel<N, true>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, times, p, cost, grad, status);
  } else {
    const size_t bytes = lay.bytes();
    hipError_t e = prepare_lds(time_cost_kernel<N, false>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_cost_kernel<N, false>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, times, p, cost, grad, status);
  }
  return hipGetLastError();
}

template <int N>
static hipError_t launch_time_opt_n(const PlanDev& pl, int64_t B, const double* df,
                                    double* times, const mtg_time_params& p,
                                    int max_evals, double* cost, int32_t* evals,
                                    int32_t* solves, int32_t* result, int32_t* status,
                                    hipStream_t st) {
  const Layout lay = make_layout(N, pl.S, pl.D);
  if (p.n_soft > 0) {
    const size_t bytes =
        sbplx_state_offset(lay, pl.S, pl.D, N, true) + sbplx::state_bytes(pl.S);
    hipError_t e = prepare_lds(time_optimize_kernel<N, true>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_optimize_kernel<N, true>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, times, p, max_evals, cost, evals, solves,
                       result, status);
  } else {
    const size_t bytes =
        sbplx_state_offset(lay, pl.S, pl.D, N, false) + sbplx::state_bytes(pl.S);
    hipError_t e = prepare_lds(time_optimize_kernel<N, false>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_optimize_kernel<N, false>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, times, p, max_evals, cost, evals, solves,
                       result, status);
  }
  return hipGetLastError();
}

#define MTG_DISPATCH_N(N_, CALL)     \
  switch (N_) {                      \
    case 4: return CALL(4);          \
    case 6: return CALL(6);          \
    case 8: return CALL(8);          \
    case 10: return CALL(10);        \
    case 12: return CALL(12);        \
    default: return hipErrorInvalidValue; \
  }

int linear_kernel_for_batch(const PlanDev& pl, int64_t B) {
  if (pl.kernel != MTG_KERNEL_AUTO) return pl.kernel;
  if (!pl.std_pattern) return MTG_KERNEL_GENERIC;
  if (has_linear_lane(pl) && B >= kLaneMinBatch) return MTG_KERNEL_LANE_PAIR;
  // The same test launch_linear_solve applies (std_pattern already implies
  // S <= kMaxStdS), so the reported kernel is the one that runs.
  return use_std_kernel(pl) ? MTG_KERNEL_STANDARD : MTG_KERNEL_GENERIC;
}

int64_t select_partials(const PlanDev& pl, int64_t B) {
  const int k = linear_kernel_for_batch(pl, B);
  if (k == MTG_KERNEL_LANE) return lane_blocks(B);
  if (k == MTG_KERNEL_LANE_PAIR) return lane2_blocks(B);
  return 0;  // one trajectory per workgroup: the costs are the partials
}

hipError_t launch_linear_solve(const PlanDev& pl, int64_t B, const double* df,
                               const double* times, double* coeffs, double* cost,
                               double* free_vals, int32_t* status, hipStream_t st,
                               const SelectArgs& sel) {
  const int k = linear_kernel_for_batch(pl, B);
  // A deferred selection (the previous step's costs, SelectArgs::prev_*):
  // an extra workgroup of the wave and lane-pair launches; a launch of its
  // own before the other kernels.
  SelectArgs own = sel;
  const bool prev_inside = k == MTG_KERNEL_LANE_PAIR || (k == MTG_KERNEL_STANDARD);
  if (sel.prev_out && !prev_inside) {
    const hipError_t e = launch_select_local(sel.prev_cost, sel.prev_count, sel.prev_start,
                                             sel.rank, sel.prev_out, st);
    if (e != hipSuccess) return e;
    own.prev_out = nullptr;
  }
  // Lane kernels: per-workgroup partials in the epilogue, then one small
  // reduction launch.  Wavefront kernels (one trajectory per workgroup): the
  // reduction reads the costs.
  if (k == MTG_KERNEL_LANE || k == MTG_KERNEL_LANE_PAIR) {
    const hipError_t e =
        k == MTG_KERNEL_LANE
            ? launch_linear_solve_lane(pl, B, df, times, coeffs, cost, free_vals, status, st, own)
            : launch_linear_solve_lane2(pl, B, df, times, coeffs, cost, free_vals, status, st,
                                        own);
    if (e != hipSuccess || !sel.out) return e;
    const int64_t n = k == MTG_KERNEL_LANE ? lane_blocks(B) : lane2_blocks(B);
    return launch_select_reduce(sel.part_cost, sel.part_idx, n, B, sel.start, sel.rank, sel.out,
                                st);
  }
  hipError_t e;
  if (use_std_kernel(pl)) {
    e = launch_linear_solve_std(pl, B, df, times, coeffs, cost, free_vals, status, st, own);
    if (e != hipSuccess || !sel.out) return e;
    return launch_select_local(cost, B, sel.start, sel.rank, sel.out, st);
  }
#define CALL(n) launch_linear_n<n>(pl, B, df, times, coeffs, cost, free_vals, status, st)
  switch (pl.N) {
    case 4: e = CALL(4); break;
    case 6: e = CALL(6); break;
    case 8: e = CALL(8); break;
    case 10: e = CALL(10); break;
    case 12: e = CALL(12); break;
    default: return hipErrorInvalidValue;
  }
#undef CALL
  if (e != hipSuccess || !sel.out) return e;
  return launch_select_local(cost, B, sel.start, sel.rank, sel.out, st);
}

hipError_t launch_coeffs_from_constraints(const PlanDev& pl, int64_t B, const double* df,
                                          const double* dp, const double* times,
                                          double* coeffs, double* cost, int32_t* status,
                                          hipStream_t st) {
#define CALL(n) launch_coeffs_n<n>(pl, B, df, dp, times, coeffs, cost, status, st)
  MTG_DISPATCH_N(pl.N, CALL)
#undef CALL
}

hipError_t launch_time_cost(const PlanDev& pl, int64_t B, const double* df,
                            const double* times, const mtg_time_params& p,
                            double* cost, double* grad, int32_t* status,
                            hipStream_t st) {
  if (has_time_std(pl)) return launch_time_cost_std(pl, B, df, times, p, cost, grad, status, st);
#define CALL(n) launch_time_cost_n<n>(pl, B, df, times, p, cost, grad, status, st)
  MTG_DISPATCH_N(pl.N, CALL)
#undef CALL
}

hipError_t launch_time_optimize(const PlanDev& pl, int64_t B, const double* df,
                                double* times, const mtg_time_params& p, int max_evals,
                                double* cost, int32_t* evals, int32_t* solves,
                                int32_t* result, int32_t* status, hipStream_t st) {
  if (has_time_std(pl))
    return launch_time_optimize_std(pl, B, df, times, p, max_evals, cost, evals, solves, result,
                                    status, st);
#define CALL(n) \
  launch_time_opt_n<n>(pl, B, df, times, p, max_evals, cost, evals, solves, result, status, st)
  MTG_DISPATCH_N(pl.N, CALL)
#undef CALL
}

hipError_t launch_segment_matrices(int N, int r, int64_t n, const double* tab,
                                   const double* times, double* Q, double* A,
                                   double* Ainv, double* H, hipStream_t st) {
  const int64_t total = n * N * N;
  const int threads = 256;
  const int64_t blocks = (total + threads - 1) / threads;
  hipLaunchKernelGGL(segment_matrices_kernel, dim3(static_cast<unsigned>(blocks)),
                     dim3(threads), 0, st, N, r, n, tab, times, Q, A, Ainv, H);
  return hipGetLastError();
}

size_t linear_lds_bytes(int N, int S, int D) { return make_layout(N, S, D).bytes(); }

#ifdef MTG_STAMPS
extern "C" int mtg_debug_stamps(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mtg_stamps), sizeof(unsigned long long) * n) ==
                 hipSuccess ? 0 : -3;
}
#endif

}  // namespace mtg
