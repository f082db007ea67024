// mtg_time_std.hip — the time-allocation objective and the batched
// segment-time optimiser (objectiveFunctionTime / getCostAndGradientTime /
// optimizeTime, nonlinear_impl:877-945, 2495-2584, 332-397) for the standard
// vertex pattern, on the standard-pattern solver (stdp::Solver,
// mtg_std_device.h).  Same objective, gradient modes and optimiser state
// machine as the generic kernels (mtg_kernels.hip: time_cost_kernel,
// time_optimize_kernel); instantiated for N = 10, r = 2..4, D = 1..3 (other
// combinations run the generic kernels).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>

#include "mtg_extrema_device.h"
#include "mtg_sbplx_device.h"
#include "mtg_std_device.h"
#include "mtg_wave_device.h"

namespace mtg {

namespace {

template <int N, int R, int D>
using StdSv = stdp::Solver<N, R, D>;

// The inner solve and computeCost at the times T (LDS) on either solver:
// stdp::Solver (runtime S) or wave::Solver (compile-time S, the C2 design).
// Every lane calls; *bad is set (and NaN returned) when a time is invalid;
// with cbuf the coefficients go there (LDS, soft searches).
template <int N, int R, int D>
__device__ __attribute__((always_inline)) double solve_cost(
    stdp::Solver<N, R, D>& sv, const double* __restrict__ tab, const double* T, double* cbuf,
    bool reload_rows, bool* bad, bool* not_spd) {
  __syncthreads();
  const bool b = sv.powers_from(T);
  __syncthreads();
  if (b) {
    *bad = true;
    return NAN;
  }
  // soft: the H(1) rows are reloaded per evaluation (L2 hits), so they are
  // not live across the extremum searches.
  if (reload_rows) sv.load_first_rows(tab);
  sv.assemble(tab);
  __syncthreads();
  *not_spd = sv.solve() || *not_spd;
  return sv.coeff_cost(cbuf);
}

template <int N, int R, int D, int S>
__device__ __attribute__((always_inline)) double solve_cost(
    wave::Solver<N, R, D, S>& sv, const double* __restrict__ /*tab*/, const double* T,
    double* cbuf, bool /*reload_rows*/, bool* bad, bool* not_spd) {
  __syncthreads();
  const int l = sv.lane;
  const double t = T[l < S ? l : S - 1];
  if (__any(l < S && (!(t > 0.0) || !(t < 1e300)))) {
    *bad = true;
    return NAN;
  }
  *not_spd = sv.solve(T) || *not_spd;
  return sv.coeff_cost(T, cbuf);
}

// J(T) = computeCost() + time_penalty (sum T)^2 [+ soft constraints] at the
// times T (LDS, S values).  Every lane calls it; returns the wave-uniform J
// (NaN and *bad set when a time is invalid).  kSoft: the coefficients go to
// cbuf (LDS) and evaluateMaximumMagnitudeAsSoftConstraint
// (nonlinear_impl:2735-2766) runs one extremum search per constraint; with
// p.hard_constraints the searches give *viol = max(0, max_c (max_c - limit_c
// - tolerance)) (evaluateMaximumMagnitudeConstraint, :2687-2733) instead of
// a cost term.
template <int N, int D, bool kSoft, class SV>
__device__ __attribute__((always_inline)) double std_objective(SV& sv, const double* __restrict__ tab,
                                const double* T, int S, const mtg_time_params& p, double* cbuf,
                                bool* bad, bool* not_spd, double* viol) {
  *viol = 0.0;
  unsigned long long tt = 0;
  MTG_TACC(511, tt);
  double J = solve_cost(sv, tab, T, kSoft ? cbuf : nullptr, kSoft, bad, not_spd);
  if (*bad) return NAN;
  double tot = 0.0;
  for (int i = 0; i < S; ++i) tot += T[i];  // nonlinear_impl:2768-2774
  J += tot * tot * p.time_penalty;
  MTG_TACC(450, tt);  // diagnostic: solve + coefficients
  if constexpr (kSoft) {
    __syncthreads();
    // Every constraint's maximum in one pass (ext_soft_maxima_wave).
    int Ks[kMaxSoftConstraints];
    int kmin = 4;
#pragma unroll
    for (int cc = 0; cc < kMaxSoftConstraints; ++cc) {
      Ks[cc] = p.soft_derivative[cc];
      if (cc < p.n_soft && Ks[cc] < kmin) kmin = Ks[cc];
    }
    double* scratch = cbuf + S * D * N;
    double* maxima = scratch + kMaxSoftConstraints * (N + 1);
    ext_soft_maxima_wave_k<N>(kmin, cbuf, T, S, D, sv.lane, p.n_soft, Ks, scratch, maxima);
    double soft = 0.0;
    for (int c = 0; c < p.n_soft; ++c) {
      double lim = 1.0;
#pragma unroll
      for (int cc = 0; cc < kMaxSoftConstraints; ++cc)  // compile-time indices
        if (cc == c) lim = p.soft_limit[cc];
      const double m = maxima[c];
      if (p.hard_constraints) {
        *viol = fmax(*viol, m - lim - p.hard_tolerance);
      } else {
        const double relative_violation = (m - lim) / lim;
        soft += fmin(p.soft_maximum_cost, exp(relative_violation * p.soft_weight));
      }
      MTG_TACC(451 + c, tt);  // diagnostic
    }
    J += soft;
  }
  return J;
}

// Loads d_f (and, for wave::Solver, H(1)) into the solver (all lanes).
template <int N, int R, int D>
__device__ void std_load_fixed(StdSv<N, R, D>& sv, const double* __restrict__ /*tab*/,
                               const double* __restrict__ fb) {
  const int nf = sv.nf;
  for (int i = sv.lane; i < D * nf; i += kWave) sv.put_fixed(i, fb[i]);
}
template <int N, int R, int D, int S>
__device__ void std_load_fixed(wave::Solver<N, R, D, S>& sv, const double* __restrict__ tab,
                               const double* __restrict__ fb) {
  sv.load_constants(tab, fb);
  wave::lds_order();
}

// Central-difference point gi (0 .. 2S-1) around base times Tb: segment
// n = gi / 2 at T_n - inc (even gi) or T_n + inc (odd), both clamped to 0.1
// when T_n <= 0.1 (nonlinear_impl:2529-2530).
__device__ inline void std_set_fd_point(double* T, const double* Tb, int S, int gi, double inc,
                                        int lane) {
  const int n = gi >> 1;
  for (int i = lane; i < S; i += kWave) {
    const double Tn = Tb[i];
    T[i] = i != n ? Tn : (Tn <= 0.1 ? 0.1 : ((gi & 1) ? Tn + inc : Tn - inc));
  }
}

}  // namespace

__host__ __device__ inline size_t time_std_bytes(int N, int S, int D, bool soft) {
  const size_t base = sizeof(double) * static_cast<size_t>(stdp::layout(N, S, D).n);
  // soft: the coefficients (S x D x N), then the soft searches' scratch and
  // maxima (ext_soft_maxima_wave).
  return soft ? (base + 15) / 16 * 16 +
                    sizeof(double) * (S * D * N + kMaxSoftConstraints * (N + 2))
              : base;
}
size_t time_std_lds_bytes(int N, int S, int D, bool soft) { return time_std_bytes(N, S, D, soft); }
// The optimiser kernels add the LN_SBPLX machine's state after that.
static size_t time_std_opt_lds_bytes(int N, int S, int D, bool soft) {
  return (time_std_bytes(N, S, D, soft) + 15) / 16 * 16 + sbplx::state_bytes(S);
}

// objectiveFunctionTime / getCostAndGradientTime on one trajectory per
// workgroup (either solver; cbuf: the soft searches' LDS).
template <int N, int D, bool kSoft, class SV>
__device__ __attribute__((always_inline)) void time_cost_body(
    SV& sv, int S, const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    const double* __restrict__ times, const mtg_time_params& p, double* __restrict__ cost,
    double* __restrict__ grad, int32_t* __restrict__ status, double* cbuf) {
  const int64_t b = blockIdx.x;
  const int lane = sv.lane;
  const int nf = N + S - 1;
  double* T = sv.aux();  // evaluation point
  double* Tb = T + S;    // base times
  double* g = Tb + S;    // gradient
  double* E = g + S;     // 2S segment energies (grad_mode 1)
  std_load_fixed(sv, tab, fixed_vals + b * D * nf);
  for (int i = lane; i < S; i += kWave) T[i] = Tb[i] = times[b * S + i];
  const bool fd = grad && p.grad_mode == 2;
  const int nevals = 1 + (fd ? 2 * S : 0);
  double J0 = 0.0, Jlo = 0.0;
  bool bad = false, not_spd = false;
  for (int e = 0; e < nevals; ++e) {
    if (e > 0) std_set_fd_point(T, Tb, S, e - 1, p.increment, lane);
    double viol;
    const double J = std_objective<N, D, kSoft>(sv, tab, T, S, p, cbuf, &bad, &not_spd, &viol);
    if (e == 0) {
      J0 = J;
      if (bad) break;
    } else if ((e - 1) & 1) {
      if (lane == 0) g[(e - 1) >> 1] = (J - Jlo) / (2.0 * p.increment);
    } else {
      Jlo = J;
    }
  }
  __syncthreads();
  if (grad && p.grad_mode == 1 && !bad) {
    // getCostAndGradientTime (nonlinear_impl:2495-2584): d held at the base
    // solution, only segment n's block of J_d = d^T R d changes.
    const double inc = p.increment;
    for (int i = lane; i < 2 * S; i += kWave) {
      const int n = i >> 1;
      const double Tn = Tb[n];
      const double tau = Tn <= 0.1 ? 0.1 : ((i & 1) ? Tn + inc : Tn - inc);
      E[i] = sv.seg_energy(n, tau);
    }
    __syncthreads();
    for (int n = lane; n < S; n += kWave)
      g[n] = p.w_d * (E[2 * n + 1] - E[2 * n]) / (2.0 * inc) + p.w_t * 1.0;
    __syncthreads();
  }
  if (lane == 0) {
    if (cost) cost[b] = bad ? NAN : J0;
    if (status)
      status[b] = bad ? MTG_TRAJ_BAD_TIME : (not_spd ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK);
  }
  if (grad && p.grad_mode != 0)
    for (int i = lane; i < S; i += kWave) grad[b * S + i] = bad ? NAN : g[i];
}

template <int N, int R, int D, bool kSoft>
__global__ __launch_bounds__(kWave) void time_cost_std_kernel(
    int S, const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    const double* __restrict__ times, mtg_time_params p, double* __restrict__ cost,
    double* __restrict__ grad, int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  StdSv<N, R, D> sv;
  sv.init(S, smem, tab);
  time_cost_body<N, D, kSoft>(sv, S, tab, fixed_vals, times, p, cost, grad, status,
                              smem + (sv.L.n + 1) / 2 * 2);
}

// The same on the compile-time-S solver (N = 10, r = 4, D = 3, S = 2..16).
template <int N, int R, int D, int S, bool kSoft>
__global__ __launch_bounds__(kWave) void time_cost_wave_kernel(
    const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    const double* __restrict__ times, mtg_time_params p, double* __restrict__ cost,
    double* __restrict__ grad, int32_t* __restrict__ status) {
  using G = wave::Geo<N, R, D, S>;
  constexpr int CB = kSoft ? S * D * N + kMaxSoftConstraints * (N + 2) : 0;
  __shared__ __attribute__((aligned(16))) double sm[G::L_N + CB];
  wave::Solver<N, R, D, S> sv;
  sv.init(sm);
  time_cost_body<N, D, kSoft>(sv, S, tab, fixed_vals, times, p, cost, grad, status,
                              sm + G::L_N);
}

// Batched segment-time optimisation (optimizeTime, nonlinear_impl:332-397):
// bounds [0.1, 2 T0]; projected, scaled steepest descent on the grad_mode 2
// gradient with an expand/backtrack step rule; `max_evals` objective
// evaluations (NLopt maxeval semantics, nonlinear_impl:101; gradient
// evaluations are not counted).  A state machine with one objective call
// site, as time_optimize_kernel.
template <int N, int D, bool kSoft, class SV>
__device__ __attribute__((always_inline)) void time_optimize_body(
    SV& sv, int S, const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    double* __restrict__ times_io, const mtg_time_params& p, int max_evals,
    double* __restrict__ cost, int32_t* __restrict__ evals_out, int32_t* __restrict__ solves_out,
    int32_t* __restrict__ result_out, int32_t* __restrict__ status, double* cbuf,
    sbplx::State* sbs) {
  const int64_t b = blockIdx.x;
  const int lane = sv.lane;
  const int nf = N + S - 1;
  double* T = sv.aux();   // evaluation point
  double* Tcur = T + S;   // accepted times
  double* T0 = Tcur + S;  // initial times (bounds)
  double* g = T0 + S;     // gradient at Tcur
  double* gv = g + S;     // gradient of the violation at Tcur (hard constraints)
  std_load_fixed(sv, tab, fixed_vals + b * D * nf);
  for (int i = lane; i < S; i += kWave) T[i] = Tcur[i] = T0[i] = times_io[b * S + i];
  constexpr double kLower = 0.1;  // kOptimizationTimeLowerBound (:370)
  enum { kBase, kGrad, kTrial, kDone };
  int phase = kBase, gi = 0, evals = 0, nsolve = 0, res = 0;
  double f = 0.0, fv = 0.0, Jlo = 0.0, vlo = 0.0;
  double alpha = 0.1;  // initial_stepsize_rel (polynomial_optimization_nonlinear.h:55)
  bool bad = false, not_spd = false;
  // LN_SBPLX (optimizer 1): the machine picks every point, lane 0 advances it
  const bool sb = p.optimizer == 1;
  sbplx::Machine mach{sbs};
  if (sb) {
    __syncthreads();
    if (lane == 0)
      mach.init(S, T, p.initial_stepsize_rel > 0.0 ? p.initial_stepsize_rel : 0.1, max_evals,
                p.f_rel, p.f_abs);
    __syncthreads();
    if (sbs->done) phase = kDone;  // start outside the bounds (NLopt: FAILURE)
  }
  MTG_STAMP(460);
  while (phase != kDone) {
    double viol;
    const double J = std_objective<N, D, kSoft>(sv, tab, T, S, p, cbuf, &bad, &not_spd, &viol);
    ++nsolve;
    if (sb) {
      if (bad) break;
      __syncthreads();
      if (lane == 0) mach.resume(J, T);
      __syncthreads();
      if (sbs->done) break;
      continue;
    }
    if (phase == kBase) {
      f = J;
      fv = viol;
      evals = 1;
      if (bad) break;
      phase = kGrad;
      gi = 0;
    } else if (phase == kGrad) {
      if (gi & 1) {
        if (lane == 0) {
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
        for (int i = lane; i < S; i += kWave) Tcur[i] = T[i];
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
      std_set_fd_point(T, Tcur, S, gi, p.increment, lane);
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
        if (lane == 0) T[i] = tn;
      }
      __syncthreads();
      if (!moved) break;
    }
  }
  __syncthreads();
  MTG_STAMP(461);
  if (sb) {  // NLopt's x and opt_f: the best point and its value
    for (int i = lane; i < S; i += kWave) Tcur[i] = sbplx::best_x(sbs)[i];
    f = sbs->minf;
    evals = sbs->nevals;
    res = sbs->result;
    __syncthreads();
  } else {
    res = evals >= max_evals ? sbplx::kMaxEval : sbplx::kXtol;
  }
  for (int i = lane; i < S; i += kWave) times_io[b * S + i] = Tcur[i];
  if (lane == 0) {
    if (cost) cost[b] = bad ? NAN : f;
    if (evals_out) evals_out[b] = evals;
    if (solves_out) solves_out[b] = nsolve;
    if (result_out) result_out[b] = res;
    if (status)
      status[b] = bad ? MTG_TRAJ_BAD_TIME : (not_spd ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK);
  }
}

template <int N, int R, int D, bool kSoft>
__global__ __launch_bounds__(kWave) void time_optimize_std_kernel(
    int S, const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    double* __restrict__ times_io, mtg_time_params p, int max_evals,
    double* __restrict__ cost, int32_t* __restrict__ evals_out, int32_t* __restrict__ solves_out,
    int32_t* __restrict__ result_out, int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  StdSv<N, R, D> sv;
  sv.init(S, smem, tab);
  auto* sbs = reinterpret_cast<sbplx::State*>(
      reinterpret_cast<char*>(smem) + (time_std_bytes(N, S, D, kSoft) + 15) / 16 * 16);
  time_optimize_body<N, D, kSoft>(sv, S, tab, fixed_vals, times_io, p, max_evals, cost,
                                  evals_out, solves_out, result_out, status,
                                  smem + (sv.L.n + 1) / 2 * 2, sbs);
}

// The same on the compile-time-S solver (N = 10, r = 4, D = 3, S = 2..16).
template <int N, int R, int D, int S, bool kSoft>
__global__ __launch_bounds__(kWave) void time_optimize_wave_kernel(
    const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    double* __restrict__ times_io, mtg_time_params p, int max_evals,
    double* __restrict__ cost, int32_t* __restrict__ evals_out, int32_t* __restrict__ solves_out,
    int32_t* __restrict__ result_out, int32_t* __restrict__ status) {
  using G = wave::Geo<N, R, D, S>;
  constexpr int CB = kSoft ? S * D * N + kMaxSoftConstraints * (N + 2) : 0;
  constexpr int SB = static_cast<int>(sbplx::state_bytes(S) / sizeof(double));
  __shared__ __attribute__((aligned(16))) double sm[(G::L_N + CB + 1) / 2 * 2 + SB];
  wave::Solver<N, R, D, S> sv;
  sv.init(sm);
  time_optimize_body<N, D, kSoft>(sv, S, tab, fixed_vals, times_io, p, max_evals, cost,
                                  evals_out, solves_out, result_out, status, sm + G::L_N,
                                  reinterpret_cast<sbplx::State*>(sm + (G::L_N + CB + 1) / 2 * 2));
}

namespace {
template <typename K>
hipError_t prepare_lds_std(K kernel, size_t bytes) {
  if (bytes > 65536)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               static_cast<int>(bytes));
  return hipSuccess;
}

template <int N, int R, int D>
hipError_t time_cost_nrd(const PlanDev& pl, int64_t B, const double* df, const double* times,
                         const mtg_time_params& p, double* cost, double* grad, int32_t* status,
                         hipStream_t st) {
  const bool soft = p.n_soft > 0;
  const size_t bytes = time_std_lds_bytes(N, pl.S, D, soft);
  if (soft) {
    hipError_t e = prepare_lds_std(time_cost_std_kernel<N, R, D, true>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_cost_std_kernel<N, R, D, true>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl.S, pl.tab, df, times, p, cost, grad, status);
  } else {
    hipError_t e = prepare_lds_std(time_cost_std_kernel<N, R, D, false>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_cost_std_kernel<N, R, D, false>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl.S, pl.tab, df, times, p, cost, grad, status);
  }
  return hipGetLastError();
}

template <int N, int R, int D>
hipError_t time_opt_nrd(const PlanDev& pl, int64_t B, const double* df, double* times,
                        const mtg_time_params& p, int max_evals, double* cost, int32_t* evals,
                        int32_t* solves, int32_t* result, int32_t* status, hipStream_t st) {
  const bool soft = p.n_soft > 0;
  const size_t bytes = time_std_opt_lds_bytes(N, pl.S, D, soft);
  if (soft) {
    hipError_t e = prepare_lds_std(time_optimize_std_kernel<N, R, D, true>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_optimize_std_kernel<N, R, D, true>),
                       dim3(static_cast<unsigned>(B)), dim3(kWave), bytes, st, pl.S, pl.tab,
                       df, times, p, max_evals, cost, evals, solves, result, status);
  } else {
    hipError_t e = prepare_lds_std(time_optimize_std_kernel<N, R, D, false>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_optimize_std_kernel<N, R, D, false>),
                       dim3(static_cast<unsigned>(B)), dim3(kWave), bytes, st, pl.S, pl.tab,
                       df, times, p, max_evals, cost, evals, solves, result, status);
  }
  return hipGetLastError();
}
template <int S>
hipError_t time_cost_wave_s(const PlanDev& pl, int64_t B, const double* df, const double* times,
                            const mtg_time_params& p, double* cost, double* grad,
                            int32_t* status, hipStream_t st) {
  if (p.n_soft > 0)
    hipLaunchKernelGGL((time_cost_wave_kernel<10, 4, 3, S, true>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), 0, st, pl.tab, df, times, p, cost, grad, status);
  else
    hipLaunchKernelGGL((time_cost_wave_kernel<10, 4, 3, S, false>),
                       dim3(static_cast<unsigned>(B)), dim3(kWave), 0, st, pl.tab, df, times, p,
                       cost, grad, status);
  return hipGetLastError();
}

template <int S>
hipError_t time_opt_wave_s(const PlanDev& pl, int64_t B, const double* df, double* times,
                           const mtg_time_params& p, int max_evals, double* cost, int32_t* evals,
                           int32_t* solves, int32_t* result, int32_t* status, hipStream_t st) {
  if (p.n_soft > 0)
    hipLaunchKernelGGL((time_optimize_wave_kernel<10, 4, 3, S, true>),
                       dim3(static_cast<unsigned>(B)), dim3(kWave), 0, st, pl.tab, df, times, p,
                       max_evals, cost, evals, solves, result, status);
  else
    hipLaunchKernelGGL((time_optimize_wave_kernel<10, 4, 3, S, false>),
                       dim3(static_cast<unsigned>(B)), dim3(kWave), 0, st, pl.tab, df, times, p,
                       max_evals, cost, evals, solves, result, status);
  return hipGetLastError();
}

// The compile-time-S kernels where the C2 kernel exists (MTG_STD_RUNTIME_S=1
// forces the runtime-S ones, for A/B runs; launch_linear_solve_std reads the
// same switch).
bool use_time_wave(const PlanDev& pl) {
  static const bool forced = [] {
    const char* e = std::getenv("MTG_STD_RUNTIME_S");
    return e && e[0] == '1';
  }();
  return has_linear_wave(pl) && !forced;
}

#define MTG_TIME_WAVE_DISPATCH(FN, ...)                                                      \
  switch (pl.S) {                                                                            \
    case 2: return FN<2>(__VA_ARGS__);   case 3: return FN<3>(__VA_ARGS__);                   \
    case 4: return FN<4>(__VA_ARGS__);   case 5: return FN<5>(__VA_ARGS__);                   \
    case 6: return FN<6>(__VA_ARGS__);   case 7: return FN<7>(__VA_ARGS__);                   \
    case 8: return FN<8>(__VA_ARGS__);   case 9: return FN<9>(__VA_ARGS__);                   \
    case 10: return FN<10>(__VA_ARGS__); case 11: return FN<11>(__VA_ARGS__);                 \
    case 12: return FN<12>(__VA_ARGS__); case 13: return FN<13>(__VA_ARGS__);                 \
    case 14: return FN<14>(__VA_ARGS__); case 15: return FN<15>(__VA_ARGS__);                 \
    case 16: return FN<16>(__VA_ARGS__);                                                     \
    default: return hipErrorInvalidValue;                                                    \
  }
}  // namespace

bool has_time_std(const PlanDev& pl) {
  return use_std_kernel(pl) && pl.N == 10 && pl.r >= 2 && pl.r <= 4 && pl.D >= 1 && pl.D <= 3;
}

#define MTG_TIME_STD_DISPATCH(FN, ...)                          \
  switch (pl.r * 4 + pl.D) {                                    \
    case 2 * 4 + 1: return FN<10, 2, 1>(__VA_ARGS__);           \
    case 2 * 4 + 2: return FN<10, 2, 2>(__VA_ARGS__);           \
    case 2 * 4 + 3: return FN<10, 2, 3>(__VA_ARGS__);           \
    case 3 * 4 + 1: return FN<10, 3, 1>(__VA_ARGS__);           \
    case 3 * 4 + 2: return FN<10, 3, 2>(__VA_ARGS__);           \
    case 3 * 4 + 3: return FN<10, 3, 3>(__VA_ARGS__);           \
    case 4 * 4 + 1: return FN<10, 4, 1>(__VA_ARGS__);           \
    case 4 * 4 + 2: return FN<10, 4, 2>(__VA_ARGS__);           \
    case 4 * 4 + 3: return FN<10, 4, 3>(__VA_ARGS__);           \
    default: return hipErrorInvalidValue;                       \
  }

hipError_t launch_time_cost_std(const PlanDev& pl, int64_t B, const double* df,
                                const double* times, const mtg_time_params& p, double* cost,
                                double* grad, int32_t* status, hipStream_t st) {
  if (!has_time_std(pl)) return hipErrorInvalidValue;
  if (use_time_wave(pl))
    MTG_TIME_WAVE_DISPATCH(time_cost_wave_s, pl, B, df, times, p, cost, grad, status, st)
  MTG_TIME_STD_DISPATCH(time_cost_nrd, pl, B, df, times, p, cost, grad, status, st)
}

hipError_t launch_time_optimize_std(const PlanDev& pl, int64_t B, const double* df,
                                    double* times, const mtg_time_params& p, int max_evals,
                                    double* cost, int32_t* evals, int32_t* solves,
                                    int32_t* result, int32_t* status, hipStream_t st) {
  if (!has_time_std(pl)) return hipErrorInvalidValue;
  if (use_time_wave(pl))
    MTG_TIME_WAVE_DISPATCH(time_opt_wave_s, pl, B, df, times, p, max_evals, cost, evals, solves,
                           result, status, st)
  MTG_TIME_STD_DISPATCH(time_opt_nrd, pl, B, df, times, p, max_evals, cost, evals, solves, result,
                        status, st)
}

}  // namespace mtg

#ifdef MTG_STAMPS
// This translation unit's stamps (the soft searches' per-lane counters).
extern "C" int mtg_debug_stamps_time(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mtg_stamps),
                             sizeof(unsigned long long) * n) == hipSuccess ? 0 : -3;
}
#endif
