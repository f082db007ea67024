// mtg_free.hip — free-derivative objectives of PolynomialOptimizationNonLinear
//  for any constraint pattern, on the generic
// per-trajectory state of mtg_device.h (one 64-lane workgroup per trajectory):
//   mode 0  objectiveFunctionFreeConstraints (nonlinear_impl:1021-1113):
//           setFreeConstraints(d_p); J = J_d [+ soft], J_d = sum_dim d^T R d
//           (getCostAndGradientDerivative, :1537-1606), gradient
//           dJ_d/dd_p = 2 (R_pf d_f + R_pp d_p) per dimension (:1591-1592);
//           the soft term is not differentiated (:1100-1110);
//   mode 1  objectiveFunctionTimeAndConstraints (:947-1019):
//           updateSegmentTimes(T); setFreeConstraints(d_p);
//           J = computeCost() + time_penalty (sum T)^2 [+ soft].
// R d is formed segment by segment: (R d) at vertex v gathers the rows of
// H_s e_s (e_s = [d(vertex s); d(vertex s+1)]) of the two segments meeting
// there, so no R is assembled.  J_d = sum_s e_s^T H_s e_s = 2 computeCost().
//
// free_optimize_kernel: the device optimiser of mtg_free_optimize on the
// mode-0 objective (oracle restatement: orc_free_optimize).
// time_free_optimize_kernel: the device optimiser of mtg_time_free_optimize
// over [T; d_p] on the mode-1 objective (optimizeTimeAndFreeConstraints,
// nonlinear_impl:610-706; oracle restatement: orc_time_free_optimize).
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_device.h"
#include "mtg_extrema_device.h"
#include "mtg_free_device.h"
#include "mtg_internal.h"
#include "mtg_sbplx_device.h"

namespace mtg {

namespace {

// J of `mode` at the current dv (all lanes; wave-uniform result).
template <int N, bool kSoft>
__device__ double free_objective(Traj<N>& t, const double* __restrict__ tab,
                                 const mtg_time_params& p, int mode, double* cbuf) {
  double c;
  if constexpr (kSoft) {
    c = t.template coeffs_and_cost<true>(tab, cbuf);  // coefficients into LDS
  } else {
    c = t.cost(tab);
  }
  double J;
  if (mode == 0) {
    J = 2.0 * c;  // J_d = d^T R d = c^T Q c = 2 computeCost()
  } else {
    double tot = 0.0;
    for (int i = 0; i < t.S; ++i) tot += t.T()[i];  // nonlinear_impl:2768-2774
    J = c + tot * tot * p.time_penalty;
  }
  if constexpr (kSoft) {
    // evaluateMaximumMagnitudeAsSoftConstraint (nonlinear_impl:2735-2766).
    __syncthreads();
    double soft = 0.0;
    for (int k = 0; k < p.n_soft; ++k) {
      int K = 0;
      double lim = 1.0;
#pragma unroll
      for (int cc = 0; cc < kMaxSoftConstraints; ++cc)  // compile-time indices
        if (cc == k) {
          K = p.soft_derivative[cc];
          lim = p.soft_limit[cc];
        }
      const double m = ext_trajectory_max_wave_k<N>(K, cbuf, t.T(), t.S, t.D, t.lane);
      soft += fmin(p.soft_maximum_cost, exp((m - lim) / lim * p.soft_weight));
    }
    J += soft;
  }
  __syncthreads();
  return J;
}

}  // namespace

template <int N, bool kSoft>
__global__ __launch_bounds__(kWave) void free_cost_kernel(
    PlanDev pl, const double* __restrict__ fixed_vals, const double* __restrict__ free_vals,
    const double* __restrict__ times, mtg_time_params p, int mode, double* __restrict__ cost,
    double* __restrict__ grad, int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int S = pl.S, D = pl.D, nf = pl.nf, np = pl.np;
  const Layout lay = make_layout(N, S, D);
  const FreeLds fl = free_lds(N, S, D, np, kSoft);
  Traj<N> t{S, D, pl.r, &lay, smem, reinterpret_cast<int*>(smem + lay.ndouble),
            static_cast<int>(threadIdx.x), pl.fmask, pl.use_mask != 0};
  const int64_t b = blockIdx.x;
  const bool bad = free_setup(t, pl, fixed_vals + b * D * nf, free_vals + b * D * np,
                              times + b * S);
  double J = NAN;
  if (!bad) J = free_objective<N, kSoft>(t, pl.tab, p, mode, lds_at<double>(smem, fl.cbuf));
  if (grad && mode == 0) {
    if (bad) {
      for (int i = t.lane; i < D * np; i += kWave) grad[b * D * np + i] = NAN;
    } else {
      double* gv = lds_at<double>(smem, fl.gv);
      free_rd(t, gv);
      for (int i = t.lane; i < D * np; i += kWave)
        grad[b * D * np + i] = 2.0 * gv[pl.free_map[i % np] * D + i / np];
    }
  }
  if (t.lane == 0) {
    if (cost) cost[b] = J;
    if (status) status[b] = bad ? MTG_TRAJ_BAD_TIME : MTG_TRAJ_OK;
  }
}

// Device optimiser on the mode-0 objective J_d + [soft] (the objective of
// optimizeFreeConstraints, nonlinear_impl:399-493, whose NLopt run is
// replaced): d* = argmin J_d by the linear solve (the Newton step of the
// quadratic J_d), then d <- clamp(d + alpha (d* - d), lower, upper) with
// alpha = 1, x1.5 (capped at 1) on a decrease, x0.5 otherwise, `max_evals`
// objective evaluations; stops when a trial moves no entry by more than
// 1e-13 (1 + |d_i|).  One objective call site (state machine).
template <int N, bool kSoft>
__global__ __launch_bounds__(kWave) void free_optimize_kernel(
    PlanDev pl, const double* __restrict__ fixed_vals, double* __restrict__ free_io,
    const double* __restrict__ times, const double* __restrict__ lower,
    const double* __restrict__ upper, mtg_time_params p, int max_evals,
    double* __restrict__ cost, int32_t* __restrict__ evals_out, int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int S = pl.S, D = pl.D, nf = pl.nf, np = pl.np, n = D * np;
  const Layout lay = make_layout(N, S, D);
  const FreeLds fl = free_lds(N, S, D, np, kSoft);
  Traj<N> t{S, D, pl.r, &lay, smem, reinterpret_cast<int*>(smem + lay.ndouble),
            static_cast<int>(threadIdx.x), pl.fmask, pl.use_mask != 0};
  const int64_t b = blockIdx.x;
  double* cbuf = lds_at<double>(smem, fl.cbuf);
  double* dstar = lds_at<double>(smem, fl.opt);  // [d][p]
  double* dcur = dstar + n;
  double* dtry = dcur + n;
  const double* lo = lower ? lower + b * n : nullptr;
  const double* hi = upper ? upper + b * n : nullptr;
  const bool bad = free_setup(t, pl, fixed_vals + b * D * nf, nullptr, times + b * S);
  int evals = 0;
  double f = NAN;
  bool not_spd = false;
  if (!bad) {
    // d* = the unconstrained minimiser (solveLinear, linear_impl:337-379).
    t.solve();
    not_spd = (t.flag()[0] & 2) != 0;
    for (int i = t.lane; i < n; i += kWave) {
      const int slot = pl.free_map[i % np] * D + i / np;
      dstar[i] = t.dv()[slot];
      const double d0 = free_io[b * n + i];
      dcur[i] = d0;
      t.dv()[slot] = d0;
    }
    __syncthreads();
    double alpha = 1.0;
    bool base = true;
    for (;;) {
      const double J = free_objective<N, kSoft>(t, pl.tab, p, 0, cbuf);
      if (base) {
        f = J;
        evals = 1;
        base = false;
      } else {
        ++evals;
        if (J < f) {
          f = J;
          for (int i = t.lane; i < n; i += kWave) dcur[i] = dtry[i];
          alpha = fmin(alpha * 1.5, 1.0);
        } else {
          alpha *= 0.5;
        }
      }
      __syncthreads();
      if (!(evals < max_evals && alpha > 1e-9)) break;
      // Next trial, unfused like the oracle: x = d + alpha (d* - d), clamped.
      bool moved = false;
      for (int i = t.lane; i < n; i += kWave) {
        const double d = dcur[i];
        double x = __dadd_rn(d, __dmul_rn(alpha, __dsub_rn(dstar[i], d)));
        if (lo) x = fmax(x, lo[i]);
        if (hi) x = fmin(x, hi[i]);
        dtry[i] = x;
        moved = moved || fabs(x - d) > 1e-13 * (1.0 + fabs(d));
        t.dv()[pl.free_map[i % np] * D + i / np] = x;
      }
      if (!__any(moved)) break;
      __syncthreads();
    }
    __syncthreads();
    for (int i = t.lane; i < n; i += kWave) free_io[b * n + i] = dcur[i];
  }
  if (t.lane == 0) {
    if (cost) cost[b] = f;
    if (evals_out) evals_out[b] = evals;
    if (status)
      status[b] = bad ? MTG_TRAJ_BAD_TIME : (not_spd ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK);
  }
}

// Device optimiser of the kOptimizeFreeConstraintsAndTime objective (mode 1,
// objectiveFunctionTimeAndConstraints, nonlinear_impl:947-1019) over
// x = [T; d_p] with the reference's bounds (optimizeTimeAndFreeConstraints,
// nonlinear_impl:610-706): T in [0.1, 2 |T0|], d_p in [-2 |d0|, 2 |d0|].
// NLopt's SBPLX is replaced by block-alternating projected steps, each trial
// one counted evaluation (NLopt maxeval, :101):
//   T block: scaled steepest descent, T' = clamp(T - aT T0 (g T0) / max|g T0|),
//     g = central differences of J in T with d_p held (step `increment`,
//     clamp rule of :2529-2530; not counted, as the time optimiser's);
//   d block: Newton step of the quadratic J in d_p toward d* = argmin_d J at
//     the current T (the linear solve), d' = clamp(d + ad (d* - d));
//   a step size grows x1.5 (capped at 1) on a decrease of J and halves
//   otherwise (aT starts at initial_stepsize_rel = 0.1, ad at 1).
// The round repeats (gradient only after an accepted step) until max_evals
// evaluations, both step sizes below 1e-9, or a round in which neither trial
// moves.  A state machine with one objective call site.
template <int N, bool kSoft>
__global__ __launch_bounds__(kWave) void time_free_optimize_kernel(
    PlanDev pl, const double* __restrict__ fixed_vals, double* __restrict__ free_io,
    double* __restrict__ times_io, mtg_time_params p, int max_evals, double* __restrict__ cost,
    int32_t* __restrict__ evals_out, int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int S = pl.S, D = pl.D, nf = pl.nf, np = pl.np, n = D * np;
  const Layout lay = make_layout(N, S, D);
  const FreeLds fl = free_lds(N, S, D, np, kSoft);
  Traj<N> t{S, D, pl.r, &lay, smem, reinterpret_cast<int*>(smem + lay.ndouble),
            static_cast<int>(threadIdx.x), pl.fmask, pl.use_mask != 0};
  const int64_t b = blockIdx.x;
  double* cbuf = lds_at<double>(smem, fl.cbuf);
  double* dstar = lds_at<double>(smem, fl.opt);  // [d][p]
  double* dcur = dstar + (n > 0 ? n : 1);
  double* dtry = dcur + (n > 0 ? n : 1);
  double* Tcur = dtry + (n > 0 ? n : 1);
  double* T0 = Tcur + S;
  double* Ttry = T0 + S;
  double* g = Ttry + S;
  const bool bad = free_setup(t, pl, fixed_vals + b * D * nf, nullptr, times_io + b * S);
  int evals = 0;
  double f = NAN;
  bool not_spd = false;
  auto slot_of = [&](int i) { return pl.free_map[i % np] * D + i / np; };
  if (!bad) {
    for (int i = t.lane; i < S; i += kWave) Tcur[i] = T0[i] = t.T()[i];
    for (int i = t.lane; i < n; i += kWave) {
      const double d0 = free_io[b * n + i];
      dcur[i] = d0;
      t.dv()[slot_of(i)] = d0;
    }
    __syncthreads();
    constexpr double kLower = 0.1;  // nonlinear_impl:675-677
    enum { kBase, kGrad, kTTrial, kDTrial };               // evaluation kinds
    enum { kEval, kDone, kRound, kTStep, kDStep, kEnd };  // transitions
    int phase = kBase, gi = 0;
    double aT = 0.1, ad = 1.0, Jlo = 0.0;
    bool stale = true, dstar_ok = false, moved_round = false;
    // Evaluation point: times src (powers recomputed), free values dsrc.
    auto set_point = [&](const double* src, const double* dsrc) {
      for (int i = t.lane; i < S; i += kWave) t.T()[i] = src[i];
      for (int i = t.lane; i < n; i += kWave) t.dv()[slot_of(i)] = dsrc[i];
      __syncthreads();
      t.compute_powers();
      __syncthreads();
    };
    for (;;) {
      const double J = free_objective<N, kSoft>(t, pl.tab, p, 1, cbuf);
      int go;
      if (phase == kBase) {
        f = J;
        evals = 1;
        go = kRound;
      } else if (phase == kGrad) {
        if (gi & 1) {
          if (t.lane == 0) g[gi >> 1] = (J - Jlo) / (2.0 * p.increment);
        } else {
          Jlo = J;
        }
        ++gi;
        go = gi < 2 * S ? kEval : kTStep;
      } else if (phase == kTTrial) {
        ++evals;
        if (J < f) {
          f = J;
          for (int i = t.lane; i < S; i += kWave) Tcur[i] = Ttry[i];
          aT = fmin(aT * 1.5, 1.0);
          stale = true;
          dstar_ok = false;
        } else {
          aT *= 0.5;
        }
        go = kDStep;
      } else {  // kDTrial
        ++evals;
        if (J < f) {
          f = J;
          for (int i = t.lane; i < n; i += kWave) dcur[i] = dtry[i];
          ad = fmin(ad * 1.5, 1.0);
          stale = true;
        } else {
          ad *= 0.5;
        }
        go = kEnd;
      }
      __syncthreads();
      while (go != kEval && go != kDone) {
        if (go == kRound) {
          moved_round = false;
          if (stale) {
            stale = false;
            phase = kGrad;
            gi = 0;
            go = kEval;
          } else {
            go = kTStep;
          }
        } else if (go == kTStep) {
          go = kDStep;
          if (!(evals < max_evals)) {
            go = kDone;
          } else if (aT > 1e-9) {
            double gmax = 0.0;
            for (int i = 0; i < S; ++i) gmax = fmax(gmax, fabs(g[i] * T0[i]));
            bool moved = false;
            if (gmax > 0.0) {
              for (int i = 0; i < S; ++i) {
                double tn = Tcur[i] - aT * T0[i] * (g[i] * T0[i]) / gmax;
                tn = fmin(fmax(tn, kLower), 2.0 * fabs(T0[i]));
                moved = moved || tn != Tcur[i];
                if (t.lane == 0) Ttry[i] = tn;
              }
            }
            __syncthreads();
            if (moved) {
              moved_round = true;
              phase = kTTrial;
              go = kEval;
            }
          }
        } else if (go == kDStep) {
          go = kEnd;
          if (!(evals < max_evals)) {
            go = kDone;
          } else if (ad > 1e-9) {
            if (!dstar_ok) {
              // d* = argmin_d J at Tcur (solveLinear, linear_impl:337-379).
              set_point(Tcur, dcur);
              t.clear_free();  // assemble() sums over dv with free entries zero
              __syncthreads();
              t.solve();
              not_spd = not_spd || (t.flag()[0] & 2) != 0;
              for (int i = t.lane; i < n; i += kWave) dstar[i] = t.dv()[slot_of(i)];
              __syncthreads();
              dstar_ok = true;
            }
            bool moved = false;
            for (int i = t.lane; i < n; i += kWave) {
              const double d = dcur[i];
              const double bnd = 2.0 * fabs(free_io[b * n + i]);  // nonlinear_impl:665-668
              double x = __dadd_rn(d, __dmul_rn(ad, __dsub_rn(dstar[i], d)));
              x = fmin(fmax(x, -bnd), bnd);
              dtry[i] = x;
              moved = moved || fabs(x - d) > 1e-13 * (1.0 + fabs(d));
            }
            __syncthreads();
            if (__any(moved)) {
              moved_round = true;
              phase = kDTrial;
              go = kEval;
            }
          }
        } else {  // kEnd
          go = (evals < max_evals && moved_round) ? kRound : kDone;
        }
      }
      if (go == kDone) break;
      // Load the evaluation point of `phase`.
      if (phase == kGrad) {
        const int nn = gi >> 1;
        for (int i = t.lane; i < S; i += kWave) {
          const double Tn = Tcur[i];
          Ttry[i] = i != nn ? Tn
                            : (Tn <= 0.1 ? 0.1 : ((gi & 1) ? Tn + p.increment : Tn - p.increment));
        }
        __syncthreads();
        set_point(Ttry, dcur);
      } else if (phase == kTTrial) {
        set_point(Ttry, dcur);
      } else {
        set_point(Tcur, dtry);
      }
    }
    __syncthreads();
    for (int i = t.lane; i < S; i += kWave) times_io[b * S + i] = Tcur[i];
    for (int i = t.lane; i < n; i += kWave) free_io[b * n + i] = dcur[i];
  }
  if (t.lane == 0) {
    if (cost) cost[b] = f;
    if (evals_out) evals_out[b] = evals;
    if (status)
      status[b] = bad ? MTG_TRAJ_BAD_TIME : (not_spd ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK);
  }
}

// LDS of the LN_SBPLX form: the free layout, then the evaluation point X
// (S + D np values) and the machine state.
struct FreeSbplxLds {
  size_t x, state, bytes;
};
__host__ __device__ inline FreeSbplxLds free_sbplx_lds(int N, int S, int D, int np, bool soft) {
  FreeSbplxLds f;
  const int n = S + D * np;
  f.x = (free_lds(N, S, D, np, soft).bytes + 15) / 16 * 16;
  f.state = (f.x + sizeof(double) * n + 15) / 16 * 16;
  f.bytes = f.state + sbplx::state_bytes(n);
  return f;
}

// kOptimizeFreeConstraintsAndTime with the reference's own algorithm:
// NLopt's LN_SBPLX (the default, polynomial_optimization_nonlinear.h:61;
// optimizeTimeAndFreeConstraints, nonlinear_impl:610-706) over
// x = [T; d_p] (d_p dimension-major, :653-662) on
// objectiveFunctionTimeAndConstraints (:947-1019: updateSegmentTimes(T),
// setFreeConstraints(d_p), computeCost() + time_penalty (sum T)^2 [+ soft];
// no re-solve).  Bounds T in [0.1, 2 |T0|], d_p in [-2 |d0|, 2 |d0|], initial
// steps initial_stepsize_rel |x0| (:664-675), maxeval, ftol (:95-101).  The
// machine (mtg_sbplx_device.h) runs on lane 0 with its state in LDS sized by
// n = S + D np; the wave evaluates.  x0 with a zero entry (a zero initial
// step) or a time below 0.1 is NLopt's invalid argument: result -1
// (nlopt::FAILURE, :681-691, 696-703), no evaluation, x unchanged.
template <int N, bool kSoft>
__global__ __launch_bounds__(kWave) void time_free_sbplx_kernel(
    PlanDev pl, const double* __restrict__ fixed_vals, double* __restrict__ free_io,
    double* __restrict__ times_io, mtg_time_params p, int max_evals, double* __restrict__ cost,
    int32_t* __restrict__ evals_out, int32_t* __restrict__ result_out,
    int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int S = pl.S, D = pl.D, nf = pl.nf, np = pl.np, n = D * np, nx = S + n;
  const Layout lay = make_layout(N, S, D);
  const FreeLds fl = free_lds(N, S, D, np, kSoft);
  const FreeSbplxLds fs = free_sbplx_lds(N, S, D, np, kSoft);
  Traj<N> t{S, D, pl.r, &lay, smem, reinterpret_cast<int*>(smem + lay.ndouble),
            static_cast<int>(threadIdx.x), pl.fmask, pl.use_mask != 0};
  const int64_t b = blockIdx.x;
  double* cbuf = lds_at<double>(smem, fl.cbuf);
  double* X = lds_at<double>(smem, fs.x);
  auto* sbs = lds_at<sbplx::State>(smem, fs.state);
  sbplx::Machine mach{sbs};
  const bool bad = free_setup(t, pl, fixed_vals + b * D * nf, nullptr, times_io + b * S);
  auto slot_of = [&](int i) { return pl.free_map[i % np] * D + i / np; };
  double f = NAN;
  int evals = 0, res = sbplx::kFailure;
  if (!bad) {
    const double step_rel = p.initial_stepsize_rel > 0.0 ? p.initial_stepsize_rel : 0.1;
    if (t.lane == 0) sbs->n = nx;
    for (int i = t.lane; i < nx; i += kWave) X[i] = i < S ? t.T()[i] : free_io[b * n + i - S];
    __syncthreads();
    for (int i = t.lane; i < nx; i += kWave) {  // the bounds of :665-677, filled in parallel
      const double v = X[i], a = fabs(v);
      mach.x()[i] = v;
      mach.lb()[i] = i < S ? 0.1 : -2.0 * a;
      mach.ub()[i] = 2.0 * a;
      mach.xstep()[i] = step_rel * a;
    }
    __syncthreads();
    if (t.lane == 0) mach.start(max_evals, p.f_rel, p.f_abs);
    __syncthreads();
    while (!sbs->done) {
      // the point X: times (powers recomputed) and d_p into the vertex table
      for (int i = t.lane; i < S; i += kWave) t.T()[i] = X[i];
      for (int i = t.lane; i < n; i += kWave) t.dv()[slot_of(i)] = X[S + i];
      __syncthreads();
      t.compute_powers();
      __syncthreads();
      const double J = free_objective<N, kSoft>(t, pl.tab, p, 1, cbuf);
      if (t.lane == 0) mach.resume(J, X);
      __syncthreads();
    }
    const double* xb = sbplx::best_x(sbs);
    for (int i = t.lane; i < S; i += kWave) times_io[b * S + i] = xb[i];
    for (int i = t.lane; i < n; i += kWave) free_io[b * n + i] = xb[S + i];
    f = sbs->minf;
    evals = sbs->nevals;
    res = sbs->result;
  }
  if (t.lane == 0) {
    if (cost) cost[b] = f;
    if (evals_out) evals_out[b] = evals;
    if (result_out) result_out[b] = res;
    if (status) status[b] = bad ? MTG_TRAJ_BAD_TIME : MTG_TRAJ_OK;
  }
}

namespace {
template <typename K>
hipError_t prepare_lds_free(K kernel, size_t bytes) {
  if (bytes > 65536)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               static_cast<int>(bytes));
  return hipSuccess;
}

template <int N>
hipError_t free_cost_n(const PlanDev& pl, int64_t B, const double* df, const double* dp,
                       const double* times, const mtg_time_params& p, int mode, double* cost,
                       double* grad, int32_t* status, hipStream_t st) {
  const bool soft = p.n_soft > 0;
  const size_t bytes = free_lds(N, pl.S, pl.D, pl.np, soft).bytes;
  if (soft) {
    hipError_t e = prepare_lds_free(free_cost_kernel<N, true>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((free_cost_kernel<N, true>), dim3(static_cast<unsigned>(B)), dim3(kWave),
                       bytes, st, pl, df, dp, times, p, mode, cost, grad, status);
  } else {
    hipError_t e = prepare_lds_free(free_cost_kernel<N, false>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((free_cost_kernel<N, false>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, dp, times, p, mode, cost, grad, status);
  }
  return hipGetLastError();
}

template <int N>
hipError_t free_opt_n(const PlanDev& pl, int64_t B, const double* df, double* dp,
                      const double* times, const double* lower, const double* upper,
                      const mtg_time_params& p, int max_evals, double* cost, int32_t* evals,
                      int32_t* status, hipStream_t st) {
  const bool soft = p.n_soft > 0;
  const size_t bytes = free_lds(N, pl.S, pl.D, pl.np, soft).bytes;
  if (soft) {
    hipError_t e = prepare_lds_free(free_optimize_kernel<N, true>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((free_optimize_kernel<N, true>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, dp, times, lower, upper, p, max_evals,
                       cost, evals, status);
  } else {
    hipError_t e = prepare_lds_free(free_optimize_kernel<N, false>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((free_optimize_kernel<N, false>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, dp, times, lower, upper, p, max_evals,
                       cost, evals, status);
  }
  return hipGetLastError();
}
}  // namespace

template <int N>
hipError_t time_free_opt_n(const PlanDev& pl, int64_t B, const double* df, double* dp,
                           double* times, const mtg_time_params& p, int max_evals, double* cost,
                           int32_t* evals, int32_t* status, hipStream_t st) {
  const bool soft = p.n_soft > 0;
  const size_t bytes = free_lds(N, pl.S, pl.D, pl.np, soft).bytes;
  if (soft) {
    hipError_t e = prepare_lds_free(time_free_optimize_kernel<N, true>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_free_optimize_kernel<N, true>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, dp, times, p, max_evals, cost, evals,
                       status);
  } else {
    hipError_t e = prepare_lds_free(time_free_optimize_kernel<N, false>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_free_optimize_kernel<N, false>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, dp, times, p, max_evals, cost, evals,
                       status);
  }
  return hipGetLastError();
}

size_t free_lds_bytes(int N, int S, int D, int np, bool soft) {
  return free_lds(N, S, D, np, soft).bytes;
}
size_t free_sbplx_lds_bytes(int N, int S, int D, int np, bool soft) {
  return free_sbplx_lds(N, S, D, np, soft).bytes;
}

template <int N>
hipError_t time_free_sbplx_n(const PlanDev& pl, int64_t B, const double* df, double* dp,
                             double* times, const mtg_time_params& p, int max_evals,
                             double* cost, int32_t* evals, int32_t* result, int32_t* status,
                             hipStream_t st) {
  const bool soft = p.n_soft > 0;
  const size_t bytes = free_sbplx_lds(N, pl.S, pl.D, pl.np, soft).bytes;
  if (soft) {
    hipError_t e = prepare_lds_free(time_free_sbplx_kernel<N, true>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_free_sbplx_kernel<N, true>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, dp, times, p, max_evals, cost, evals,
                       result, status);
  } else {
    hipError_t e = prepare_lds_free(time_free_sbplx_kernel<N, false>, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((time_free_sbplx_kernel<N, false>), dim3(static_cast<unsigned>(B)),
                       dim3(kWave), bytes, st, pl, df, dp, times, p, max_evals, cost, evals,
                       result, status);
  }
  return hipGetLastError();
}

#define MTG_FREE_DISPATCH(FN, ...)        \
  switch (pl.N) {                         \
    case 4: return FN<4>(__VA_ARGS__);    \
    case 6: return FN<6>(__VA_ARGS__);    \
    case 8: return FN<8>(__VA_ARGS__);    \
    case 10: return FN<10>(__VA_ARGS__);  \
    case 12: return FN<12>(__VA_ARGS__);  \
    default: return hipErrorInvalidValue; \
  }

hipError_t launch_free_cost(const PlanDev& pl, int64_t B, const double* df, const double* dp,
                            const double* times, const mtg_time_params& p, int mode,
                            double* cost, double* grad, int32_t* status, hipStream_t st) {
  MTG_FREE_DISPATCH(free_cost_n, pl, B, df, dp, times, p, mode, cost, grad, status, st)
}

hipError_t launch_time_free_optimize(const PlanDev& pl, int64_t B, const double* df, double* dp,
                                     double* times, const mtg_time_params& p, int max_evals,
                                     double* cost, int32_t* evals, int32_t* result,
                                     int32_t* status, hipStream_t st) {
  if (p.optimizer == 1) {
    MTG_FREE_DISPATCH(time_free_sbplx_n, pl, B, df, dp, times, p, max_evals, cost, evals, result,
                      status, st)
  }
  MTG_FREE_DISPATCH(time_free_opt_n, pl, B, df, dp, times, p, max_evals, cost, evals, status, st)
}

hipError_t launch_free_optimize(const PlanDev& pl, int64_t B, const double* df, double* dp,
                                const double* times, const double* lower, const double* upper,
                                const mtg_time_params& p, int max_evals, double* cost,
                                int32_t* evals, int32_t* status, hipStream_t st) {
  MTG_FREE_DISPATCH(free_opt_n, pl, B, df, dp, times, lower, upper, p, max_evals, cost, evals,
                    status, st)
}

}  // namespace mtg
