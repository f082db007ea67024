// mtg_tube_time.hip — the segment-time objective of the fork's nonlinear
// class with the tube QCQP as its inner solve (objectiveFunctionTime,
// nonlinear_impl:877-945: updateSegmentTimes(T), solveQCQP() at :892,
// computeCost() + time_penalty (sum T)^2 [+ soft]), and a batched optimiser
// over it (optimizeTime, nonlinear_impl:332-397).
//
// A QCQP solve is one workgroup of tube_solve_kernel (mtg_tube.hip).  Every
// objective evaluation a trajectory needs in a round is a problem of one
// tube launch: the point T (row 0) and, for the gradient, the 2S
// central-difference points (rows 2n+1, 2n+2), all sharing the trajectory's
// geometry (TubeArgs::rep).  Small kernels around the launch build the
// points, form J from the QCQP cost, and (optimiser) advance a per-trajectory
// state machine.  The optimiser evaluates the gradient points of every trial
// together with the trial itself, so one round = one counted evaluation; the
// call enqueues max_evals rounds and a finished trajectory is skipped by
// every later kernel (no host round trip).  All scratch is the caller's
// workspace (mtg_tube_time_workspace_bytes): the call never allocates or
// synchronises.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_internal.h"
#include "mtg_sbplx_device.h"

namespace mtg {

namespace {

constexpr double kLower = 0.1;  // kOptimizationTimeLowerBound (nonlinear_impl:370)

// Row j of the evaluation points of trajectory b from its times T:
// j = 0: T; j = 2n+1 / 2n+2: T_n lowered / raised by h, both set to 0.1 when
// T_n <= 0.1 (getCostAndGradientTime's clamp, nonlinear_impl:2525-2530).
__global__ void tube_time_points_kernel(int S, int64_t B, int P, const double* __restrict__ T,
                                        double h, double* __restrict__ pts) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= B * P * S) return;
  const int64_t b = idx / (static_cast<int64_t>(P) * S);
  const int j = static_cast<int>((idx / S) % P), i = static_cast<int>(idx % S);
  double t = T[b * S + i];
  if (j > 0 && i == (j - 1) / 2) t = t <= kLower ? kLower : ((j & 1) ? t - h : t + h);
  pts[idx] = t;
}

// J of every point: QCQP computeCost + time_penalty (sum T)^2 (+ soft);
// NaN where the QCQP broke down or a time is not positive.  With cost / grad
// (cost API): J of row 0 and the central differences.
__global__ void tube_time_finish_kernel(int S, int64_t B, int P, const double* __restrict__ pts,
                                        const double* __restrict__ qcost,
                                        const int32_t* __restrict__ qstatus,
                                        const double* __restrict__ soft, double time_penalty,
                                        double h, const int32_t* __restrict__ skip,
                                        double* __restrict__ Jall,
                                        double* __restrict__ cost, double* __restrict__ grad,
                                        int32_t* __restrict__ status) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B || (skip && skip[b])) return;
  double J0 = 0.0, Jprev = 0.0;
  for (int j = 0; j < P; ++j) {
    const int64_t q = b * P + j;
    double total = 0.0;
    for (int i = 0; i < S; ++i) total += pts[q * S + i];  // nonlinear_impl:2768-2774
    const int st = qstatus[q];
    double J = qcost[q] + total * total * time_penalty;
    if (soft) J += soft[q];
    if (st == MTG_TRAJ_BAD_TIME || st == MTG_TRAJ_NOT_SPD) J = NAN;
    if (Jall) Jall[q] = J;
    if (j == 0) {
      J0 = J;
    } else if (j & 1) {
      Jprev = J;
    } else if (grad) {
      grad[b * S + (j - 1) / 2] = (J - Jprev) / (2.0 * h);
    }
  }
  if (cost) cost[b] = J0;
  if (status) status[b] = qstatus[b * P];
}

struct OptState {
  double *T0, *Tc, *g, *Ttr, *f, *alpha;
  int32_t *evals, *done, *st;
  char* sb;         // LN_SBPLX: one machine state per trajectory (sb_bytes each)
  size_t sb_bytes;
  double* warm;     // LN_SBPLX: the IPM warm-start state per trajectory
  int32_t* warm_ok;
  int32_t* iters;   // LN_SBPLX: IPM iterations of each trajectory's last solve
  int32_t* order;   // LN_SBPLX: the next round's dispatch order (TubeArgs::order)
};

__global__ void tube_time_opt_init_kernel(int S, int64_t B, const double* __restrict__ times,
                                          OptState s) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx < B * S) {
    const double t = times[idx];
    s.T0[idx] = t;
    s.Tc[idx] = t;
    s.Ttr[idx] = t;
    s.g[idx] = 0.0;
  }
  if (idx < B) {
    s.f[idx] = 0.0;
    s.alpha[idx] = 0.1;  // initial_stepsize_rel (polynomial_optimization_nonlinear.h:55)
    s.evals[idx] = 0;
    s.done[idx] = 0;
    s.st[idx] = MTG_TRAJ_OK;
  }
}

// One round of the projected, scaled steepest descent of the linear-inner
// optimiser (time_optimize_kernel, mtg_kernels.hip; oracle timeOptimizeImpl):
// consume the trial's J and gradient, accept or backtrack, then place the
// next trial (or finish).
__global__ void tube_time_opt_step_kernel(int S, int64_t B, int P, int first, int max_evals,
                                          double h, const double* __restrict__ Jall,
                                          const int32_t* __restrict__ qstatus, OptState s) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B || s.done[b]) return;
  const double* J = Jall + b * P;
  double* Tc = s.Tc + b * S;
  double* T0 = s.T0 + b * S;
  double* g = s.g + b * S;
  double* Ttr = s.Ttr + b * S;
  double alpha = s.alpha[b];
  int evals = s.evals[b] + 1;
  bool accept = false;
  if (first) {
    s.f[b] = J[0];
    if (!std::isfinite(J[0])) {
      s.st[b] = qstatus[b * P] != MTG_TRAJ_OK ? qstatus[b * P] : MTG_TRAJ_NOT_SPD;
      s.evals[b] = evals;
      s.done[b] = 1;
      return;
    }
    accept = true;
  } else if (J[0] < s.f[b]) {
    s.f[b] = J[0];
    for (int i = 0; i < S; ++i) Tc[i] = Ttr[i];
    alpha = fmin(alpha * 1.5, 1.0);
    accept = true;
  } else {
    alpha *= 0.5;
  }
  if (accept)
    for (int n = 0; n < S; ++n) g[n] = (J[2 * n + 2] - J[2 * n + 1]) / (2.0 * h);
  s.alpha[b] = alpha;
  s.evals[b] = evals;
  bool stop = !(evals < max_evals && alpha > 1e-9);
  double gmax = 0.0;
  bool finite = true;
  for (int n = 0; n < S; ++n) {
    finite = finite && std::isfinite(g[n]);
    gmax = fmax(gmax, fabs(g[n] * T0[n]));
  }
  stop = stop || !finite || !(gmax > 0.0);
  if (!stop) {
    bool same = true;
    for (int n = 0; n < S; ++n) {
      const double x = Tc[n] - alpha * T0[n] * (g[n] * T0[n]) / gmax;
      const double t = fmin(fmax(x, kLower), 2.0 * T0[n]);
      Ttr[n] = t;
      same = same && t == Tc[n];
    }
    stop = same;
  }
  if (stop) s.done[b] = 1;
}

__global__ void tube_time_opt_final_kernel(int S, int64_t B, OptState s,
                                           double* __restrict__ times_io,
                                           double* __restrict__ cost,
                                           int32_t* __restrict__ evals,
                                           int32_t* __restrict__ status) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx < B * S) times_io[idx] = s.Tc[idx];
  if (idx < B) {
    if (cost) cost[idx] = s.f[idx];
    if (evals) evals[idx] = s.evals[idx];
    if (status) status[idx] = s.st[idx];
  }
}

// LN_SBPLX over the QCQP objective (optimizer 1), the reference's default
// optimizeTime (nonlinear_impl:332-397: NLopt's Subplex from T0, bounds
// [0.1, 2 T0], initial steps initial_stepsize_rel T0, maxeval, ftol) on
// objectiveFunctionTime with solveQCQP() at every evaluation (:891-892).  One
// evaluation per trajectory per round; the machine (mtg_sbplx_device.h) of
// trajectory b lives in the workspace and one thread advances it between
// rounds.  NLopt evaluates T0 first, so the initial solveQCQP (:342) is the
// first round's solve.
__device__ inline sbplx::State* sb_state(const OptState& s, int64_t b) {
  return reinterpret_cast<sbplx::State*>(s.sb + static_cast<size_t>(b) * s.sb_bytes);
}

__global__ void tube_time_sbplx_init_kernel(int S, int64_t B, const double* __restrict__ times,
                                            double step_rel, int max_evals, double ftol_rel,
                                            double ftol_abs, OptState s) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  for (int i = 0; i < S; ++i) {
    const double t = times[b * S + i];
    s.T0[b * S + i] = t;
    s.Ttr[b * S + i] = t;
  }
  sbplx::Machine m{sb_state(s, b)};
  m.init(S, s.Ttr + b * S, step_rel, max_evals, ftol_rel, ftol_abs);
  s.done[b] = m.s->done;  // a start outside the bounds: no evaluation
  s.st[b] = MTG_TRAJ_OK;
  s.warm_ok[b] = 0;  // the first evaluation (T0) starts cold
}

// Hand the round's J to the machine; it writes the next point into Ttr or
// finishes.  The QCQP status of the first evaluation (T0) is the one
// reported.
__global__ void tube_time_sbplx_step_kernel(int S, int64_t B, int first,
                                            const double* __restrict__ Jall,
                                            const int32_t* __restrict__ qstatus, OptState s) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B || s.done[b]) return;
  if (first) s.st[b] = qstatus[b];
  sbplx::Machine m{sb_state(s, b)};
  m.resume(Jall[b], s.Ttr + b * S);
  if (m.s->done) s.done[b] = 1;
}

// NLopt's x and opt_f (the best point and its value), the evaluations used
// and the nlopt_result code.
__global__ void tube_time_sbplx_final_kernel(int S, int64_t B, OptState s,
                                             double* __restrict__ times_io,
                                             double* __restrict__ cost,
                                             int32_t* __restrict__ evals,
                                             int32_t* __restrict__ result,
                                             int32_t* __restrict__ status) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const sbplx::State* st = sb_state(s, b);
  const double* x = sbplx::best_x(st);
  for (int i = 0; i < S; ++i) times_io[b * S + i] = x[i];
  if (cost) cost[b] = st->minf;
  if (evals) evals[b] = st->nevals;
  if (result) result[b] = st->result;
  if (status) status[b] = s.st[b];
}

__global__ void tube_time_opt_result_kernel(int64_t B, int max_evals, OptState s,
                                            int32_t* __restrict__ result) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b < B) result[b] = s.evals[b] >= max_evals ? sbplx::kMaxEval : sbplx::kXtol;
}

// The next round's dispatch order (TubeArgs::order): a counting sort of the
// trajectories by their last solve's IPM iterations, most first, the
// finished ones last.  A solve's iteration count is the best predictor of
// the next one's (consecutive points of a trajectory are close and share
// their constraints), so dispatching longest-first keeps a round's few long
// solves (up to the 100-iteration cap) from starting last and forming its
// tail.  Ties are placed in any order: results do not depend on the order.
constexpr int kOrderKeys = 128;
__global__ __launch_bounds__(1024) void tube_time_order_kernel(int64_t B,
                                                               const int32_t* __restrict__ iters,
                                                               const int32_t* __restrict__ done,
                                                               int32_t* __restrict__ order) {
  __shared__ int cnt[kOrderKeys], off[kOrderKeys];
  const int t = static_cast<int>(threadIdx.x);
  for (int k = t; k < kOrderKeys; k += blockDim.x) cnt[k] = 0;
  __syncthreads();
  auto key = [&](int64_t b) {
    const int it = iters[b];
    return done[b] ? 0 : 1 + (it < 0 ? 0 : (it > kOrderKeys - 2 ? kOrderKeys - 2 : it));
  };
  for (int64_t b = t; b < B; b += blockDim.x) atomicAdd(&cnt[key(b)], 1);
  __syncthreads();
  if (t == 0) {
    int run = 0;
    for (int k = kOrderKeys - 1; k >= 0; --k) {
      off[k] = run;
      run += cnt[k];
    }
  }
  __syncthreads();
  for (int64_t b = t; b < B; b += blockDim.x)
    order[atomicAdd(&off[key(b)], 1)] = static_cast<int32_t>(b);
}

unsigned blocks_for(int64_t n) { return static_cast<unsigned>((n + 255) / 256); }

// Caller-owned workspace (mtg_tube_time_workspace_bytes), carved in a fixed
// order; each array starts on a 256-byte boundary.  With base == nullptr only
// the size is computed.
struct Workspace {
  double *coeffs, *pts, *qcost, *softc, *Jall, *maxima;
  int32_t* qstatus;
  OptState s;  // optimiser only
};
struct Carver {
  char* base;
  size_t off = 0;
  template <typename T>
  T* take(int64_t n) {
    off = (off + 255) & ~size_t(255);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += sizeof(T) * static_cast<size_t>(n);
    return p;
  }
};
size_t carve(void* base, int N, int S, int64_t B, int P, int n_soft, bool optimiser,
             bool sbplx_opt, Workspace* w) {
  Carver c{static_cast<char*>(base)};
  const int64_t BP = B * P;
  w->coeffs = c.take<double>(BP * S * 3 * N);
  w->pts = c.take<double>(BP * S);
  w->qcost = c.take<double>(BP);
  w->softc = c.take<double>(BP);
  w->Jall = c.take<double>(BP);
  w->maxima = c.take<double>(BP * (n_soft > 0 ? n_soft : 1));
  w->qstatus = c.take<int32_t>(BP);
  w->s = OptState{};
  if (optimiser) {
    w->s.T0 = c.take<double>(B * S);
    w->s.Tc = c.take<double>(B * S);
    w->s.g = c.take<double>(B * S);
    w->s.Ttr = c.take<double>(B * S);
    w->s.f = c.take<double>(B);
    w->s.alpha = c.take<double>(B);
    w->s.evals = c.take<int32_t>(B);
    w->s.done = c.take<int32_t>(B);
    w->s.st = c.take<int32_t>(B);
    if (sbplx_opt) {
      w->s.sb_bytes = sbplx::state_bytes(S);
      w->s.sb = c.take<char>(B * static_cast<int64_t>(w->s.sb_bytes));
      w->s.warm = c.take<double>(B * tube_warm_doubles(N, S));
      w->s.warm_ok = c.take<int32_t>(B);
      w->s.iters = c.take<int32_t>(B);
      w->s.order = c.take<int32_t>(B);
    }
  }
  return c.off;
}

// Points -> QCQP -> soft -> J for B trajectories x P rows.  Every array the
// finish kernel reads (pts, qcost, qstatus, softc) is written earlier in the
// same stream for every row: points by tube_time_points_kernel, qcost and
// qstatus by every workgroup of tube_solve_kernel (also where a trajectory
// fails), softc by the last extremum launch.  With `skip`, trajectories whose
// flag is set are left untouched by the QCQP launch and by the finish kernel.
hipError_t evaluate_points(const TubeArgs& a, int P, const double* T, double tol, int max_iter,
                           const mtg_time_params& p, const Workspace& w, const int32_t* skip,
                           double* Jall, double* cost, double* grad, int32_t* status,
                           hipStream_t st, int32_t* iters = nullptr) {
  const int S = a.S;
  const int64_t BP = a.B * P;
  hipLaunchKernelGGL(tube_time_points_kernel, dim3(blocks_for(BP * S)), dim3(256), 0, st, S,
                     a.B, P, T, p.increment, w.pts);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  TubeArgs q = a;
  q.B = BP;
  q.times = w.pts;
  q.rep = P;
  q.skip = skip;
  e = launch_tube_solve(q, tol, max_iter, nullptr, w.coeffs, w.qcost, iters, w.qstatus, st);
  if (e != hipSuccess) return e;
  if (p.n_soft > 0) {
    SoftLimits lim{};
    lim.n = p.n_soft;
    for (int c = 0; c < p.n_soft; ++c) lim.value[c] = p.soft_limit[c];
    // Finished trajectories (skip) are left out of the searches too.
    SoftCostArgs none{};
    none.skip = skip;
    none.skip_rep = P;
    SoftCostArgs last{w.softc, lim, p.soft_weight, p.soft_maximum_cost};
    last.skip = skip;
    last.skip_rep = P;
    for (int c = 0; c < p.n_soft; ++c) {
      e = launch_max_magnitude(a.N, 3, S, BP, p.soft_derivative[c], w.coeffs, w.pts, nullptr,
                               w.maxima, nullptr, p.n_soft, c, c == p.n_soft - 1 ? last : none,
                               st);
      if (e != hipSuccess) return e;
    }
  }
  hipLaunchKernelGGL(tube_time_finish_kernel, dim3(blocks_for(a.B)), dim3(256), 0, st, S, a.B,
                     P, w.pts, w.qcost, w.qstatus, p.n_soft > 0 ? w.softc : nullptr,
                     p.time_penalty, p.increment, skip, Jall, cost, grad, status);
  return hipGetLastError();
}

// LN_SBPLX is gradient-free: one point per round.
bool sbplx_of(const mtg_time_params& p, bool optimiser) { return optimiser && p.optimizer == 1; }
int points_of(const mtg_time_params& p, int S, bool optimiser) {
  if (sbplx_of(p, optimiser)) return 1;
  return (optimiser || p.grad_mode == 2) ? 2 * S + 1 : 1;
}

}  // namespace

size_t tube_time_workspace_bytes(int N, int S, int64_t B, const mtg_time_params& p,
                                 bool optimiser) {
  Workspace w;
  return carve(nullptr, N, S, B, points_of(p, S, optimiser), p.n_soft, optimiser,
               sbplx_of(p, optimiser), &w) +
         256;
}

int64_t tube_time_problems(int S, int64_t B, const mtg_time_params& p, bool optimiser) {
  return B * points_of(p, S, optimiser);
}

int tube_time_cost(const TubeArgs& a, double tol, int max_iter, const mtg_time_params& p,
                   double* cost, double* grad, int32_t* status, void* workspace,
                   size_t workspace_bytes, hipStream_t st) {
  const int P = points_of(p, a.S, false);
  Workspace w;
  if (tube_time_workspace_bytes(a.N, a.S, a.B, p, false) > workspace_bytes)
    return MTG_ERR_INVALID_ARG;
  carve(workspace, a.N, a.S, a.B, P, p.n_soft, false, false, &w);
  const hipError_t e = evaluate_points(a, P, a.times, tol, max_iter, p, w, nullptr, nullptr,
                                       cost, p.grad_mode == 2 ? grad : nullptr, status, st);
  return e == hipSuccess ? MTG_OK : MTG_ERR_HIP;
}

// The optimiser runs max_evals rounds, all stream-ordered: a trajectory that
// has stopped sets its `done` flag, and later rounds skip it in every kernel
// (its QCQP workgroups return at once), so no host round trip is needed to
// know when to stop and the whole call can be captured in a graph.
int tube_time_optimize(const TubeArgs& a, double* times_io, double tol, int max_iter,
                       const mtg_time_params& p, int max_evals, double* cost, int32_t* evals,
                       int32_t* result, int32_t* status, void* workspace, size_t workspace_bytes,
                       hipStream_t st) {
  const int S = a.S, P = points_of(p, S, true);
  const int64_t B = a.B;
  const bool sb = sbplx_of(p, true);
  Workspace w;
  if (tube_time_workspace_bytes(a.N, S, B, p, true) > workspace_bytes) return MTG_ERR_INVALID_ARG;
  carve(workspace, a.N, S, B, P, p.n_soft, true, sb, &w);
  const OptState& s = w.s;
  if (sb) {
    hipLaunchKernelGGL(tube_time_sbplx_init_kernel, dim3(blocks_for(B)), dim3(256), 0, st, S, B,
                       times_io, p.initial_stepsize_rel > 0.0 ? p.initial_stepsize_rel : 0.1,
                       max_evals, p.f_rel, p.f_abs, s);
  } else {
    hipLaunchKernelGGL(tube_time_opt_init_kernel, dim3(blocks_for(B * S)), dim3(256), 0, st, S,
                       B, times_io, s);
  }
  if (hipGetLastError() != hipSuccess) return MTG_ERR_HIP;
  // Control-point maps stay at the initial times (built once at setup,
  // qcqp_impl:152-157); Q and A^-1 follow the evaluation points.
  TubeArgs q = a;
  q.times_cp = s.T0;
  if (sb) {
    // Consecutive evaluations of a trajectory share the constraints (maps at
    // T0): each solve warm-starts from the trajectory's previous one
    // (Tube::warm_start; the oracle's driver does the same).
    q.warm = s.warm;
    q.warm_ok = s.warm_ok;
  }
  for (int round = 0; round < max_evals; ++round) {
    // LN_SBPLX: from the second round on, the longest solves go first
    if (sb) q.order = round > 0 ? s.order : nullptr;
    hipError_t e = evaluate_points(q, P, s.Ttr, tol, max_iter, p, w, s.done, w.Jall, nullptr,
                                   nullptr, nullptr, st, sb ? s.iters : nullptr);
    if (e != hipSuccess) return MTG_ERR_HIP;
    if (sb) {
      hipLaunchKernelGGL(tube_time_sbplx_step_kernel, dim3(blocks_for(B)), dim3(256), 0, st, S,
                         B, round == 0 ? 1 : 0, w.Jall, w.qstatus, s);
      if (round + 1 < max_evals)
        hipLaunchKernelGGL(tube_time_order_kernel, dim3(1), dim3(1024), 0, st, B, s.iters,
                           s.done, s.order);
    }
    else
      hipLaunchKernelGGL(tube_time_opt_step_kernel, dim3(blocks_for(B)), dim3(256), 0, st, S, B,
                         P, round == 0 ? 1 : 0, max_evals, p.increment, w.Jall, w.qstatus, s);
    if (hipGetLastError() != hipSuccess) return MTG_ERR_HIP;
  }
  if (sb) {
    hipLaunchKernelGGL(tube_time_sbplx_final_kernel, dim3(blocks_for(B)), dim3(256), 0, st, S, B,
                       s, times_io, cost, evals, result, status);
  } else {
    hipLaunchKernelGGL(tube_time_opt_final_kernel, dim3(blocks_for(B * S)), dim3(256), 0, st, S,
                       B, s, times_io, cost, evals, status);
    // the descent's stopping reason: 5 at max_evals, 4 when its step vanished
    if (result && hipGetLastError() == hipSuccess)
      hipLaunchKernelGGL(tube_time_opt_result_kernel, dim3(blocks_for(B)), dim3(256), 0, st, B,
                         max_evals, s, result);
  }
  return hipGetLastError() == hipSuccess ? MTG_OK : MTG_ERR_HIP;
}

}  // namespace mtg
