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
// together with the trial itself, so one round = one counted evaluation and
// the host loop runs at most max_evals rounds (ending early when no
// trajectory is active).
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_internal.h"

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
                                        double h, double* __restrict__ Jall,
                                        double* __restrict__ cost, double* __restrict__ grad,
                                        int32_t* __restrict__ status) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
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
                                          const int32_t* __restrict__ qstatus, OptState s,
                                          int32_t* __restrict__ n_active) {
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
  if (stop) {
    s.done[b] = 1;
  } else {
    atomicAdd(n_active, 1);
  }
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

unsigned blocks_for(int64_t n) { return static_cast<unsigned>((n + 255) / 256); }

// Scratch for one call, released in the destructor after the stream's work.
// Plain hipMalloc/hipFree, not the stream-ordered pool: the C++ shim's
// hipMalloc'd buffers interleaved with hipMallocAsync/hipFreeAsync on the
// null stream intermittently read a stale cost back (one run in three on
// MI355X, tests/cpp TimeCostWithQCQPInnerSolve); the allocation is
// microseconds against a QCQP launch of milliseconds.
struct Scratch {
  hipStream_t st;
  void* p = nullptr;
  explicit Scratch(hipStream_t s) : st(s) {}
  ~Scratch() {
    if (p) {
      (void)hipStreamSynchronize(st);
      (void)hipFree(p);
    }
  }
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes); }
};

// Points -> QCQP -> soft -> J for B trajectories x P rows.
hipError_t evaluate_points(const TubeArgs& a, int P, const double* T, double tol, int max_iter,
                           const mtg_time_params& p, double* pts, double* coeffs,
                           double* qcost, int32_t* qstatus, double* maxima, double* softc,
                           double* Jall, double* cost, double* grad, int32_t* status,
                           hipStream_t st) {
  const int S = a.S;
  const int64_t BP = a.B * P;
  hipLaunchKernelGGL(tube_time_points_kernel, dim3(blocks_for(BP * S)), dim3(256), 0, st, S,
                     a.B, P, T, p.increment, pts);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  TubeArgs q = a;
  q.B = BP;
  q.times = pts;
  q.rep = P;
  e = launch_tube_solve(q, tol, max_iter, nullptr, coeffs, qcost, nullptr, qstatus, st);
  if (e != hipSuccess) return e;
  if (p.n_soft > 0) {
    SoftLimits lim{};
    lim.n = p.n_soft;
    for (int c = 0; c < p.n_soft; ++c) lim.value[c] = p.soft_limit[c];
    const SoftCostArgs none{};
    const SoftCostArgs last{softc, lim, p.soft_weight, p.soft_maximum_cost};
    for (int c = 0; c < p.n_soft; ++c) {
      e = launch_max_magnitude(a.N, 3, S, BP, p.soft_derivative[c], coeffs, pts, nullptr, maxima,
                               nullptr, p.n_soft, c, c == p.n_soft - 1 ? last : none, st);
      if (e != hipSuccess) return e;
    }
  }
  hipLaunchKernelGGL(tube_time_finish_kernel, dim3(blocks_for(a.B)), dim3(256), 0, st, S, a.B,
                     P, pts, qcost, qstatus, p.n_soft > 0 ? softc : nullptr, p.time_penalty,
                     p.increment, Jall, cost, grad, status);
  return hipGetLastError();
}

// Workspace of evaluate_points for B x P problems, carved from one block.
struct PointBuffers {
  double *pts, *coeffs, *qcost, *maxima, *softc, *Jall;
  int32_t* qstatus;
};
size_t point_bytes(int N, int S, int64_t BP, int n_soft) {
  return sizeof(double) * BP * (S + static_cast<size_t>(S) * 3 * N + 3 + (n_soft > 0 ? n_soft : 1)) +
         sizeof(int32_t) * (BP + 2);
}
PointBuffers carve_points(void* base, int N, int S, int64_t BP, int n_soft) {
  PointBuffers pb;
  double* d = static_cast<double*>(base);
  pb.coeffs = d;  // 16-byte aligned first (S * 3 * N doubles per problem)
  d += BP * S * 3 * N;
  pb.pts = d;
  d += BP * S;
  pb.qcost = d;
  d += BP;
  pb.softc = d;
  d += BP;
  pb.Jall = d;
  d += BP;
  pb.maxima = d;
  d += BP * (n_soft > 0 ? n_soft : 1);
  pb.qstatus = reinterpret_cast<int32_t*>(d);
  return pb;
}

}  // namespace

int tube_time_cost(const TubeArgs& a, double tol, int max_iter, const mtg_time_params& p,
                   double* cost, double* grad, int32_t* status, hipStream_t st) {
  const int P = p.grad_mode == 2 ? 2 * a.S + 1 : 1;
  const int64_t BP = a.B * P;
  Scratch ws(st);
  if (ws.alloc(point_bytes(a.N, a.S, BP, p.n_soft)) != hipSuccess) return MTG_ERR_HIP;
  const PointBuffers pb = carve_points(ws.p, a.N, a.S, BP, p.n_soft);
  const hipError_t e =
      evaluate_points(a, P, a.times, tol, max_iter, p, pb.pts, pb.coeffs, pb.qcost, pb.qstatus,
                      pb.maxima, pb.softc, nullptr, cost, p.grad_mode == 2 ? grad : nullptr,
                      status, st);
  return e == hipSuccess ? MTG_OK : MTG_ERR_HIP;
}

int tube_time_optimize(const TubeArgs& a, double* times_io, double tol, int max_iter,
                       const mtg_time_params& p, int max_evals, double* cost, int32_t* evals,
                       int32_t* status, hipStream_t st) {
  const int S = a.S, P = 2 * S + 1;
  const int64_t B = a.B, BP = B * P;
  const size_t state_bytes = sizeof(double) * (4 * B * S + 2 * B) + sizeof(int32_t) * (3 * B + 2);
  Scratch ws(st);
  const size_t pbytes = point_bytes(a.N, S, BP, p.n_soft);
  if (ws.alloc(pbytes + state_bytes + 64) != hipSuccess) return MTG_ERR_HIP;
  const PointBuffers pb = carve_points(ws.p, a.N, S, BP, p.n_soft);
  double* d = reinterpret_cast<double*>(static_cast<char*>(ws.p) + ((pbytes + 15) & ~size_t(15)));
  OptState s;
  s.T0 = d;
  s.Tc = d + B * S;
  s.g = d + 2 * B * S;
  s.Ttr = d + 3 * B * S;
  s.f = d + 4 * B * S;
  s.alpha = s.f + B;
  s.evals = reinterpret_cast<int32_t*>(s.alpha + B);
  s.done = s.evals + B;
  s.st = s.done + B;
  int32_t* n_active = s.st + B;
  hipLaunchKernelGGL(tube_time_opt_init_kernel, dim3(blocks_for(B * S)), dim3(256), 0, st, S, B,
                     times_io, s);
  if (hipGetLastError() != hipSuccess) return MTG_ERR_HIP;
  // Control-point maps stay at the initial times (built once at setup,
  // qcqp_impl:152-157); Q and A^-1 follow the evaluation points.
  TubeArgs q = a;
  q.times_cp = s.T0;
  int32_t host_active = 0;
  for (int round = 0; round < max_evals; ++round) {
    hipError_t e = evaluate_points(q, P, s.Ttr, tol, max_iter, p, pb.pts, pb.coeffs, pb.qcost,
                                   pb.qstatus, pb.maxima, pb.softc, pb.Jall, nullptr, nullptr,
                                   nullptr, st);
    if (e != hipSuccess) return MTG_ERR_HIP;
    if (hipMemsetAsync(n_active, 0, sizeof(int32_t), st) != hipSuccess) return MTG_ERR_HIP;
    hipLaunchKernelGGL(tube_time_opt_step_kernel, dim3(blocks_for(B)), dim3(256), 0, st, S, B, P,
                       round == 0 ? 1 : 0, max_evals, p.increment, pb.Jall, pb.qstatus, s,
                       n_active);
    if (hipGetLastError() != hipSuccess) return MTG_ERR_HIP;
    if (hipMemcpyAsync(&host_active, n_active, sizeof(int32_t), hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return MTG_ERR_HIP;
    if (host_active == 0) break;
  }
  hipLaunchKernelGGL(tube_time_opt_final_kernel, dim3(blocks_for(B * S)), dim3(256), 0, st, S, B,
                     s, times_io, cost, evals, status);
  return hipGetLastError() == hipSuccess ? MTG_OK : MTG_ERR_HIP;
}

}  // namespace mtg
