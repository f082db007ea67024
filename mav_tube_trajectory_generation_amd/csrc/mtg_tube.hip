// mtg_tube.hip — tube QCQP kernels (solveQCQP replacement and constraint
// residuals), one 64-lane workgroup per trajectory (mtg_tube_device.h).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>

#include "mtg_internal.h"
#include "mtg_tube_device.h"

namespace mtg {

template <int N>
__device__ inline Tube<N> make_tube(const TubeLayout* L, double* smem, int S, int r,
                                    const double* tab) {
  const int tid = static_cast<int>(threadIdx.x);
  return Tube<N>{S,   r,         S - 1, tube_ncon(N, S), L, smem, tid & (kWave - 1), tab,
                 tid, static_cast<int>(blockDim.x),
                 __builtin_amdgcn_readfirstlane(tid / kWave)};
}

// Constraint residuals g_k(x) (compute_sphere/tube/tube_end_constraints,
// qcqp_impl:357-474) at x given in the reference's dimension-major order.
template <int N>
__global__ __launch_bounds__(kWave) void tube_residuals_kernel(
    int S, int r, int rep, const double* __restrict__ tab, const double* __restrict__ positions,
    const double* __restrict__ fixed_vals, const double* __restrict__ times_cp,
    const double* __restrict__ times, const double* __restrict__ radii,
    const double* __restrict__ x, double* __restrict__ resid) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const TubeLayout L = make_tube_layout(N, S);
  Tube<N> t = make_tube<N>(&L, smem, S, r, tab);
  int* bad = reinterpret_cast<int*>(smem + L.ndouble);
  const int64_t b = blockIdx.x;
  constexpr int M = N / 2;
  t.setup(tab, b, b / rep, positions, fixed_vals, times_cp, times, radii, bad);
  const int n = t.nv * 3 * M;
  for (int idx = t.tid; idx < n; idx += t.nthr) {
    // reference order d*(S-1)*M + (u-1)*M + m  ->  internal ((u-1)*3+d)*M + m
    const int d = idx / ((S - 1) * M), a = (idx / M) % (S - 1), m = idx % M;
    smem[L.x + (a * 3 + d) * M + m] = x[b * n + idx];
  }
  __syncthreads();
  t.control_points(smem + L.x, L.cp);
  __syncthreads();
  for (int k = t.tid; k < t.nc; k += t.nthr) {
    double w[3];
    resid[b * t.nc + k] = t.con_eval(k, L.cp, w);
  }
}

// Two waves per trajectory for N <= 10: both run the data-parallel phases,
// wave 0 the block factorisation and solves; with 40 KB of LDS per
// trajectory a CU holds 4 trajectories = 8 waves, two per SIMD (registers
// capped at 256 per wave).  N = 12 keeps one wave (its 18 x 18 blocks need
// more registers than two waves per SIMD leave).
template <int N>
constexpr int tube_threads() { return N <= 10 ? 2 * kWave : kWave; }

// The kernel body for S segments (a kernel argument, or a compile-time
// constant in tube_solve_s_kernel).
template <int N>
__device__ __attribute__((always_inline)) void tube_solve_body(
    int S, int r, int rep, const double* __restrict__ tab, const double* __restrict__ positions,
    const double* __restrict__ fixed_vals, const double* __restrict__ times_cp,
    const double* __restrict__ times, const double* __restrict__ radii, double tol,
    int max_iter, const int32_t* __restrict__ skip, double* __restrict__ x_out,
    double* __restrict__ coeffs, double* __restrict__ cost, int32_t* __restrict__ iters,
    int32_t* __restrict__ status, double* __restrict__ warm, int32_t* __restrict__ warm_ok,
    const int32_t* __restrict__ order) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  // The problem of this workgroup: order[blockIdx.x] (TubeArgs::order:
  // workgroups are dispatched in blockIdx order, so the longest solves go
  // first), else the XCD-contiguous map (mtg_device.h).
  const int64_t b = order ? order[blockIdx.x] : xcd_problem(blockIdx.x, gridDim.x);
  if (skip && skip[b / rep]) return;  // workgroup-uniform
  const TubeLayout L = make_tube_layout(N, S);
  Tube<N> t = make_tube<N>(&L, smem, S, r, tab);
  int* bad = reinterpret_cast<int*>(smem + L.ndouble);
  constexpr int M = N / 2;
  t.setup(tab, b, b / rep, positions, fixed_vals, times_cp, times, radii, bad);
  int st = 1;
  int it = 0;
  // Warm-start state of problem b (TubeArgs::warm): x, s, lam of its last
  // usable solve, valid where warm_ok[b].
  double* ws = warm ? warm + b * static_cast<int64_t>(t.nv * 3 * M + 2 * t.nc) : nullptr;
  const bool use_ws = warm && warm_ok[b];
  if (!(*bad & 1)) it = t.ipm(tol, max_iter, &st, bad, use_ws ? ws : nullptr);
  __syncthreads();
  if (warm && !(*bad & 3) && st != 2) {
    t.save_state(ws);
    if (t.tid == 0) warm_ok[b] = 1;
  }
  // Bit 0: a time is not positive; bit 1: the start system is not positive
  // definite, so x was never written.  Either way the outputs are NaN.
  const int fl = *bad;
  const bool no_x = (fl & 3) != 0;
  // The powers share LDS with the factors: recompute them for the outputs.
  if (!(fl & 1)) t.compute_powers();
  __syncthreads();
  // Outputs: x (reference order), coefficients (qcqp_impl:777-785 ->
  // linear_impl:254-275) and computeCost (linear_impl:113-130).
  const int n = t.nv * 3 * M;
  if (x_out)
    for (int idx = t.tid; idx < n; idx += t.nthr) {
      const int d = idx / ((S - 1) * M), a = (idx / M) % (S - 1), m = idx % M;
      x_out[b * n + idx] = no_x ? NAN : smem[L.x + (a * 3 + d) * M + m];
    }
  const double* xv = smem + L.x;
  double acc = 0.0;
  const int per = S * 3 * N;
  for (int i = t.tid; i < per; i += t.nthr) {
    const int s = i / (3 * N), d = (i / N) % 3, k = i % N;
    const int lk = k % M;
    double c = 0.0, h = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int l = j % M;
      const double e = t.xval(xv, s + j / M, d, l);
      c += tab[N * N + k * N + j] * t.pwr(s, l - k) * e;
      h += tab[k * N + j] * t.pwr(s, 1 - 2 * r + lk + l) * e;
    }
    coeffs[b * per + i] = no_x ? NAN : c;
    acc += h * t.xval(xv, s + k / M, d, lk);
  }
  const double J = 0.5 * t.block_sum(acc);
  if (t.tid == 0) {
    if (cost) cost[b] = no_x ? NAN : J;
    if (iters) iters[b] = it;
    if (status)
      status[b] = (fl & 1) ? MTG_TRAJ_BAD_TIME
                           : ((fl & 2) || st == 2) ? MTG_TRAJ_NOT_SPD
                           : st == 0 ? MTG_TRAJ_OK
                           : st == 3 ? MTG_TRAJ_NEAR_OPTIMAL : MTG_TRAJ_NOT_CONVERGED;
  }
}

#define MTG_TUBE_SOLVE_PARAMS                                                                  \
  int S, int r, int rep, const double* __restrict__ tab, const double* __restrict__ positions, \
      const double* __restrict__ fixed_vals, const double* __restrict__ times_cp,              \
      const double* __restrict__ times, const double* __restrict__ radii, double tol,          \
      int max_iter, const int32_t* __restrict__ skip, double* __restrict__ x_out,              \
      double* __restrict__ coeffs, double* __restrict__ cost, int32_t* __restrict__ iters,     \
      int32_t* __restrict__ status, double* __restrict__ warm, int32_t* __restrict__ warm_ok,  \
      const int32_t* __restrict__ order

template <int N>
__global__ __launch_bounds__(tube_threads<N>())
__attribute__((amdgpu_waves_per_eu(tube_threads<N>() / kWave, tube_threads<N>() / kWave)))
void tube_solve_kernel(MTG_TUBE_SOLVE_PARAMS) {
  tube_solve_body<N>(S, r, rep, tab, positions, fixed_vals, times_cp, times, radii, tol, max_iter,
                     skip, x_out, coeffs, cost, iters, status, warm, warm_ok, order);
}

// S a compile-time constant (the argument S is ignored): every layout
// offset, loop bound and index division by S folds into the code, which
// frees the registers that held them (N = 10, S = 2..16).
template <int N, int SC>
__global__ __launch_bounds__(tube_threads<N>())
__attribute__((amdgpu_waves_per_eu(tube_threads<N>() / kWave, tube_threads<N>() / kWave)))
void tube_solve_s_kernel(MTG_TUBE_SOLVE_PARAMS) {
  tube_solve_body<N>(SC, r, rep, tab, positions, fixed_vals, times_cp, times, radii, tol, max_iter,
                     skip, x_out, coeffs, cost, iters, status, warm, warm_ok, order);
}

#ifdef MTG_STAMPS
extern "C" int mtg_debug_tube_stamps(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mtg_stamps), sizeof(unsigned long long) * n) ==
                 hipSuccess ? 0 : -3;
}
#endif

int64_t tube_warm_doubles(int N, int S) {
  return static_cast<int64_t>(S - 1) * 3 * (N / 2) + 2 * tube_ncon(N, S);
}

size_t tube_lds_bytes(int N, int S) {
  if (S < 2) return 0;
  return make_tube_layout(N, S).bytes() + 16;  // + 2 ints (bad, fail)
}

namespace {
template <typename K>
hipError_t prepare_lds(K kernel, size_t bytes) {
  if (bytes > 65536)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               static_cast<int>(bytes));
  return hipSuccess;
}

template <int N>
hipError_t residuals_n(const TubeArgs& a, const double* x, double* resid, hipStream_t st) {
  const size_t bytes = tube_lds_bytes(N, a.S);
  hipError_t e = prepare_lds(tube_residuals_kernel<N>, bytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tube_residuals_kernel<N>, dim3(static_cast<unsigned>(a.B)), dim3(kWave),
                     bytes, st, a.S, a.r, a.rep, a.tab, a.positions, a.fixed_vals, a.times_cp,
                     a.times, a.radii, x, resid);
  return hipGetLastError();
}

template <typename K>
hipError_t solve_launch(K kernel, int threads, const TubeArgs& a, double tol, int max_iter,
                        double* x, double* coeffs, double* cost, int32_t* iters, int32_t* status,
                        hipStream_t st) {
  const size_t bytes = tube_lds_bytes(a.N, a.S);
  hipError_t e = prepare_lds(kernel, bytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(a.B)), dim3(threads), bytes, st, a.S,
                     a.r, a.rep, a.tab, a.positions, a.fixed_vals, a.times_cp, a.times, a.radii,
                     tol, max_iter, a.skip, x, coeffs, cost, iters, status, a.warm, a.warm_ok,
                     a.order);
  return hipGetLastError();
}

// The compile-time-S kernels unless MTG_TUBE_RUNTIME_S=1 (A/B runs).
bool tube_runtime_s_forced() {
  static const bool forced = [] {
    const char* e = std::getenv("MTG_TUBE_RUNTIME_S");
    return e && e[0] == '1';
  }();
  return forced;
}

template <int N>
hipError_t solve_n(const TubeArgs& a, double tol, int max_iter, double* x, double* coeffs,
                   double* cost, int32_t* iters, int32_t* status, hipStream_t st) {
  constexpr int T = tube_threads<N>();
  if constexpr (N == 10) {
    if (!tube_runtime_s_forced()) {
      switch (a.S) {
#define MTG_TUBE_S(SS)                                                                     \
  case SS:                                                                                 \
    return solve_launch(tube_solve_s_kernel<10, SS>, T, a, tol, max_iter, x, coeffs, cost, \
                        iters, status, st);
        MTG_TUBE_S(2) MTG_TUBE_S(3) MTG_TUBE_S(4) MTG_TUBE_S(5) MTG_TUBE_S(6) MTG_TUBE_S(7)
        MTG_TUBE_S(8) MTG_TUBE_S(9) MTG_TUBE_S(10) MTG_TUBE_S(11) MTG_TUBE_S(12) MTG_TUBE_S(13)
        MTG_TUBE_S(14) MTG_TUBE_S(15) MTG_TUBE_S(16)
#undef MTG_TUBE_S
        default: break;
      }
    }
  }
  return solve_launch(tube_solve_kernel<N>, T, a, tol, max_iter, x, coeffs, cost, iters, status,
                      st);
}
}  // namespace

#define MTG_TUBE_DISPATCH(CALL)              \
  switch (a.N) {                             \
    case 4: return CALL(4);                  \
    case 6: return CALL(6);                  \
    case 8: return CALL(8);                  \
    case 10: return CALL(10);                \
    case 12: return CALL(12);                \
    default: return hipErrorInvalidValue;    \
  }

hipError_t launch_tube_residuals(const TubeArgs& a, const double* x, double* resid,
                                 hipStream_t st) {
#define CALL(n) residuals_n<n>(a, x, resid, st)
  MTG_TUBE_DISPATCH(CALL)
#undef CALL
}

hipError_t launch_tube_solve(const TubeArgs& a, double tol, int max_iter, double* x,
                             double* coeffs, double* cost, int32_t* iters, int32_t* status,
                             hipStream_t st) {
#define CALL(n) solve_n<n>(a, tol, max_iter, x, coeffs, cost, iters, status, st)
  MTG_TUBE_DISPATCH(CALL)
#undef CALL
}

}  // namespace mtg
