// mtg_extrema.hip — batched magnitude extrema:
// PolynomialOptimization::computeMaximumOfMagnitude (reference
// polynomial_optimization_linear_impl.h:455-487) over a batch of solved
// trajectories, and the soft-constraint cost built on it
// (evaluateMaximumMagnitudeAsSoftConstraint, nonlinear_impl:2735-2766).
//
// The reference's candidates for segment s are t = 0, T_s and the real roots
// in [0, T_s] of f = sum_d p_d^(k) p_d^(k+1) = (1/2) d/dt |p^(k)|^2 (the
// convolution of segment.cpp:82-133), found with Jenkins-Traub
// (rpoly_ak1.cpp:70-117); the maximum of |p^(k)| over the candidates wins.
// The maximum over [0, T_s] is attained at an endpoint or at a sign change of
// f, so the kernel only needs the real roots of f in [0, T_s], not all
// complex roots.  It isolates them by Bernstein subdivision (Descartes' rule
// of signs on the Bernstein coefficients: the number of sign variations
// bounds the number of roots in the interval, and exactly one variation
// means exactly one root) and refines each isolated root by
// Laguerre iteration (bisection-safeguarded).
//
// Layout: one lane = one segment part.  A segment's [0, T] is split into
// P dyadic parts (P = 8 by default) so that B x S x P lanes fill the chip;
// each lane walks the dyadic tree of its part depth-first without a stack:
// the Bernstein coefficients of a node are recomputed from the segment's
// [0, 1] coefficients by two de Casteljau splits, so all arrays stay in
// registers with compile-time indices.  Candidate magnitudes are evaluated
// from the coefficients (L1-resident).  The lanes of one trajectory sit in
// one workgroup and reduce through LDS in the reference's candidate order
// (segment ascending, first maximum wins).  The last constraint's launch of
// a soft-constraint evaluation also forms the cost (nonlinear_impl:
// 2747-2763).  FP64 VALU bound.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_extrema_device.h"

namespace mtg {

constexpr int kExtBlock = 256;

template <int N, int K, bool kMin>
__global__ __launch_bounds__(kExtBlock) void max_magnitude_kernel(
    int D, int S, int64_t B, int parts, int log2parts, const double* __restrict__ coeffs,
    const double* __restrict__ times, double* __restrict__ max_time,
    double* __restrict__ max_value, int32_t* __restrict__ max_segment, int value_stride,
    int value_offset, SoftCostArgs soft, MinOut mino) {
  __shared__ double val_s[kExtBlock];
  __shared__ double time_s[kExtBlock];
  __shared__ double mval_s[kMin ? kExtBlock : 1];
  __shared__ double mtime_s[kMin ? kExtBlock : 1];
  // The block's trajectories (coefficients, then segment times), staged
  // once with coalesced loads: every magnitude evaluation reads LDS.
  extern __shared__ double traj_s[];
  const int tid = threadIdx.x;
  const int lanes_per_traj = S * parts;
  const int traj_per_block = kExtBlock / lanes_per_traj;
  const int bl = tid / lanes_per_traj;
  const int rem = tid - bl * lanes_per_traj;
  const int s = rem >> log2parts;
  const int part = rem & (parts - 1);
  const int64_t b = static_cast<int64_t>(blockIdx.x) * traj_per_block + bl;
  const bool skipped = b < B && soft.skip && soft.skip[b / soft.skip_rep];
  const bool active = bl < traj_per_block && b < B && !skipped;
  {
    const int64_t b0 = static_cast<int64_t>(blockIdx.x) * traj_per_block;
    const int nt = static_cast<int>(min(static_cast<int64_t>(traj_per_block), B - b0));
    const int per = S * D * N;
    const double* src = coeffs + b0 * per;
    for (int i = tid; i < nt * per; i += kExtBlock) traj_s[i] = src[i];
    double* ts = traj_s + traj_per_block * per;
    for (int i = tid; i < nt * S; i += kExtBlock) ts[i] = times[b0 * S + i];
  }
  __syncthreads();

  double best_v = -1.0, best_t = 0.0;  // |p|^2 and time of this lane's best
  double min_v = HUGE_VAL, min_t = 0.0;
  if (active) {
    const double T = traj_s[traj_per_block * S * D * N + bl * S + s];
    const double* c = traj_s + (bl * S + s) * D * N;
    // Pruning bound: |p^(K)|^2 at the part's right end (a wave may hold
    // several trajectories, so the bound stays per lane).
    const double lb = kMin ? 0.0 : ext_mag2<N, K>(c, D, ldexp(T * (part + 1), -log2parts));
    ext_segment_search<N, K, kMin>(c, D, T, part, parts, log2parts, best_v, best_t, min_v,
                                   min_t, lb);
  }
  val_s[tid] = best_v;
  time_s[tid] = best_t;
  if constexpr (kMin) {
    mval_s[tid] = min_v;
    mtime_s[tid] = min_t;
  }
  __syncthreads();
  // Reduction in candidate order: segment ascending, part ascending; strict
  // '>' keeps the first maximum (Extremum::operator<, extremum.h:35-36;
  // linear_impl:474).  Extremum() starts at {0, 0, 0}.
  if (active && rem == 0) {  // skipped trajectories keep their outputs
    double v = 0.0, t = 0.0;
    int seg = 0;
    for (int i = 0; i < lanes_per_traj; ++i) {
      const double x = val_s[tid + i];
      if (x > v) {
        v = x;
        t = time_s[tid + i];
        seg = i >> log2parts;
      }
    }
    const double vmax = sqrt(v);
    if (max_value) max_value[b * value_stride + value_offset] = vmax;
    if (soft.cost) {
      // Last constraint of a soft-constraint evaluation: the earlier
      // constraints' maxima are in max_value (stream-ordered launches).
      double total = 0.0;
#pragma unroll
      for (int cidx = 0; cidx < kMaxSoftConstraints; ++cidx) {  // compile-time index
        if (cidx >= soft.lim.n) break;
        const double m = cidx == value_offset ? vmax : max_value[b * value_stride + cidx];
        const double abs_violation = m - soft.lim.value[cidx];
        const double relative_violation = abs_violation / soft.lim.value[cidx];
        total += fmin(soft.maximum_cost, exp(relative_violation * soft.weight));
      }
      soft.cost[b] = total;
    }
    if (max_time) max_time[b] = t;
    if (max_segment) max_segment[b] = seg;
    if constexpr (kMin) {
      // Same order, strict '<' from +max (trajectory.cpp:191-215).
      double mv = HUGE_VAL, mt = 0.0;
      int mseg = 0;
      for (int i = 0; i < lanes_per_traj; ++i) {
        const double x = mval_s[tid + i];
        if (x < mv) {
          mv = x;
          mt = mtime_s[tid + i];
          mseg = i >> log2parts;
        }
      }
      if (mino.value) mino.value[b] = sqrt(mv);
      if (mino.time) mino.time[b] = mt;
      if (mino.segment) mino.segment[b] = mseg;
    }
  }
}

template <int N, bool kMin>
static hipError_t launch_max_n(int K, int D, int S, int64_t B, int parts, int log2parts,
                               const double* coeffs, const double* times, double* tmax,
                               double* vmax, int32_t* smax, int stride, int offset,
                               const SoftCostArgs& soft, const MinOut& mino, hipStream_t st) {
  const int tpb = kExtBlock / (S * parts);
  const dim3 grid(static_cast<unsigned>((B + tpb - 1) / tpb));
  const size_t lds = sizeof(double) * static_cast<size_t>(tpb) * S * (D * N + 1);
#define CALL(k)                                                                                \
  if (lds > 65536) {                                                                           \
    const hipError_t e = hipFuncSetAttribute(                                                  \
        reinterpret_cast<const void*>(max_magnitude_kernel<N, k, kMin>),                       \
        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));                     \
    if (e != hipSuccess) return e;                                                             \
  }                                                                                            \
  hipLaunchKernelGGL((max_magnitude_kernel<N, k, kMin>), grid, dim3(kExtBlock), lds, st, D, S,    \
                     B, parts, log2parts, coeffs, times, tmax, vmax, smax, stride, offset, soft,  \
                     mino)
  switch (K) {
    case 0: CALL(0); break;
    case 1: CALL(1); break;
    case 2: CALL(2); break;
    case 3:
      if constexpr (N >= 5) { CALL(3); break; }
      return hipErrorInvalidValue;
    case 4:
      if constexpr (N >= 6) { CALL(4); break; }
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
#undef CALL
  return hipGetLastError();
}

hipError_t launch_max_magnitude(int N, int D, int S, int64_t B, int derivative,
                                const double* coeffs, const double* times, double* max_time,
                                double* max_value, int32_t* max_segment, int value_stride,
                                int value_offset, const SoftCostArgs& soft, hipStream_t st,
                                const MinOut* mino) {
  if (S < 1 || S > kExtBlock || derivative < 0 || derivative > kMaxExtremaDerivative ||
      N - derivative - 1 <= 0)
    return hipErrorInvalidValue;
  int parts = kExtParts, log2parts = 3;
  while (S * parts > kExtBlock) {
    parts >>= 1;
    --log2parts;
  }
  const MinOut none{};
#define CALL(n)                                                                               \
  (mino ? launch_max_n<n, true>(derivative, D, S, B, parts, log2parts, coeffs, times,          \
                                max_time, max_value, max_segment, value_stride, value_offset, \
                                soft, *mino, st)                                              \
        : launch_max_n<n, false>(derivative, D, S, B, parts, log2parts, coeffs, times,         \
                                 max_time, max_value, max_segment, value_stride, value_offset, \
                                 soft, none, st))
  switch (N) {
    case 4: return CALL(4);
    case 6: return CALL(6);
    case 8: return CALL(8);
    case 10: return CALL(10);
    case 12: return CALL(12);
    default: return hipErrorInvalidValue;
  }
#undef CALL
}

// ---------------------------------------------------------------------------
// The candidate lists themselves (computeMaximumOfMagnitude's optional
// `candidates`, linear_impl:455-487; Segment::computeMinMaxMagnitudeCandidates,
// segment.cpp:82-161): one lane per (trajectory, segment) walks the whole
// segment (one part) with the exhaustive search and writes t = 0, T and the
// real roots of f in [0, T] ascending, with |p^(K)| at each.  A segment with
// T < 0 or NaN has no candidates (the reference's t_start > t_end warning).
template <int N, int K>
__global__ __launch_bounds__(kExtBlock) void magnitude_candidates_kernel(
    int D, int64_t n_seg, const double* __restrict__ coeffs, const double* __restrict__ times,
    int cap, double* __restrict__ cand_time, double* __restrict__ cand_value,
    int32_t* __restrict__ n_cand) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kExtBlock + threadIdx.x;
  if (i >= n_seg) return;
  const double T = times[i];
  ExtEmit em{cand_time + i * cap, cand_value + i * cap, cap, 0, D == 1};
  if (T >= 0.0) {
    double bv = 0.0, bt = 0.0, mv = HUGE_VAL, mt = 0.0;
    ext_segment_search<N, K, true, true>(coeffs + i * D * N, D, T, 0, 1, 0, bv, bt, mv, mt, 0.0,
                                         &em);
  }
  n_cand[i] = em.n;
}

template <int N>
static hipError_t launch_cand_n(int K, int D, int64_t n_seg, const double* coeffs,
                                const double* times, int cap, double* ct, double* cv,
                                int32_t* nc, hipStream_t st) {
  const dim3 grid(static_cast<unsigned>((n_seg + kExtBlock - 1) / kExtBlock));
#define CALL(k)                                                                           \
  hipLaunchKernelGGL((magnitude_candidates_kernel<N, k>), grid, dim3(kExtBlock), 0, st, D, \
                     n_seg, coeffs, times, cap, ct, cv, nc)
  switch (K) {
    case 0: CALL(0); break;
    case 1: CALL(1); break;
    case 2: CALL(2); break;
    case 3:
      if constexpr (N >= 5) { CALL(3); break; }
      return hipErrorInvalidValue;
    case 4:
      if constexpr (N >= 6) { CALL(4); break; }
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
#undef CALL
  return hipGetLastError();
}

hipError_t launch_magnitude_candidates(int N, int D, int64_t n_seg, int derivative,
                                       const double* coeffs, const double* times, int cap,
                                       double* cand_time, double* cand_value, int32_t* n_cand,
                                       hipStream_t st) {
  if (derivative < 0 || derivative > kMaxExtremaDerivative || N - derivative - 1 <= 0)
    return hipErrorInvalidValue;
  if (n_seg == 0) return hipSuccess;
#define CALL(n) launch_cand_n<n>(derivative, D, n_seg, coeffs, times, cap, cand_time, \
                                 cand_value, n_cand, st)
  switch (N) {
    case 4: return CALL(4);
    case 6: return CALL(6);
    case 8: return CALL(8);
    case 10: return CALL(10);
    case 12: return CALL(12);
    default: return hipErrorInvalidValue;
  }
#undef CALL
}

// ---------------------------------------------------------------------------
// evaluateMaximumMagnitudeAsSoftConstraint (nonlinear_impl:2735-2766) for
// every constraint in one launch.  Workgroup = one trajectory; lane group c
// (a whole number of waves, so the derivative switch is wave-uniform) runs
// constraint c's search over the (segment, part) items; each group reduces
// in the reference's candidate order, then lane 0 forms
// cost = sum_c min(maximum_cost, exp((max_c - lim_c) / lim_c * weight)).
// The searches of all constraints run concurrently instead of one dependent
// launch each.
constexpr int kSoftBlockMax = 512;  // 2 waves per SIMD: up to 256 VGPRs, no scratch

template <int N>
__global__ __launch_bounds__(kSoftBlockMax) void soft_cost_kernel(int D, int S, int parts, int log2parts,
                                                         int group, const double* __restrict__ coeffs,
                                                         const double* __restrict__ times,
                                                         SoftSpec spec, double* __restrict__ maxima,
                                                         double* __restrict__ cost) {
  extern __shared__ double sm_soft[];
  const int per = S * D * N;
  double* c_s = sm_soft;          // per + S
  double* val_s = sm_soft + per + S;  // blockDim.x
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.x;
  if (spec.skip && spec.skip[b / spec.skip_rep]) return;  // workgroup-uniform
  for (int i = tid; i < per; i += blockDim.x) c_s[i] = coeffs[b * per + i];
  for (int i = tid; i < S; i += blockDim.x) c_s[per + i] = times[b * S + i];
  __syncthreads();
  const int cidx = tid / group, r = tid - cidx * group;
  const bool group_on = cidx < spec.n;  // wave-uniform: groups are whole waves
  const bool active = group_on && r < S * parts;
  double best_v = -1.0, best_t = 0.0, mv = 0.0, mt = 0.0;
  if (group_on) {
    const int s = active ? r >> log2parts : 0, part = r & (parts - 1);
    const double* c = c_s + s * D * N;
    const double T = c_s[per + s];
    int K = 0;
#pragma unroll
    for (int q = 0; q < kMaxSoftConstraints; ++q)  // compile-time indices
      if (q == cidx) K = spec.derivative[q];
    // Every lane of a wave searches the same trajectory and derivative, so
    // the wave's largest |p^(K)|^2 at the parts' right ends bounds the
    // maximum from below for the pruning (idle lanes give 0; all lanes of
    // the wave take part in the exchange).
#define MTG_SOFT_SEARCH(k)                                                                     \
  {                                                                                            \
    double lb = active ? ext_mag2<N, k>(c, D, ldexp(T * (part + 1), -log2parts)) : 0.0;       \
    for (int off = 32; off > 0; off >>= 1) lb = fmax(lb, __shfl_xor(lb, off, 64));             \
    if (active)                                                                                \
      ext_segment_search<N, k>(c, D, T, part, parts, log2parts, best_v, best_t, mv, mt, lb);   \
  }
    switch (K) {
      case 0: MTG_SOFT_SEARCH(0) break;
      case 1: MTG_SOFT_SEARCH(1) break;
      case 2: MTG_SOFT_SEARCH(2) break;
      case 3:
        if constexpr (N >= 5) MTG_SOFT_SEARCH(3)
        break;
      case 4:
        if constexpr (N >= 6) MTG_SOFT_SEARCH(4)
        break;
      default: break;
    }
#undef MTG_SOFT_SEARCH
  }
  val_s[tid] = best_v;
  __syncthreads();
  // Group leaders: maximum in candidate order (strict '>', Extremum() = 0).
  if (cidx < spec.n && r == 0) {
    double v = 0.0;
    for (int i = 0; i < S * parts; ++i) {
      const double x = val_s[tid + i];
      if (x > v) v = x;
    }
    val_s[tid] = sqrt(v);
  }
  __syncthreads();
  if (tid == 0) {
    double total = 0.0;
#pragma unroll
    for (int q = 0; q < kMaxSoftConstraints; ++q) {
      if (q >= spec.n) break;
      const double m = val_s[q * group];
      if (maxima) maxima[b * spec.n + q] = m;
      const double relative_violation = (m - spec.limit[q]) / spec.limit[q];
      total += fmin(spec.maximum_cost, exp(relative_violation * spec.weight));
    }
    cost[b] = total;
  }
}

hipError_t launch_soft_cost(int N, int D, int S, int64_t B, const double* coeffs,
                            const double* times, const SoftSpec& spec, double* maxima,
                            double* cost, hipStream_t st) {
  if (S < 1 || spec.n < 1 || spec.n > kMaxSoftConstraints) return hipErrorInvalidValue;
  int parts = kExtParts, log2parts = 3;
  auto group_of = [&](int p) { return (S * p + 63) / 64 * 64; };
  while (parts > 1 && spec.n * group_of(parts) > kSoftBlockMax) {
    parts >>= 1;
    --log2parts;
  }
  const int group = group_of(parts);
  const int threads = spec.n * group;
  if (threads > kSoftBlockMax) return hipErrorNotSupported;  // caller: one launch per constraint
  const size_t lds = sizeof(double) * (static_cast<size_t>(S) * D * N + S + threads);
  const dim3 grid(static_cast<unsigned>(B));
#define CALL(n)                                                                                 \
  {                                                                                             \
    if (lds > 65536) {                                                                          \
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(soft_cost_kernel<n>), \
                                               hipFuncAttributeMaxDynamicSharedMemorySize,      \
                                               static_cast<int>(lds));                          \
      if (e != hipSuccess) return e;                                                            \
    }                                                                                           \
    hipLaunchKernelGGL(soft_cost_kernel<n>, grid, dim3(threads), lds, st, D, S, parts, log2parts, \
                       group, coeffs, times, spec, maxima, cost);                               \
    return hipGetLastError();                                                                   \
  }
  switch (N) {
    case 4: CALL(4)
    case 6: CALL(6)
    case 8: CALL(8)
    case 10: CALL(10)
    case 12: CALL(12)
    default: return hipErrorInvalidValue;
  }
#undef CALL
}

// Soft-constraint cost of B problems by whichever launch shape fits: all
// constraints in one launch below kSoftOneLaunchMaxBatch problems (latency
// bound), else one launch per constraint, the last forming the cost (maxima:
// B x n scratch).  spec.skip is honoured by both.
hipError_t launch_soft_cost_any(int N, int D, int S, int64_t B, const double* coeffs,
                                const double* times, const SoftSpec& spec, double* maxima,
                                double* cost, hipStream_t st) {
  if (B < kSoftOneLaunchMaxBatch) {
    const hipError_t e = launch_soft_cost(N, D, S, B, coeffs, times, spec, maxima, cost, st);
    if (e != hipErrorNotSupported) return e;
  }
  SoftLimits lim{};
  lim.n = spec.n;
  for (int c = 0; c < spec.n; ++c) lim.value[c] = spec.limit[c];
  SoftCostArgs none{};
  none.skip = spec.skip;
  none.skip_rep = spec.skip_rep;
  SoftCostArgs last{cost, lim, spec.weight, spec.maximum_cost};
  last.skip = spec.skip;
  last.skip_rep = spec.skip_rep;
  for (int c = 0; c < spec.n; ++c) {
    const hipError_t e =
        launch_max_magnitude(N, D, S, B, spec.derivative[c], coeffs, times, nullptr, maxima,
                             nullptr, spec.n, c, c == spec.n - 1 ? last : none, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace mtg
