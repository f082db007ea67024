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

#include "mtg_internal.h"

namespace mtg {

constexpr int kExtBlock = 256;
constexpr int kExtParts = 8;       // dyadic parts per segment (power of 2)
constexpr int kExtMaxLevel = 30;   // node width 2^-30 of the segment: cluster
constexpr int kExtRefineIters = 80;

__host__ __device__ constexpr double ext_falling(int k, int i) {
  double p = 1.0;
  for (int m = 0; m < k; ++m) p *= static_cast<double>(i - m);
  return p;
}

__host__ __device__ constexpr double ext_binom(int n, int k) {
  double r = 1.0;
  for (int i = 1; i <= k; ++i) r = r * static_cast<double>(n - k + i) / static_cast<double>(i);
  return r;
}

// |p^(K)(t)|^2 over the D dimensions of one segment (Polynomial::evaluate,
// polynomial.h:135-149: Horner over base(K, i) c_i).
template <int N, int K>
__device__ inline double ext_mag2(const double* c, int D, double t) {
  double sq = 0.0;
#pragma unroll
  for (int d = 0; d < kMaxD; ++d) {
    if (d >= D) break;
    const double* cd = c + d * N;
    double v = ext_falling(K, N - 1) * cd[N - 1];
#pragma unroll
    for (int i = N - 2; i >= K; --i) v = fma(v, t, ext_falling(K, i) * cd[i]);
    sq = fma(v, v, sq);
  }
  return sq;
}

template <int N, int K>
__global__ __launch_bounds__(kExtBlock) void max_magnitude_kernel(
    int D, int S, int64_t B, int parts, int log2parts, const double* __restrict__ coeffs,
    const double* __restrict__ times, double* __restrict__ max_time,
    double* __restrict__ max_value, int32_t* __restrict__ max_segment, int value_stride,
    int value_offset, SoftCostArgs soft) {
  constexpr int ND = N - K;       // terms of p^(K)
  constexpr int NDD = ND - 1;     // terms of p^(K+1)
  constexpr int M = ND + NDD - 2; // degree of f
  __shared__ double val_s[kExtBlock];
  __shared__ double time_s[kExtBlock];
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
  const bool active = bl < traj_per_block && b < B;
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
  if (active) {
    const double T = traj_s[traj_per_block * S * D * N + bl * S + s];
    const double* c = traj_s + (bl * S + s) * D * N;
    // Endpoint candidates first (the reference lists 0, 0, T, roots).
    if (part == 0) {
      best_v = ext_mag2<N, K>(c, D, 0.0);
      best_t = 0.0;
    }
    if (part == parts - 1) {
      const double v = ext_mag2<N, K>(c, D, T);
      if (v > best_v) {
        best_v = v;
        best_t = T;
      }
    }
    // f(t) = sum_d conv(p_d^(K), p_d^(K+1)), then q(u) = f(T u) on [0, 1].
    double q[M + 1];
#pragma unroll
    for (int j = 0; j <= M; ++j) q[j] = 0.0;
#pragma unroll
    for (int d = 0; d < kMaxD; ++d) {
      if (d >= D) break;
      const double* cd = c + d * N;
      double dv[ND], ddv[NDD];
#pragma unroll
      for (int j = 0; j < ND; ++j) dv[j] = ext_falling(K, j + K) * cd[j + K];
#pragma unroll
      for (int j = 0; j < NDD; ++j) ddv[j] = ext_falling(K + 1, j + K + 1) * cd[j + K + 1];
#pragma unroll
      for (int a = 0; a < ND; ++a)
#pragma unroll
        for (int e = 0; e < NDD; ++e) q[a + e] = fma(dv[a], ddv[e], q[a + e]);
    }
    {
      double tp = T;
#pragma unroll
      for (int j = 1; j <= M; ++j) {
        q[j] *= tp;
        tp *= T;
      }
    }
    // Bernstein coefficients on [0, 1]: beta_i = sum_{j<=i} C(i,j)/C(M,j) q_j,
    // normalised to max |beta| = 1.
    double beta[M + 1];
    double mx = 0.0;
#pragma unroll
    for (int i = 0; i <= M; ++i) {
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j <= i; ++j) acc = fma(ext_binom(i, j) / ext_binom(M, j), q[j], acc);
      beta[i] = acc;
      mx = fmax(mx, fabs(acc));
    }
    if (mx > 0.0) {
      const double inv = 1.0 / mx;
#pragma unroll
      for (int i = 0; i <= M; ++i) {
        beta[i] *= inv;
        q[i] *= inv;
      }
      // Depth-first walk of the dyadic tree under node (log2parts, part).
      int level = log2parts, idx = part;
      for (;;) {
        const double w = ldexp(1.0, -level);
        const double a = idx * w;
        const double e = a + w;
        // Node coefficients: left part of a split at e, then the right part
        // of that at a / e.
        double bb[M + 1];
#pragma unroll
        for (int i = 0; i <= M; ++i) bb[i] = beta[i];
        if (e < 1.0) {
#pragma unroll
          for (int r = 1; r <= M; ++r)
#pragma unroll
            for (int i = M; i >= r; --i) bb[i] = fma(e, bb[i] - bb[i - 1], bb[i - 1]);
        }
        if (a > 0.0) {
          const double u = a / e;
#pragma unroll
          for (int r = 1; r <= M; ++r)
#pragma unroll
            for (int i = 0; i <= M - r; ++i) bb[i] = fma(u, bb[i + 1] - bb[i], bb[i]);
        }
        // Sign variations (zeros skipped), first / last nonzero signs.
        int var = 0;
        double first = 0.0, last = 0.0;
#pragma unroll
        for (int i = 0; i <= M; ++i) {
          const double x = bb[i];
          const bool nz = x != 0.0;
          var += (nz && last != 0.0 && ((x > 0.0) != (last > 0.0))) ? 1 : 0;
          first = (first == 0.0) ? x : first;
          last = nz ? x : last;
        }
        double root = -1.0;
        if (bb[0] == 0.0 && a > 0.0) {  // root exactly at the node's left end
          const double v = ext_mag2<N, K>(c, D, a * T);
          if (v > best_v) {
            best_v = v;
            best_t = a * T;
          }
        }
        bool descend = false;
        if (var == 1) {
          // Laguerre's method safeguarded by the bracket (bisection when a
          // step leaves it); lo keeps the sign of q just right of a.  Laguerre
          // models the other roots as one cluster, which is what the
          // high-multiplicity roots at rest-to-rest vertices look like, so it
          // converges in a few steps where Newton crawls.  Stops at the
          // rounding floor of the Horner evaluation.
          double lo = a, hi = e, x = 0.5 * (a + e);
          const bool pos_lo = first > 0.0;
          for (int it = 0; it < kExtRefineIters; ++it) {
            double fx = q[M], d1 = 0.0, d2 = 0.0, ab = fabs(q[M]);
#pragma unroll
            for (int j = M - 1; j >= 0; --j) {
              d2 = fma(d2, x, d1);
              d1 = fma(d1, x, fx);
              fx = fma(fx, x, q[j]);
              ab = fma(ab, x, fabs(q[j]));
            }
            if (fabs(fx) <= 32.0 * 2.220446049250313e-16 * ab) break;
            if ((fx > 0.0) == pos_lo) lo = x; else hi = x;
            const double G = d1 / fx;
            const double H = G * G - 2.0 * d2 / fx;
            const double rad = fmax((M - 1) * (M * H - G * G), 0.0);
            const double sq = sqrt(rad);
            const double den = G >= 0.0 ? G + sq : G - sq;
            double xn = den != 0.0 ? x - M / den : 0.5 * (lo + hi);
            if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
            const bool done = fabs(xn - x) <= 1.0e-12 || hi - lo <= 1.0e-12;
            x = xn;
            if (done) break;
          }
          root = x;
        } else if (var > 1) {
          if (level >= kExtMaxLevel) root = 0.5 * (a + e);  // unresolved cluster
          else descend = true;
        }
        if (root >= 0.0) {
          const double t = root * T;
          const double v = ext_mag2<N, K>(c, D, t);
          if (v > best_v) {
            best_v = v;
            best_t = t;
          }
        }
        if (descend) {
          ++level;
          idx *= 2;
          continue;
        }
        while (level > log2parts && (idx & 1)) {
          idx >>= 1;
          --level;
        }
        if (level == log2parts) break;
        ++idx;
      }
    }
  }
  val_s[tid] = best_v;
  time_s[tid] = best_t;
  __syncthreads();
  // Reduction in candidate order: segment ascending, part ascending; strict
  // '>' keeps the first maximum (Extremum::operator<, extremum.h:35-36;
  // linear_impl:474).  Extremum() starts at {0, 0, 0}.
  if (active && rem == 0) {
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
  }
}

template <int N>
static hipError_t launch_max_n(int K, int D, int S, int64_t B, int parts, int log2parts,
                               const double* coeffs, const double* times, double* tmax,
                               double* vmax, int32_t* smax, int stride, int offset,
                               const SoftCostArgs& soft, hipStream_t st) {
  const int tpb = kExtBlock / (S * parts);
  const dim3 grid(static_cast<unsigned>((B + tpb - 1) / tpb));
  const size_t lds = sizeof(double) * static_cast<size_t>(tpb) * S * (D * N + 1);
#define CALL(k)                                                                                \
  if (lds > 65536) {                                                                           \
    const hipError_t e = hipFuncSetAttribute(                                                  \
        reinterpret_cast<const void*>(max_magnitude_kernel<N, k>),                             \
        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));                     \
    if (e != hipSuccess) return e;                                                             \
  }                                                                                            \
  hipLaunchKernelGGL((max_magnitude_kernel<N, k>), grid, dim3(kExtBlock), lds, st, D, S, B,      \
                     parts, log2parts, coeffs, times, tmax, vmax, smax, stride, offset, soft)
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
                                int value_offset, const SoftCostArgs& soft, hipStream_t st) {
  if (S < 1 || S > kExtBlock || derivative < 0 || derivative > kMaxExtremaDerivative ||
      N - derivative - 1 <= 0)
    return hipErrorInvalidValue;
  int parts = kExtParts, log2parts = 3;
  while (S * parts > kExtBlock) {
    parts >>= 1;
    --log2parts;
  }
#define CALL(n)                                                                           \
  launch_max_n<n>(derivative, D, S, B, parts, log2parts, coeffs, times, max_time, max_value, \
                  max_segment, value_stride, value_offset, soft, st)
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

}  // namespace mtg
