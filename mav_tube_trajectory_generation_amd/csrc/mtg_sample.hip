// mtg_sample.hip — batched trajectory sampling (Trajectory::evaluateRange,
// reference src/trajectory.cpp:74-134; the [t, p, v, a, j, s] rows of
// printMatlabSampledTrajectory, nonlinear_impl:2907-3003).  SURVEY.md §8f
// rank 3.
//
// One workgroup = 1024 consecutive samples of one trajectory (4 per lane).  The
// trajectory's coefficients and segment times are staged in LDS once; each
// lane locates its segment by the reference's rule (advance while the time
// in the segment exceeds the segment time), evaluates derivatives
// 0..max_derivative of every dimension by Horner's rule, and writes them
// channel-major (samples[b][ch][k], ch = derivative * D + d) so every store
// instruction is coalesced.  The kernel is HBM-write bound.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_internal.h"

namespace mtg {

constexpr int kSampleBlock = 256;
constexpr int kSamplesPerLane = 4;  // amortises the per-workgroup staging
constexpr int kScaledMax = 4096;    // doubles of pre-scaled coefficients in LDS
typedef double v2d __attribute__((ext_vector_type(2)));  // 16-byte non-temporal stores

// base(n, i) = i! / (i-n)! (polynomial.cpp:145-161), i >= n.
__device__ inline double falling_f(int n, int i) {
  double p = 1.0;
  for (int m = 0; m < n; ++m) p *= static_cast<double>(i - m);
  return p;
}

template <int N>
__global__ __launch_bounds__(kSampleBlock) void sample_kernel(
    int D, int S, const double* __restrict__ coeffs, const double* __restrict__ times,
    double t_start, double t_end_in, double dt, int n_max, int max_deriv,
    double* __restrict__ samples, double* __restrict__ sample_times,
    int32_t* __restrict__ n_samples) {
  // Dynamic LDS sized to this launch (small footprint -> full occupancy):
  // coefficients, segment times, base table, and the pre-scaled table
  // base(dv, j) * c[seg][d][j] ([seg][dv][d][j]) when it fits, with which
  // Horner needs one FMA per term.
  extern __shared__ double dyn[];
  double* c_s = dyn;
  double* T_s = c_s + S * D * N;
  double* base_s = T_s + S;
  double* cs_s = base_s + N * N;
  __shared__ double seg0_s[2];  // start segment's accumulated start, time in it
  __shared__ int i0_s;
  __shared__ int cnt_s;
  const int64_t b = blockIdx.y;
  const int tid = threadIdx.x;
  const int per = S * D * N;
  for (int i = tid; i < per; i += kSampleBlock) c_s[i] = coeffs[b * per + i];
  for (int i = tid; i < S; i += kSampleBlock) T_s[i] = times[b * S + i];
  for (int i = tid; i < N * N; i += kSampleBlock) {
    const int n = i / N, j = i % N;
    base_s[i] = j >= n ? falling_f(n, j) : 0.0;
  }
  __syncthreads();
  const int nK = max_deriv + 1;
  const bool scaled = S * nK * D * N <= kScaledMax;
  if (scaled) {
    for (int i = tid; i < S * nK * D * N; i += kSampleBlock) {
      const int j = i % N, d = (i / N) % D, dv = (i / (N * D)) % nK, seg = i / (N * D * nK);
      cs_s[i] = base_s[dv * N + j] * c_s[(seg * D + d) * N + j];
    }
  }
  if (tid == 0) {
    cnt_s = 0;
    // Start segment: first i with accumulated end > t_start (:88-103).
    double acc = 0.0;
    int i = 0;
    for (i = 0; i < S; ++i) {
      acc += T_s[i];
      if (acc > t_start) break;
    }
    if (t_start > acc || i >= S) {
      i0_s = -1;
    } else {
      acc -= T_s[i];
      i0_s = i;
      seg0_s[0] = acc;            // accumulated_time of the first sample
      seg0_s[1] = t_start - acc;  // time_in_segment of the first sample
    }
  }
  __syncthreads();
  const int i0 = i0_s;
  double t_end = t_end_in;
  if (t_end < 0.0) {  // whole trajectory
    t_end = 0.0;
    for (int i = 0; i < S; ++i) t_end += T_s[i];
  }
  const int nch = (max_deriv + 1) * D;
  const int64_t out0 = b * static_cast<int64_t>(nch) * n_max;
  int nvalid = 0;
  // Sample k's segment and time in it by the reference's rule (the valid
  // samples form a prefix of 0 .. n_max-1).
  auto locate = [&](int k, int* seg_o, double* tin_o, double* acc_o) {
    bool valid = false;
    int seg = 0;
    double tin = 0.0, acc = 0.0;
    if (i0 >= 0 && k < n_max) {
      acc = seg0_s[0] + static_cast<double>(k) * dt;
      tin = seg0_s[1] + static_cast<double>(k) * dt;
      seg = i0;
      while (seg < S && tin > T_s[seg]) {
        tin -= T_s[seg];
        ++seg;
      }
      valid = acc < t_end && seg < S;
    }
    *seg_o = seg;
    *tin_o = tin;
    *acc_o = acc;
    return valid;
  };
  if (scaled && (n_max & 1) == 0) {
    // Two consecutive samples per lane and 16-byte stores: each store
    // instruction writes 1 KB contiguous (round 5; the 8-byte stores below
    // write 512 B).  Rows start at even sample offsets (n_max even).
    for (int rep = 0; rep < kSamplesPerLane / 2; ++rep) {
      const int k = blockIdx.x * kSamplesPerLane * kSampleBlock + rep * 2 * kSampleBlock + 2 * tid;
      int sg0, sg1;
      double tn0, tn1, ac0, ac1;
      const bool v0 = locate(k, &sg0, &tn0, &ac0);
      const bool v1 = locate(k + 1, &sg1, &tn1, &ac1);
      if (v0) {
        const double* cs0 = cs_s + sg0 * nK * D * N;
        const double* cs1 = cs_s + (v1 ? sg1 : sg0) * nK * D * N;
        double* out = samples + out0 + k;
#pragma unroll
        for (int dv = 0; dv < N; ++dv) {
          if (dv >= nK) break;
#pragma unroll
          for (int d = 0; d < kMaxD; ++d) {
            if (d >= D) break;
            const double* c0 = cs0 + (dv * D + d) * N;
            const double* c1 = cs1 + (dv * D + d) * N;
            double a = c0[N - 1], c = c1[N - 1];
#pragma unroll
            for (int j = N - 2; j >= dv; --j) {
              a = fma(a, tn0, c0[j]);
              c = fma(c, tn1, c1[j]);
            }
            double* o = out + static_cast<int64_t>(dv * D + d) * n_max;
            if (v1)  // streamed once: non-temporal stores
              __builtin_nontemporal_store(v2d{a, c}, reinterpret_cast<v2d*>(o));
            else
              __builtin_nontemporal_store(a, o);
          }
        }
        if (sample_times) {
          double* o = sample_times + b * static_cast<int64_t>(n_max) + k;
          if (v1)
            __builtin_nontemporal_store(v2d{ac0, ac1}, reinterpret_cast<v2d*>(o));
          else
            __builtin_nontemporal_store(ac0, o);
        }
      }
      nvalid += (v0 ? 1 : 0) + (v1 ? 1 : 0);
    }
  } else
  for (int rep = 0; rep < kSamplesPerLane; ++rep) {
    const int k = (blockIdx.x * kSamplesPerLane + rep) * kSampleBlock + tid;
    // Sample k exists iff acc0 + k dt < t_end and its segment stays below S
    // (the reference stops at the first sample that runs off the last
    // segment); the valid samples are a prefix.
    bool valid = false;
    int seg = 0;
    double tin = 0.0, acc = 0.0;
    if (i0 >= 0 && k < n_max) {
      acc = seg0_s[0] + static_cast<double>(k) * dt;
      tin = seg0_s[1] + static_cast<double>(k) * dt;
      seg = i0;
      while (seg < S && tin > T_s[seg]) {
        tin -= T_s[seg];
        ++seg;
      }
      valid = acc < t_end && seg < S;
    }
    if (valid && scaled) {
      // Derivative and dimension loops unrolled with compile-time Horner
      // lengths (N - dv terms); runtime bounds only break out.
      const double* cs = cs_s + seg * nK * D * N;
      double* out = samples + out0 + k;
#pragma unroll
      for (int dv = 0; dv < N; ++dv) {
        if (dv >= nK) break;
#pragma unroll
        for (int d = 0; d < kMaxD; ++d) {
          if (d >= D) break;
          const double* cd = cs + (dv * D + d) * N;
          double v = cd[N - 1];
#pragma unroll
          for (int j = N - 2; j >= dv; --j) v = fma(v, tin, cd[j]);
          // streamed once: non-temporal stores
          __builtin_nontemporal_store(v, out + static_cast<int64_t>(dv * D + d) * n_max);
        }
      }
      if (sample_times)
        __builtin_nontemporal_store(acc, sample_times + b * static_cast<int64_t>(n_max) + k);
    } else if (valid) {
      const double* c = c_s + seg * D * N;
      for (int dv = 0; dv <= max_deriv; ++dv) {
        const double* bs = base_s + dv * N;
        for (int d = 0; d < D; ++d) {
          const double* cd = c + d * N;
          double v = bs[N - 1] * cd[N - 1];
#pragma unroll
          for (int j = N - 2; j >= 0; --j)
            if (j >= dv) v = fma(v, tin, bs[j] * cd[j]);
          samples[out0 + static_cast<int64_t>(dv * D + d) * n_max + k] = v;
        }
      }
      if (sample_times) sample_times[b * static_cast<int64_t>(n_max) + k] = acc;
    }
    nvalid += valid ? 1 : 0;
  }
  // Count: the valid samples are a prefix of 0..n_max-1, so exactly one
  // workgroup sees the end of the prefix (or holds sample n_max-1 with all
  // valid, or is workgroup 0 with none valid) and writes the count; no
  // zero-initialisation or global atomics needed.
  if (n_samples) {
    for (int off = 32; off > 0; off >>= 1) nvalid += __shfl_xor(nvalid, off, 64);
    if ((tid & 63) == 0 && nvalid) atomicAdd(&cnt_s, nvalid);
    __syncthreads();
    if (tid == 0) {
      const int k0 = blockIdx.x * kSamplesPerLane * kSampleBlock;
      const int kend = min(k0 + kSamplesPerLane * kSampleBlock, n_max);
      const int cnt = cnt_s;
      // Is sample k0-1 (last of the previous workgroup) valid?
      bool prev_valid = false;
      if (k0 > 0 && i0 >= 0) {
        const int k = k0 - 1;
        const double acc = seg0_s[0] + static_cast<double>(k) * dt;
        double tin = seg0_s[1] + static_cast<double>(k) * dt;
        int seg = i0;
        while (seg < S && tin > T_s[seg]) {
          tin -= T_s[seg];
          ++seg;
        }
        prev_valid = acc < t_end && seg < S;
      }
      if (cnt < kend - k0) {
        if (cnt > 0 || k0 == 0 || prev_valid) n_samples[b] = k0 + cnt;
      } else if (kend == n_max) {
        n_samples[b] = n_max;
      }
    }
  }
}

template <int N>
static hipError_t launch_sample_n(int D, int S, int64_t B, const double* coeffs,
                                  const double* times, double t_start, double t_end,
                                  double dt, int n_max, int max_deriv, double* samples,
                                  double* sample_times, int32_t* n_samples, hipStream_t st) {
  const int per_block = kSampleBlock * kSamplesPerLane;
  const dim3 grid(static_cast<unsigned>((n_max + per_block - 1) / per_block),
                  static_cast<unsigned>(B));
  const int nK = max_deriv + 1;
  const int scaled = S * nK * D * N <= kScaledMax ? S * nK * D * N : 0;
  const size_t bytes = sizeof(double) * (S * D * N + S + N * N + scaled);
  hipLaunchKernelGGL(sample_kernel<N>, grid, dim3(kSampleBlock), bytes, st, D, S, coeffs, times,
                     t_start, t_end, dt, n_max, max_deriv, samples, sample_times, n_samples);
  return hipGetLastError();
}

hipError_t launch_sample(int N, int D, int S, int64_t B, const double* coeffs,
                         const double* times, double t_start, double t_end, double dt,
                         int n_max, int max_deriv, double* samples, double* sample_times,
                         int32_t* n_samples, hipStream_t st) {
#define CALL(n)                                                                          \
  launch_sample_n<n>(D, S, B, coeffs, times, t_start, t_end, dt, n_max, max_deriv, samples, \
                     sample_times, n_samples, st)
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
