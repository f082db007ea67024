// mtg_free_device.h — helpers of the free-derivative objectives on the
// generic per-trajectory state (mtg_device.h), shared by mtg_free.hip and the
// collision objectives (mtg_coll_opt.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "mtg_device.h"

namespace mtg {

// LDS after the generic layout: [cbuf S*D*N (kSoft)] [gv (S+1)*M*D]
// [free-optimiser state 3*D*np] [time state 4*S (time_free_optimize)].
struct FreeLds {
  size_t cbuf, gv, opt, bytes;
};

__host__ __device__ inline FreeLds free_lds(int N, int S, int D, int np, bool soft) {
  const Layout lay = make_layout(N, S, D);
  FreeLds f;
  size_t o = (lay.bytes() + 15) / 16 * 16;
  f.cbuf = o;
  if (soft) o += sizeof(double) * S * D * N;
  f.gv = o;
  o += sizeof(double) * (S + 1) * (N / 2) * D;
  f.opt = o;
  o += sizeof(double) * 3 * D * (np > 0 ? np : 1);
  o += sizeof(double) * 4 * S;
  f.bytes = o;
  return f;
}

template <typename T>
__device__ inline T* lds_at(double* smem, size_t byte_offset) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(smem) + byte_offset);
}

// Loads d_f, d_p (free values into dv via free_map), times and powers.
// Returns true on an invalid segment time (wave-uniform).
template <int N>
__device__ bool free_setup(Traj<N>& t, const PlanDev& pl, const double* __restrict__ fixed_b,
                           const double* __restrict__ free_b, const double* __restrict__ times_b) {
  t.load_inputs(pl.tab, pl.slots, pl.fixed_map, times_b, fixed_b, pl.nf);
  if (free_b)
    for (int i = t.lane; i < t.D * pl.np; i += kWave)
      t.dv()[pl.free_map[i % pl.np] * t.D + i / pl.np] = free_b[i];
  __syncthreads();
  t.compute_powers();
  __syncthreads();
  return (t.flag()[0] & 1) != 0;
}

// gv[(v*M + k)*D + d] = (R d)_(v, k) for dimension d: two passes so each
// vertex row is written by one lane at a time (half 0 of segment v, then
// half 1 of segment v-1).
template <int N>
__device__ void free_rd(Traj<N>& t, double* gv) {
  constexpr int M = N / 2;
  const int S = t.S, D = t.D;
  for (int i = t.lane; i < (S + 1) * M * D; i += kWave) gv[i] = 0.0;
  __syncthreads();
  for (int h = 0; h < 2; ++h) {
    for (int item = t.lane; item < S * D; item += kWave) {
      const int s = item / D, d = item % D;
      double e[N];
#pragma unroll
      for (int j = 0; j < N; ++j) e[j] = t.dval(s + j / M, j % M, d);
#pragma unroll 1
      for (int kk = 0; kk < M; ++kk) {
        const int a = h * M + kk;
        double row = 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j)
          row = fma(t.tabH()[a * N + j] * t.pwr(s, 1 - 2 * t.r + kk + (j % M)), e[j], row);
        gv[((s + h) * M + kk) * D + d] += row;
      }
    }
    __syncthreads();
  }
}

}  // namespace mtg
