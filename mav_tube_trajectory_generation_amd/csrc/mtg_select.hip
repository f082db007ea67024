// mtg_select.hip — the selection step of the multi-GPU path (SURVEY.md §8e,
// BASELINE config 4: shards solve independently, the ranks all-gather their
// costs for selection).  Each rank reduces its shard to one (cost, global
// index, rank) triple with select_reduce_kernel; after the all-gather of the
// triples (RCCL over xGMI, 24 B per rank) select_global_kernel picks the
// winner.  One launch each, so the whole step stays a handful of launches
// that a HIP graph can hold.
//
// Ordering (the reference's selection is "lowest cost"): NaN never wins (as
// +inf), ties go to the lowest index, i.e. the first rank holding the minimum
// since shards are contiguous and in rank order.  An empty shard reports
// (+inf, -1, rank) and only wins when every shard is empty; when every cost
// is NaN or +inf the winner is the first triple (global index 0 of a
// single-process argmin).
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_internal.h"
#include "mtg_select_device.h"

namespace mtg {

constexpr int kSelBlock = 256;

// (cost, index) pairs c[0..n), idx[0..n) (idx == nullptr: index = position)
// to the shard's triple.  One workgroup: each thread scans a strided share
// with eight loads in flight, then a wave minimum by shuffles and one LDS
// step across the four waves.
__global__ __launch_bounds__(kSelBlock) void select_reduce_kernel(
    const double* __restrict__ c, const int64_t* __restrict__ idx, int64_t n, int64_t count,
    int64_t start, int rank, double* __restrict__ out) {
  __shared__ double ws_c[kSelBlock / 64];
  __shared__ int64_t ws_i[kSelBlock / 64];
  double bc = HUGE_VAL;
  int64_t bi = INT64_MAX;
  constexpr int kU = 8;
  for (int64_t k0 = threadIdx.x; k0 < n; k0 += kSelBlock * kU) {
    double pc[kU];
    int64_t pi[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t k = k0 + u * kSelBlock;
      pc[u] = k < n ? c[k] : HUGE_VAL;
      pi[u] = k < n ? (idx ? idx[k] : k) : INT64_MAX;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const double v = pc[u] != pc[u] ? HUGE_VAL : pc[u];  // NaN never wins
      if (sel_better(v, pi[u], bc, bi)) {
        bc = v;
        bi = pi[u];
      }
    }
  }
  sel_wave_min(bc, bi);
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    ws_c[w] = bc;
    ws_i[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
#pragma unroll
  for (int q = 1; q < kSelBlock / 64; ++q)
    if (sel_better(ws_c[q], ws_i[q], bc, bi)) {
      bc = ws_c[q];
      bi = ws_i[q];
    }
  const bool empty = count <= 0;
  const int64_t at = (bi >= count || bi < 0) ? 0 : bi;  // all +inf: the first index
  out[0] = empty ? HUGE_VAL : bc;
  out[1] = empty ? -1.0 : static_cast<double>(at + start);
  out[2] = static_cast<double>(rank);
}

__global__ void select_global_kernel(const double* __restrict__ triples, int world,
                                     double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  int w = 0;
  double best = HUGE_VAL;
  for (int r = 0; r < world; ++r) {
    double key = triples[3 * r];
    if (triples[3 * r + 1] < 0.0 || key != key) key = HUGE_VAL;
    if (key < best) {
      best = key;
      w = r;
    }
  }
  out[0] = triples[3 * w];
  out[1] = triples[3 * w + 1];
  out[2] = triples[3 * w + 2];
}

// Per-step global argmin of G steps' triples gathered from every rank
// (triples: world x G x 3, rank-major as all_gather_into_tensor lays them
// out): out[g] for g < n, the select_global rule per step.
__global__ void select_global_steps_kernel(const double* __restrict__ triples, int world, int G,
                                           int n, double* __restrict__ out) {
  const int g = threadIdx.x + blockIdx.x * blockDim.x;
  if (g >= n) return;
  int w = 0;
  double best = HUGE_VAL;
  for (int r = 0; r < world; ++r) {
    const double* t = triples + (static_cast<int64_t>(r) * G + g) * 3;
    double key = t[0];
    if (t[1] < 0.0 || key != key) key = HUGE_VAL;
    if (key < best) {
      best = key;
      w = r;
    }
  }
  const double* t = triples + (static_cast<int64_t>(w) * G + g) * 3;
  out[3 * g] = t[0];
  out[3 * g + 1] = t[1];
  out[3 * g + 2] = t[2];
}

hipError_t launch_select_global_steps(const double* triples, int world, int G, int n,
                                      double* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(select_global_steps_kernel, dim3((n + 63) / 64), dim3(64), 0, st, triples,
                     world, G, n, out);
  return hipGetLastError();
}

hipError_t launch_select_local(const double* costs, int64_t count, int64_t start, int rank,
                               double* out, hipStream_t st) {
  return launch_select_reduce(costs, nullptr, count, count, start, rank, out, st);
}

hipError_t launch_select_reduce(const double* cost, const int64_t* idx, int64_t n, int64_t count,
                                int64_t start, int rank, double* out, hipStream_t st) {
  hipLaunchKernelGGL(select_reduce_kernel, dim3(1), dim3(kSelBlock), 0, st, cost, idx,
                     n > 0 ? n : 0, count, start, rank, out);
  return hipGetLastError();
}

hipError_t launch_select_global(const double* triples, int world, double* out, hipStream_t st) {
  hipLaunchKernelGGL(select_global_kernel, dim3(1), dim3(64), 0, st, triples, world, out);
  return hipGetLastError();
}

}  // namespace mtg
