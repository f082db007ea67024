// mtg_select.hip — the selection step of the multi-GPU path (SURVEY.md §8e,
// BASELINE config 4: shards solve independently, the ranks all-gather their
// costs for selection).  Each rank reduces its shard to one (cost, global
// index, rank) triple with select_local_kernel; after the all-gather of the
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

namespace mtg {

constexpr int kSelBlock = 1024;

__global__ __launch_bounds__(kSelBlock) void select_local_kernel(const double* __restrict__ costs,
                                                                 int64_t count, int64_t start,
                                                                 int rank, double* __restrict__ out) {
  __shared__ double vs[kSelBlock];
  __shared__ int64_t is[kSelBlock];
  const int tid = threadIdx.x;
  double best = HUGE_VAL;
  int64_t bi = count > 0 ? 0 : -1;
  for (int64_t i = tid; i < count; i += kSelBlock) {
    double v = costs[i];
    if (v != v) v = HUGE_VAL;
    if (v < best || (v == best && i < bi)) {
      best = v;
      bi = i;
    }
  }
  if (bi < 0 && count > 0) bi = count;  // no element seen by this thread
  vs[tid] = best;
  is[tid] = (count > 0 && tid >= count) ? count : bi;
  __syncthreads();
  for (int w = kSelBlock / 2; w > 0; w >>= 1) {
    if (tid < w) {
      const double v = vs[tid + w];
      const int64_t j = is[tid + w];
      if (v < vs[tid] || (v == vs[tid] && j < is[tid])) {
        vs[tid] = v;
        is[tid] = j;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    const bool empty = count <= 0;
    // All +inf: the first element (a single-process argmin's answer).
    const int64_t idx = empty ? -1 : (is[0] >= count ? 0 : is[0]);
    out[0] = empty ? HUGE_VAL : vs[0];
    out[1] = empty ? -1.0 : static_cast<double>(idx + start);
    out[2] = static_cast<double>(rank);
  }
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

hipError_t launch_select_local(const double* costs, int64_t count, int64_t start, int rank,
                               double* out, hipStream_t st) {
  hipLaunchKernelGGL(select_local_kernel, dim3(1), dim3(kSelBlock), 0, st, costs, count, start,
                     rank, out);
  return hipGetLastError();
}

hipError_t launch_select_global(const double* triples, int world, double* out, hipStream_t st) {
  hipLaunchKernelGGL(select_global_kernel, dim3(1), dim3(64), 0, st, triples, world, out);
  return hipGetLastError();
}

}  // namespace mtg
