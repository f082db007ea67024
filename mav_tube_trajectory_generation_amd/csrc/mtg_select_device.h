// mtg_select_device.h — the selection step of the multi-GPU path (SURVEY.md
// 8e) fused into the epilogue of a solve kernel: every workgroup publishes
// the (cost, index) of the best trajectory it solved, and one small launch
// reduces those partials to the shard's (cost, global index, rank) triple,
// with the ordering of select_local_kernel (mtg_select.hip): NaN never wins,
// the lowest index wins ties, all +inf gives the shard's first index.
//
// A last-workgroup-done reduction (release fence + device-scope atomic
// counter in every workgroup) was measured first: on gfx950 the per-
// workgroup fence and same-address atomic serialise at ~40 ns per workgroup
// (24.6 us over the solve at 1,024 workgroups, 131 us at 3,121), far more
// than the second launch costs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

#include "mtg_internal.h"

namespace mtg {

// (cost, index) a beats b: smaller cost, or equal cost and lower index.
// NaN costs are mapped to +inf by the caller.
__device__ inline bool sel_better(double ca, int64_t ia, double cb, int64_t ib) {
  return ca < cb || (ca == cb && ia < ib);
}

// Wave-wide lexicographic minimum of (c, i); every lane receives it.
__device__ inline void sel_wave_min(double& c, int64_t& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double c2 = __shfl_xor(c, off, 64);
    const int64_t i2 = __shfl_xor(i, off, 64);
    if (sel_better(c2, i2, c, i)) {
      c = c2;
      i = i2;
    }
  }
}

// Called by all 64 threads of the first wave of every workgroup after the
// workgroup's costs are written: (c, i) is this lane's candidate (i < 0:
// none; NaN allowed), `block` the workgroup's partial slot.  Lane 0 writes
// the workgroup's best (cost, index) to the partial arrays; the reduction of
// the partials is a separate one-workgroup launch (select_partials_kernel,
// mtg_select.hip) on the same stream, so the kernel boundary orders the
// partials before it without any fence or atomic.
__device__ inline void select_partial(const SelectArgs& sel, double c, int64_t i, int64_t block) {
  if (c != c || i < 0) c = HUGE_VAL;
  if (i < 0) i = INT64_MAX;
  sel_wave_min(c, i);
  if ((threadIdx.x & 63) == 0) {
    sel.part_cost[block] = c;
    sel.part_idx[block] = i;
  }
}

// The shard's triple of costs c[0 .. count) (global indices start ..) by
// the NT threads of one workgroup: the deferred selection's extra workgroup
// (SelectArgs::prev_*), the rule of select_reduce_kernel.  Sixteen loads in
// flight per thread (a reduction of 8192 costs is four rounds of L2 latency
// at NT = 128); the waves combine through ws_c / ws_i (LDS, NT / 64 each).
template <int NT>
__device__ inline void select_reduce_block(const double* __restrict__ c, int64_t count,
                                           int64_t start, int rank, double* __restrict__ out,
                                           double* ws_c, int64_t* ws_i) {
  const int t = threadIdx.x;
  double bc = HUGE_VAL;
  int64_t bi = INT64_MAX;
  constexpr int kU = 16;
  for (int64_t k0 = t; k0 < count; k0 += NT * kU) {
    double pc[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t k = k0 + u * NT;
      pc[u] = k < count ? c[k] : HUGE_VAL;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t k = k0 + u * NT;
      const double v = pc[u] != pc[u] ? HUGE_VAL : pc[u];  // NaN never wins
      if (k < count && sel_better(v, k, bc, bi)) {
        bc = v;
        bi = k;
      }
    }
  }
  sel_wave_min(bc, bi);
  if constexpr (NT > 64) {
    if ((t & 63) == 0) {
      ws_c[t / 64] = bc;
      ws_i[t / 64] = bi;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NT / 64; ++q)
      if (sel_better(ws_c[q], ws_i[q], bc, bi)) {
        bc = ws_c[q];
        bi = ws_i[q];
      }
  }
  if (t == 0) {
    const bool empty = count <= 0;
    const int64_t at = (bi >= count || bi < 0) ? 0 : bi;  // all +inf: the first index
    out[0] = empty ? HUGE_VAL : bc;
    out[1] = empty ? -1.0 : static_cast<double>(at + start);
    out[2] = static_cast<double>(rank);
  }
}

}  // namespace mtg
