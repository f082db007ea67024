// mtg_select_device.h — the selection step of the multi-GPU path (SURVEY.md
// 8e) fused into the epilogue of a solve kernel: every workgroup publishes
// the (cost, index) of the best trajectory it solved, and the last workgroup
// to finish (a device-scope atomic counter) reduces those partials to the
// shard's (cost, global index, rank) triple, with the ordering of
// select_local_kernel (mtg_select.hip): NaN never wins, the lowest index wins
// ties, all +inf gives the shard's first index.  It replaces the separate
// single-workgroup launch that scanned the whole shard after the solve.
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

// Called by all 64 threads of every workgroup (one wave) after the
// workgroup's costs are written: (c, i) is this lane's candidate (i < 0:
// none; NaN allowed), `block` the workgroup's partial slot, `nblocks` the
// grid size.  The last workgroup writes sel.out = (cost, start + index, rank)
// and re-arms the counter.
__device__ inline void select_epilogue(const SelectArgs& sel, double c, int64_t i, int64_t block,
                                       int64_t nblocks, int64_t count) {
  __shared__ int last;
  if (c != c || i < 0) c = HUGE_VAL;
  if (i < 0) i = INT64_MAX;
  sel_wave_min(c, i);
  if (threadIdx.x == 0) {
    sel.part_cost[block] = c;
    sel.part_idx[block] = i;
    __threadfence();  // the partial is visible device-wide before the count
    const unsigned prev = atomicAdd(sel.counter, 1u);
    last = prev == static_cast<unsigned>(nblocks - 1) ? 1 : 0;
  }
  __syncthreads();
  if (!last) return;
  // Acquire side: the agent-scope fence invalidates this CU's vector L1, so
  // the plain loads below read the other workgroups' partials from L2.  They
  // are independent, so eight are issued before any is used (device-scope
  // atomic loads here were serialised by the compiler: ~1 us each).
  __threadfence();
  double bc = HUGE_VAL;
  int64_t bi = INT64_MAX;
  constexpr int kU = 8;
  for (int64_t k0 = threadIdx.x; k0 < nblocks; k0 += 64 * kU) {
    double pc[kU];
    int64_t pi[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t k = k0 + u * 64;
      pc[u] = k < nblocks ? sel.part_cost[k] : HUGE_VAL;
      pi[u] = k < nblocks ? sel.part_idx[k] : INT64_MAX;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (sel_better(pc[u], pi[u], bc, bi)) {
        bc = pc[u];
        bi = pi[u];
      }
  }
  sel_wave_min(bc, bi);
  if (threadIdx.x == 0) {
    const bool empty = count <= 0;
    const int64_t idx = (bi >= count || bi < 0) ? 0 : bi;  // all +inf: the first index
    sel.out[0] = empty ? HUGE_VAL : bc;
    sel.out[1] = empty ? -1.0 : static_cast<double>(idx + sel.start);
    sel.out[2] = static_cast<double>(sel.rank);
    *sel.counter = 0u;  // every workgroup has counted: re-arm for the next launch
  }
}

}  // namespace mtg
