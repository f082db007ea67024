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

}  // namespace mtg
