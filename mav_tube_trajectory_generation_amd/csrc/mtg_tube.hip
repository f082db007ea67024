// mtg_tube.hip — tube QCQP kernels (placeholder until the batched IPM lands).
#include <hip/hip_runtime.h>

#include "mtg_internal.h"

namespace mtg {

size_t tube_lds_bytes(int N, int S) { return 0; }

hipError_t launch_tube_residuals(const TubeArgs&, const double*, double*, hipStream_t) {
  return hipErrorNotSupported;
}

hipError_t launch_tube_solve(const TubeArgs&, double, int, double*, double*, double*,
                             int32_t*, int32_t*, hipStream_t) {
  return hipErrorNotSupported;
}

}  // namespace mtg
