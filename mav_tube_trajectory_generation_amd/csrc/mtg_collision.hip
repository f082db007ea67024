// mtg_collision.hip — collision cost of PolynomialOptimizationNonLinear over an
// occupancy map: getCostAndGradientCollision
// (nonlinear_impl:1609-1780), getCostAndGradientPotentialOctree (:1782-1917),
// the nearest-occupied-voxel search (findOccupiedVoxels :1920-2018,
// getDistanceOctree :2031-2043) and getCostPotential (:2660-2684).
//
// One 256-thread workgroup per trajectory runs the walk of
// mtg_collision_device.h (thread 0 steps through the samples, the workgroup
// searches the voxel box of every evaluated sample).  The coefficient
// gradient is finally mapped to the free derivatives of the plan through
// A_s^-1(T) (L = A^-1 M, :1650-1656).
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_collision_device.h"

namespace mtg {

template <int N>
__global__ __launch_bounds__(kCollBlock) void collision_cost_kernel(
    int S, int np, const double* __restrict__ tab, const int* __restrict__ free_map,
    const double* __restrict__ coeffs, const double* __restrict__ times,
    const float* __restrict__ occ, int nx, int ny, int nz, mtg_collision_params p,
    double* __restrict__ cost, int32_t* __restrict__ collision, double* __restrict__ grad_coeffs,
    double* __restrict__ grad_free) {
  constexpr int D = 3;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* c_s = sm;                 // S x D x N coefficients
  double* T_s = c_s + S * D * N;    // S
  double* g_s = T_s + S;            // S x D x N  dJ/dc
  double* scratch = g_s + S * D * N;
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.x;
  for (int i = tid; i < S * D * N; i += kCollBlock) {
    c_s[i] = coeffs[b * S * D * N + i];
    g_s[i] = 0.0;
  }
  for (int i = tid; i < S; i += kCollBlock) T_s[i] = times[b * S + i];
  __syncthreads();
  const bool grad = grad_coeffs || grad_free;
  double J;
  bool hit;
  collision_walk<N>(S, c_s, T_s, occ, nx, ny, nz, p, grad, g_s, scratch, &J, &hit);
  if (tid == 0) {
    if (cost) cost[b] = J;
    if (collision) collision[b] = hit ? 1 : 0;
  }
  // On a collision the gradient keeps the terms accumulated before it (the
  // reference's zeroing loop works on copies, :1773-1777).
  if (grad_coeffs)
    for (int i = tid; i < S * D * N; i += kCollBlock) grad_coeffs[b * S * D * N + i] = g_s[i];
  if (grad_free)
    for (int i = tid; i < D * np; i += kCollBlock)
      grad_free[b * D * np + i] = coll_grad_free<N>(S, D, np, tab + N * N, free_map, T_s, g_s, i);
}

size_t collision_lds_bytes(int N, int S) {
  return sizeof(double) * (2 * S * 3 * N + S + kCollScratch);
}

hipError_t launch_collision_cost(const PlanDev& pl, int64_t B, const double* coeffs,
                                 const double* times, const float* occ, int nx, int ny, int nz,
                                 const mtg_collision_params& p, double* cost, int32_t* coll,
                                 double* grad_coeffs, double* grad_free, hipStream_t st) {
  const size_t lds = collision_lds_bytes(pl.N, pl.S);
#define CALL(n)                                                                              \
  hipLaunchKernelGGL(collision_cost_kernel<n>, dim3(static_cast<unsigned>(B)), dim3(kCollBlock), \
                     lds, st, pl.S, pl.np, pl.tab, pl.free_map, coeffs, times, occ, nx, ny, nz, \
                     p, cost, coll, grad_coeffs, grad_free)
  switch (pl.N) {
    case 4: CALL(4); break;
    case 6: CALL(6); break;
    case 8: CALL(8); break;
    case 10: CALL(10); break;
    case 12: CALL(12); break;
    default: return hipErrorInvalidValue;
  }
#undef CALL
  return hipGetLastError();
}

}  // namespace mtg
