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

// Near field of the map (mtg_coll_field): every voxel's seven box minima
// (collision_walk's m[0..6]) computed once per map.  A workgroup takes an
// 8 x 8 x 8 tile of voxels and stages the occupancy flags of the tile's
// box-extended window (8 + side + 1 voxels a side) in LDS as bytes; each
// thread then scans its voxel's box there in integer arithmetic (squared
// voxel offsets are small integers, so the minima are exact and equal the
// walk's double-precision ones).
constexpr int kFieldTile = 8;

__global__ __launch_bounds__(kFieldTile* kFieldTile* kFieldTile) void coll_field_kernel(
    const float* __restrict__ occ, int nx, int ny, int nz, int side,
    uint16_t* __restrict__ field) {
  extern __shared__ unsigned char flags[];
  const int lo = coll_box_lo(side), ext = side + 2;
  const int te = kFieldTile + ext - 1;  // window extent
  const int tiles_x = (nx + kFieldTile - 1) / kFieldTile;
  const int tiles_y = (ny + kFieldTile - 1) / kFieldTile;
  const int tile = blockIdx.x;
  const int x0 = (tile % tiles_x) * kFieldTile, y0 = (tile / tiles_x % tiles_y) * kFieldTile,
            z0 = tile / (tiles_x * tiles_y) * kFieldTile;
  const int wx = x0 + lo, wy = y0 + lo, wz = z0 + lo;  // window origin
  const int tid = threadIdx.x;
  for (int i = tid; i < te * te * te; i += blockDim.x) {
    const int x = wx + i % te, y = wy + (i / te) % te, z = wz + i / (te * te);
    const bool in = x >= 0 && y >= 0 && z >= 0 && x < nx && y < ny && z < nz;
    flags[i] = in && occ[(static_cast<int64_t>(z) * ny + y) * nx + x] >= 0.0f ? 1 : 0;
  }
  __syncthreads();
  const int tx = tid % kFieldTile, ty = tid / kFieldTile % kFieldTile,
            tz = tid / (kFieldTile * kFieldTile);
  const int vx = x0 + tx, vy = y0 + ty, vz = z0 + tz;
  if (vx >= nx || vy >= ny || vz >= nz) return;
  int m[7];
  for (int q = 0; q < 7; ++q) m[q] = 0x7FFFFFFF;
  for (int k = 0; k < ext; ++k) {
    const int az = lo + k;
    for (int j = 0; j < ext; ++j) {
      const int ay = lo + j;
      const unsigned char* row = flags + ((tz + k) * te + (ty + j)) * te + tx;
      for (int i = 0; i < ext; ++i) {
        if (!row[i]) continue;
        const int ax = lo + i;
        const int yz = ay * ay + az * az, xz = ax * ax + az * az, xy = ax * ax + ay * ay;
        m[0] = min(m[0], ax * ax + yz);
        m[1] = min(m[1], (ax + 1) * (ax + 1) + yz);  // v - e_x
        m[2] = min(m[2], (ax - 1) * (ax - 1) + yz);  // v + e_x
        m[3] = min(m[3], (ay + 1) * (ay + 1) + xz);
        m[4] = min(m[4], (ay - 1) * (ay - 1) + xz);
        m[5] = min(m[5], (az + 1) * (az + 1) + xy);
        m[6] = min(m[6], (az - 1) * (az - 1) + xy);
      }
    }
  }
  unsigned u[8];
  for (int q = 0; q < 7; ++q) u[q] = m[q] == 0x7FFFFFFF ? kFieldNone : static_cast<unsigned>(m[q]);
  u[7] = kFieldNone;
  *reinterpret_cast<uint4*>(field + ((static_cast<int64_t>(vz) * ny + vy) * nx + vx) *
                                        kFieldSlots) =
      make_uint4(u[0] | (u[1] << 16), u[2] | (u[3] << 16), u[4] | (u[5] << 16),
                 u[6] | (u[7] << 16));
}

bool coll_field_supported(int side) {
  // squared offsets up to 3 (side/2 + 2)^2 must stay below kFieldNone; the
  // LDS window (8 + side + 1)^3 bytes within 64 KB
  const int a = side / 2 + 2;
  const int te = kFieldTile + side + 1;
  return side >= 1 && 3 * a * a < static_cast<int>(kFieldNone) && te * te * te <= 65536;
}

hipError_t launch_coll_field(const float* occ, int nx, int ny, int nz, int side,
                             uint16_t* field, hipStream_t st) {
  if (!coll_field_supported(side)) return hipErrorInvalidValue;
  const int te = kFieldTile + side + 1;
  const size_t lds = static_cast<size_t>(te) * te * te;
  const int64_t tiles = static_cast<int64_t>((nx + kFieldTile - 1) / kFieldTile) *
                        ((ny + kFieldTile - 1) / kFieldTile) * ((nz + kFieldTile - 1) / kFieldTile);
  if (lds > 65536 - 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(coll_field_kernel, dim3(static_cast<unsigned>(tiles)),
                     dim3(kFieldTile * kFieldTile * kFieldTile), lds, st, occ, nx, ny, nz, side,
                     field);
  return hipGetLastError();
}

size_t collision_lds_bytes(int N, int S) {
  return sizeof(double) * (2 * S * 3 * N + S + coll_scratch_doubles(N));
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
