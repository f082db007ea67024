// mtg_collision_device.h — the collision walk of getCostAndGradientCollision
// (nonlinear_impl:1609-1780) as a workgroup-wide device function, shared by
// collision_cost_kernel (mtg_collision.hip) and the collision objectives'
// walk kernel (mtg_coll_opt.hip).
//
// The reference reads a supereight octree (absent here; parity unpinned).  The
// map is a caller-supplied dense grid of occupancy log-odds (voxel occupied
// iff value >= 0, checkIfOccupied :2022-2027), voxel (x, y, z) at index
// (z ny + y) nx + x; voxels outside the grid are unallocated, i.e. free.
//
// Thread 0 walks the sample sequence exactly as the reference does (per
// segment t = 0, dt, ... < T_i by repeated addition; the first sample only
// seeds the running distance; a sample is evaluated once the path length
// since the last evaluation reaches map_resolution; time_sum carries over
// segment ends).  Every evaluated sample is one parallel search: the
// workgroup scans the box of voxels that overlaps the side^3 box around the
// sample's voxel (supereight's aabb_aabb_collision, inclusive half-plane
// test) and reduces the nearest occupied distance from the voxel and from its
// 6 axis neighbours (the central-difference gradient of the potential,
// :1850-1876, which reuses the centre's occupied set).  Thread 0 adds
// c |v| time_sum to J_c and, with `grad`, the eq. (14) terms to dJ/dc (per
// segment coefficient).  A collision (distance - robot_radius <= 0, or a
// position within one voxel of the map bounds, :1803-1811) ends the walk
// with J_c = 0; the coefficient gradient keeps what the walk accumulated
// before it, because the reference's zeroing loop (:1773-1777) iterates over
// copies of the gradient vectors and leaves them unchanged.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include <stdint.h>

#include "mtg_device.h"
#include "mtg_internal.h"

namespace mtg {

constexpr int kCollBlock = 256;

// getCostPotential (nonlinear_impl:2660-2684).
__device__ inline double coll_potential(double d, const mtg_collision_params& p, bool* coll) {
  d -= p.robot_radius;
  *coll = false;
  if (d <= 0.0) {
    *coll = true;
    return p.coll_pot_multiplier * (-d) + 0.5 * p.epsilon;
  }
  if (d <= p.epsilon) {
    const double e = d - p.epsilon;
    return 0.5 / p.epsilon * e * e;
  }
  return 0.0;
}

// The seven box minima reduced over the workgroup at once (one barrier
// pair); red holds 7 x (kCollBlock / kWave) doubles.
__device__ inline void coll_wg_min7(double (&m)[7], double* red) {
  constexpr int W = kCollBlock / kWave;
#pragma unroll
  for (int q = 0; q < 7; ++q)
    for (int off = 32; off > 0; off >>= 1) m[q] = fmin(m[q], __shfl_xor(m[q], off, kWave));
  const int w = threadIdx.x / kWave;
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0)
#pragma unroll
    for (int q = 0; q < 7; ++q) red[q * W + w] = m[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    double x = red[q * W];
    for (int i = 1; i < W; ++i) x = fmin(x, red[q * W + i]);
    m[q] = x;
  }
}

// LDS scratch of one walk: smp (10 doubles) + red (7 x kCollBlock / kWave).
constexpr int kCollScratch = 10 + 7 * (kCollBlock / kWave);

// The walk's box around voxel v: offsets a in [coll_box_lo(side),
// coll_box_lo(side) + side + 1] on every axis.
__host__ __device__ inline int coll_box_lo(int side) { return -(side / 2) - 1; }

// m[0..6] of voxel (vx, vy, vz) from the near field; false outside the grid.
__device__ inline bool coll_field_lookup(const uint16_t* __restrict__ field, int nx, int ny,
                                         int nz, int vx, int vy, int vz, double (&m)[7]) {
  if (vx < 0 || vy < 0 || vz < 0 || vx >= nx || vy >= ny || vz >= nz) return false;
  const uint4 raw = *reinterpret_cast<const uint4*>(
      field + ((static_cast<int64_t>(vz) * ny + vy) * nx + vx) * kFieldSlots);
  const unsigned w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    const unsigned u = (w[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
    m[q] = u == kFieldNone ? HUGE_VAL : static_cast<double>(u);
  }
  return true;
}

// The walk's box search for voxel (vx, vy, vz), voxels i = first, first +
// stride, ... of the box (one thread: first = 0, stride = 1); minima folded
// into m.
__device__ inline void coll_box_scan(const float* __restrict__ occ, int nx, int ny, int nz,
                                     int vx, int vy, int vz, int side, int first, int stride,
                                     double (&m)[7]) {
  const int lo = coll_box_lo(side), ext = side + 2;
  const int lo_x = vx + lo, lo_y = vy + lo, lo_z = vz + lo;
  const int nbox = ext * ext * ext;
  for (int i = first; i < nbox; i += stride) {
    const int x = lo_x + i % ext, y = lo_y + (i / ext) % ext, z = lo_z + i / (ext * ext);
    if (x < 0 || y < 0 || z < 0 || x >= nx || y >= ny || z >= nz) continue;
    if (!(occ[(static_cast<int64_t>(z) * ny + y) * nx + x] >= 0.0f)) continue;
    const double ax = x - vx, ay = y - vy, az = z - vz;
    m[0] = fmin(m[0], ax * ax + ay * ay + az * az);
    m[1] = fmin(m[1], (ax + 1) * (ax + 1) + ay * ay + az * az);  // v - e_x
    m[2] = fmin(m[2], (ax - 1) * (ax - 1) + ay * ay + az * az);  // v + e_x
    m[3] = fmin(m[3], ax * ax + (ay + 1) * (ay + 1) + az * az);
    m[4] = fmin(m[4], ax * ax + (ay - 1) * (ay - 1) + az * az);
    m[5] = fmin(m[5], ax * ax + ay * ay + (az + 1) * (az + 1));
    m[6] = fmin(m[6], ax * ax + ay * ay + (az - 1) * (az - 1));
  }
}

// Thread 0's walk state (nonlinear_impl:1670-1768).
struct CollWalk {
  int seg = 0;
  double t = 0.0, time_sum = -1.0, dist_sum = 0.0, J = 0.0;
  double prev[3] = {0.0, 0.0, 0.0};
  bool in_seg = false;

  // Advances to the next evaluated sample: smp = pos[3], vel[3], time_sum,
  // t, seg.  False when the walk is over.
  template <int N>
  __device__ bool next(int S, const double* c_s, const double* T_s,
                       const mtg_collision_params& p, double* smp) {
    constexpr int D = 3;
    const double res = p.map_resolution, dt = p.coll_check_time_increment;
    while (seg < S) {
      if (!in_seg) {
        t = 0.0;
        in_seg = true;
      } else {
        t += dt;
      }
      if (!(t < T_s[seg])) {  // segment done: time_sum += -dt + (T_i - t)
        time_sum += -dt + (T_s[seg] - t);
        ++seg;
        in_seg = false;
        continue;
      }
      double pos[3], vel[3];
      for (int d = 0; d < D; ++d) {
        const double* cd = c_s + (seg * D + d) * N;
        double x = cd[N - 1], v = (N - 1) * cd[N - 1];
        for (int n = N - 2; n >= 0; --n) x = fma(x, t, cd[n]);
        for (int n = N - 2; n >= 1; --n) v = fma(v, t, n * cd[n]);
        pos[d] = x;
        vel[d] = v;
      }
      if (time_sum < 0.0) {  // the first sample only seeds the integrals
        time_sum = 0.0;
        for (int d = 0; d < D; ++d) prev[d] = pos[d];
        continue;
      }
      time_sum += dt;
      double dd = 0.0;
      for (int d = 0; d < D; ++d) dd += (pos[d] - prev[d]) * (pos[d] - prev[d]);
      dist_sum += sqrt(dd);
      for (int d = 0; d < D; ++d) prev[d] = pos[d];
      if (dist_sum < res) continue;
      for (int d = 0; d < D; ++d) {
        smp[d] = pos[d];
        smp[3 + d] = vel[d];
      }
      smp[6] = time_sum;
      smp[7] = t;
      smp[8] = seg;
      return true;
    }
    return false;
  }

  // Consumes the evaluated sample smp with its box minima m (valid: inside
  // the map bounds): J_c and (grad) dJ_c/dc.  True on a collision.
  template <int N>
  __device__ bool take(const double* smp, bool valid, const double (&m)[7],
                       const mtg_collision_params& p, bool grad, double* g_s) {
    constexpr int D = 3;
    const double res = p.map_resolution;
    // getDistanceOctree (:2031-2043): min |voxel - v| times res (an empty
    // set gives max double); invalid states keep distance 0 (:1832-1839).
    auto dist = [&](double d2) {
      return d2 == HUGE_VAL ? 1.7976931348623157e308 * res : sqrt(d2) * res;
    };
    bool coll;
    const double c = coll_potential(valid ? dist(m[0]) : 0.0, p, &coll);
    if (coll) return true;
    const double ts = smp[6], tt = smp[7];
    const int s = static_cast<int>(smp[8]);
    const double* vel = smp + 3;
    const double vn = sqrt(vel[0] * vel[0] + vel[1] * vel[1] + vel[2] * vel[2]);
    J += c * vn * ts;
    if (grad && vn > 1e-6) {  // :1729-1750 (else the gradient term is dropped)
      double gp[3];
      for (int k = 0; k < D; ++k) {
        bool cl, cr;
        const double left = coll_potential(dist(m[1 + 2 * k]), p, &cl);
        const double right = coll_potential(dist(m[2 + 2 * k]), p, &cr);
        gp[k] = (right - left) / (2.0 * res);
      }
      // eq. (14): d/dc_n of vn ts c(pos) with pos = sum c_n t^n,
      // vel = sum n c_n t^(n-1).
      for (int k = 0; k < D; ++k) {
        double* g = g_s + (s * D + k) * N;
        const double a = vn * ts * gp[k], bcoef = ts * c * vel[k] / vn;
        double tn = 1.0, tn1 = 0.0;  // t^n, n t^(n-1)
        for (int n = 0; n < N; ++n) {
          g[n] += a * tn + bcoef * tn1;
          tn1 = (n + 1) * tn;
          tn *= tt;
        }
      }
    }
    dist_sum = 0.0;
    time_sum = 0.0;
    return false;
  }
};

// is_valid_state (:1803-1811): within one voxel of the map bounds.
__device__ inline bool coll_valid_state(const double* pos, const mtg_collision_params& p) {
  const double res = p.map_resolution;
  return !(pos[0] < p.min_bound[0] + res || pos[0] > p.max_bound[0] - res ||
           pos[1] < p.min_bound[1] + res || pos[1] > p.max_bound[1] - res ||
           pos[2] < p.min_bound[2] + res || pos[2] > p.max_bound[2] - res);
}

// The walk over segments with coefficients c_s (S x 3 x N) and segment times
// T_s (LDS).  g_s (S x 3 x N, LDS, zeroed by the caller) receives dJ_c/dc
// when `grad`.  Called by every thread of the workgroup (blockDim.x, a
// multiple of 64 up to kCollBlock); on return every thread holds J_c (0 on a
// collision) and the collision flag.  With a near field (mtg_coll_field)
// thread 0 walks alone and looks every sample's minima up (a serial box
// scan for a voxel outside the grid); without, the workgroup scans each
// sample's box in parallel.
template <int N>
__device__ void collision_walk(int S, const double* c_s, const double* T_s, const float* occ,
                               int nx, int ny, int nz, const mtg_collision_params& p, bool grad,
                               double* g_s, double* scratch, double* J_out, bool* hit_out,
                               const uint16_t* field = nullptr) {
  double* smp = scratch;       // pos[3], vel[3], time_sum, t, seg, flag
  double* red = scratch + 10;  // reduction scratch
  const int tid = threadIdx.x;
  const double res = p.map_resolution;
  CollWalk wk;
  if (field) {
    if (tid == 0) {
      bool hit = false;
      while (wk.next<N>(S, c_s, T_s, p, smp)) {
        const bool valid = coll_valid_state(smp, p);
        // Voxel of the sample: (position / res).cast<int>() truncates
        // toward zero.
        const int vx = static_cast<int>(smp[0] / res), vy = static_cast<int>(smp[1] / res),
                  vz = static_cast<int>(smp[2] / res);
        double m[7];
        for (int q = 0; q < 7; ++q) m[q] = HUGE_VAL;
        if (valid && !coll_field_lookup(field, nx, ny, nz, vx, vy, vz, m))
          coll_box_scan(occ, nx, ny, nz, vx, vy, vz, p.box_side, 0, 1, m);
        if (wk.take<N>(smp, valid, m, p, grad, g_s)) {
          hit = true;
          break;
        }
      }
      smp[9] = hit ? -1.0 : 0.0;
      smp[6] = hit ? 0.0 : wk.J;
    }
    __syncthreads();
    *J_out = smp[6];
    *hit_out = smp[9] < 0.0;
    __syncthreads();
    return;
  }
  for (;;) {
    if (tid == 0) smp[9] = wk.next<N>(S, c_s, T_s, p, smp) ? 1.0 : 0.0;
    __syncthreads();
    if (smp[9] == 0.0) break;
    const bool valid = coll_valid_state(smp, p);
    const int vx = static_cast<int>(smp[0] / res), vy = static_cast<int>(smp[1] / res),
              vz = static_cast<int>(smp[2] / res);
    double m[7];
    for (int q = 0; q < 7; ++q) m[q] = HUGE_VAL;
    if (valid) {
      coll_box_scan(occ, nx, ny, nz, vx, vy, vz, p.box_side, tid, kCollBlock, m);
      coll_wg_min7(m, red);
    }
    if (tid == 0 && wk.take<N>(smp, valid, m, p, grad, g_s)) smp[9] = -1.0;  // collision: stop
    __syncthreads();
    if (smp[9] < 0.0) break;
  }
  __syncthreads();
  const bool hit = smp[9] < 0.0;
  if (tid == 0) smp[6] = hit ? 0.0 : wk.J;
  __syncthreads();
  *J_out = smp[6];
  *hit_out = hit;
  __syncthreads();
}

// dJ/d(vertex v, derivative j) of dimension k = sum over the segments s in
// {v-1, v} of A_s^-1(T_s)[n][(v - s) M + j] dJ/dc_s[n] (L = A^-1 M restricted
// to the free columns, nonlinear_impl:1650-1656), A_s^-1(T) =
// D_T^-1 A(1)^-1 S_T.  Free index i of the D x np layout.
template <int N>
__device__ inline double coll_grad_free(int S, int D, int np, const double* __restrict__ ai,
                                        const int* __restrict__ free_map, const double* T_s,
                                        const double* g_s, int i) {
  constexpr int M = N / 2;
  const int k = i / np, slot = free_map[i % np];
  const int v = slot / M, j = slot % M;
  double acc = 0.0;
  for (int h = 0; h < 2; ++h) {
    const int s = v - h;  // h = 0: start vertex of segment v; 1: end of v-1
    if (s < 0 || s >= S) continue;
    const double T = T_s[s];
    double tj = 1.0;
    for (int q = 0; q < j; ++q) tj *= T;
    double tinv = 1.0;
    const double* g = g_s + (s * D + k) * N;
    for (int n = 0; n < N; ++n) {
      acc += tinv * ai[n * N + h * M + j] * tj * g[n];
      tinv /= T;
    }
  }
  return acc;
}

}  // namespace mtg
