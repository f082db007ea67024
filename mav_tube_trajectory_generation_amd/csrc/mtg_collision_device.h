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

// is_valid_state (:1803-1811): within one voxel of the map bounds.
__device__ inline bool coll_valid_state(const double* pos, const mtg_collision_params& p) {
  const double res = p.map_resolution;
  return !(pos[0] < p.min_bound[0] + res || pos[0] > p.max_bound[0] - res ||
           pos[1] < p.min_bound[1] + res || pos[1] > p.max_bound[1] - res ||
           pos[2] < p.min_bound[2] + res || pos[2] > p.max_bound[2] - res);
}

// Scratch doubles of one walk (LDS, after c_s / T_s / g_s): control words,
// the chunk's evaluated voxels (for the workgroup box scans), the min
// reduction, and the chunk's gradient rows (t^0..t^(N-1), a[3], b[3] per
// sample).
__host__ __device__ constexpr int coll_scratch_doubles(int N) {
  return 8 + 2 * kWave + 7 * (kCollBlock / kWave) + kWave * (N + 6);
}

// Lane l's x (l wave-uniform).
__device__ inline double coll_readlane(double x, int l) {
  const unsigned long long v = static_cast<unsigned long long>(__double_as_longlong(x));
  const unsigned lo = static_cast<unsigned>(
      __builtin_amdgcn_readlane(static_cast<int>(static_cast<unsigned>(v)), l));
  const unsigned hi = static_cast<unsigned>(
      __builtin_amdgcn_readlane(static_cast<int>(static_cast<unsigned>(v >> 32)), l));
  return __longlong_as_double(
      static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}

// LDS written by some lanes of a wave and read by others after it.
__device__ inline void coll_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The walk over segments with coefficients c_s (S x 3 x N) and segment times
// T_s (LDS).  g_s (S x 3 x N, LDS, zeroed by the caller) receives dJ_c/dc
// when `grad`.  Called by every thread of the workgroup (blockDim.x = kWave
// with a near field, kCollBlock without); on return every thread holds J_c
// (0 on a collision) and the collision flag.
//
// Wave 0 takes the sample sequence in chunks of up to 64 samples of one
// segment, lane j holding sample j:
//   1. the times t0, t0 + dt, ... (the reference's repeated addition, a
//      64-step uniform chain), positions and velocities by Horner per lane,
//      the path length from the previous sample by a lane shuffle;
//   2. a uniform scan in sample order applies the reference's running sums
//      (the first sample, or one after time_sum went negative at a segment
//      end, only seeds; a sample is evaluated once dist_sum >= res; both sums
//      reset after it), marking the evaluated samples and their time_sum;
//   3. every evaluated sample's seven box minima at once: a near-field lookup
//      per lane (a serial scan for a voxel outside the grid), or without the
//      field one workgroup box scan per evaluated sample;
//   4. the potential per lane; the first colliding evaluated sample ends the
//      walk; J_c += c |v| time_sum over the evaluated samples before it, in
//      order, and with `grad` the eq. (14) terms, lane (k, n) of the
//      coefficient gradient adding sample after sample from the LDS rows.
// Every floating-point sum runs in the reference's order, so a chunked walk
// equals the sample-by-sample one bit for bit.
template <int N>
__device__ void collision_walk(int S, const double* c_s, const double* T_s, const float* occ,
                               int nx, int ny, int nz, const mtg_collision_params& p, bool grad,
                               double* g_s, double* scratch, double* J_out, bool* hit_out,
                               const uint16_t* field = nullptr) {
  constexpr int D = 3, RW = N + 6;
  static_assert(D * N <= kWave, "one lane per gradient coefficient");
  double* ctl = scratch;                           // [0] chunk, [1] boxes, [2] J, [3] hit
  int* evl = reinterpret_cast<int*>(scratch + 8);  // kWave x {vx, vy, vz, lane}
  double* red = scratch + 8 + 2 * kWave;
  double* rows = red + 7 * (kCollBlock / kWave);   // kWave x RW
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const bool w0 = tid < kWave;
  const double res = p.map_resolution, dt = p.coll_check_time_increment;
  auto dist = [&](double d2) {  // getDistanceOctree (:2031-2043); empty set: max double
    return d2 == HUGE_VAL ? 1.7976931348623157e308 * res : sqrt(d2) * res;
  };
  // Wave 0's walk state, uniform over its lanes (nonlinear_impl:1670-1768).
  int seg = 0;
  double t0 = 0.0, time_sum = -1.0, dist_sum = 0.0, J = 0.0;
  double prev[3] = {0.0, 0.0, 0.0};
  bool hit = false;
  for (;;) {
    int n_in = 0;
    double T = 0.0, t_end = 0.0, tj = 0.0, ts_me = 0.0;
    double pos[3] = {0.0, 0.0, 0.0}, vel[3] = {0.0, 0.0, 0.0};
    unsigned long long ev = 0;
    if (w0) {
      while (!hit && seg < S) {  // the next segment with samples left
        T = T_s[seg];
        double cur = t0;
        int k = 0;
        for (; k < kWave && cur < T; ++k) {
          if (lane == k) tj = cur;
          cur += dt;
        }
        n_in = k;
        t_end = cur;
        if (n_in > 0) break;
        time_sum += -dt + (T - cur);  // segment done: its first failing t
        ++seg;
        t0 = 0.0;
      }
      if (lane < n_in) {
        for (int d = 0; d < D; ++d) {
          const double* cd = c_s + (seg * D + d) * N;
          double x = cd[N - 1], v = (N - 1) * cd[N - 1];
          for (int n = N - 2; n >= 0; --n) x = fma(x, tj, cd[n]);
          for (int n = N - 2; n >= 1; --n) v = fma(v, tj, n * cd[n]);
          pos[d] = x;
          vel[d] = v;
        }
      }
      double dd = 0.0;
      for (int d = 0; d < D; ++d) {
        double q = __shfl(pos[d], (lane + kWave - 1) & (kWave - 1), kWave);
        if (lane == 0) q = prev[d];
        dd += (pos[d] - q) * (pos[d] - q);
      }
      const double sl = sqrt(dd);
      for (int j = 0; j < n_in; ++j) {
        const double s = coll_readlane(sl, j);
        if (time_sum < 0.0) {  // seeds the integrals only
          time_sum = 0.0;
          continue;
        }
        time_sum += dt;
        dist_sum += s;
        if (dist_sum < res) continue;
        ev |= 1ull << j;
        ts_me = lane == j ? time_sum : ts_me;
        dist_sum = 0.0;
        time_sum = 0.0;
      }
      if (!field) {  // the evaluated voxels inside the bounds, in order
        const bool e = (ev >> lane) & 1ull;
        const bool valid = e && coll_valid_state(pos, p);
        const unsigned long long vm = __ballot(valid);
        if (valid) {
          int* en = evl + 4 * __popcll(vm & ((1ull << lane) - 1ull));
          en[0] = static_cast<int>(pos[0] / res);
          en[1] = static_cast<int>(pos[1] / res);
          en[2] = static_cast<int>(pos[2] / res);
          en[3] = lane;
        }
        if (lane == 0) ctl[1] = __popcll(vm);
      }
      if (lane == 0) ctl[0] = n_in > 0 ? 1.0 : 0.0;
    }
    __syncthreads();
    if (ctl[0] == 0.0) break;
    double m[7];
    for (int q = 0; q < 7; ++q) m[q] = HUGE_VAL;
    if (!field) {
      const int n_box = static_cast<int>(ctl[1]);
      for (int e = 0; e < n_box; ++e) {
        const int* en = evl + 4 * e;
        double mm[7];
        for (int q = 0; q < 7; ++q) mm[q] = HUGE_VAL;
        coll_box_scan(occ, nx, ny, nz, en[0], en[1], en[2], p.box_side, tid, kCollBlock, mm);
        coll_wg_min7(mm, red);
        if (tid == en[3])
          for (int q = 0; q < 7; ++q) m[q] = mm[q];
      }
    }
    if (w0) {
      const bool e = (ev >> lane) & 1ull;
      bool valid = false, coll = false;
      double c = 0.0;
      if (e) {
        valid = coll_valid_state(pos, p);
        // Voxel of the sample: (position / res).cast<int>() truncates toward zero.
        const int vx = static_cast<int>(pos[0] / res), vy = static_cast<int>(pos[1] / res),
                  vz = static_cast<int>(pos[2] / res);
        if (field && valid && !coll_field_lookup(field, nx, ny, nz, vx, vy, vz, m))
          coll_box_scan(occ, nx, ny, nz, vx, vy, vz, p.box_side, 0, 1, m);
        // invalid states keep distance 0 (:1832-1839), i.e. collide
        c = coll_potential(valid ? dist(m[0]) : 0.0, p, &coll);
      }
      const unsigned long long cm = __ballot(e && coll);
      const unsigned long long live = cm ? ev & ((cm & (0ull - cm)) - 1ull) : ev;
      const double vn = sqrt(vel[0] * vel[0] + vel[1] * vel[1] + vel[2] * vel[2]);
      const double cv = c * vn;
      for (unsigned long long mm = live; mm; mm &= mm - 1ull) {
        const int j = __builtin_ctzll(mm);
        J += coll_readlane(cv, j) * coll_readlane(ts_me, j);
      }
      if (grad) {  // :1729-1750 (vn <= 1e-6 drops the gradient term)
        const bool gl = ((live >> lane) & 1ull) && vn > 1e-6;
        const unsigned long long gm = __ballot(gl);
        if (gm) {
          coll_wave_sync();  // the previous chunk's rows are read
          if (gl) {
            double* row = rows + lane * RW;
            double tn = 1.0;
            for (int n = 0; n < N; ++n) {
              row[n] = tn;
              tn *= tj;
            }
            for (int k = 0; k < D; ++k) {
              bool cl, cr;
              const double left = coll_potential(dist(m[1 + 2 * k]), p, &cl);
              const double right = coll_potential(dist(m[2 + 2 * k]), p, &cr);
              const double gp = (right - left) / (2.0 * res);
              row[N + k] = vn * ts_me * gp;
              row[N + 3 + k] = ts_me * c * vel[k] / vn;
            }
          }
          coll_wave_sync();
          if (lane < D * N) {  // eq. (14), lane (k, n), sample after sample
            const int k = lane / N, n = lane - k * N;
            double* gp = g_s + (seg * D + k) * N + n;
            double g = *gp;
            for (unsigned long long mm = gm; mm; mm &= mm - 1ull) {
              const double* row = rows + __builtin_ctzll(mm) * RW;
              const double a = row[N + k], bcoef = row[N + 3 + k];
              const double tn = row[n], tn1 = n > 0 ? n * row[n - 1] : 0.0;
              g += a * tn + bcoef * tn1;
            }
            *gp = g;
          }
        }
      }
      if (cm) {
        hit = true;
      } else {
        for (int d = 0; d < D; ++d) prev[d] = coll_readlane(pos[d], n_in - 1);
        // A segment ends at its first t >= T (a full chunk continues; one
        // whose times stopped growing is ended rather than walked forever).
        if (n_in < kWave || !(t_end > t0)) {
          time_sum += -dt + (T - t_end);
          ++seg;
          t0 = 0.0;
        } else {
          t0 = t_end;
        }
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    ctl[2] = hit ? 0.0 : J;
    ctl[3] = hit ? 1.0 : 0.0;
  }
  __syncthreads();
  *J_out = ctl[2];
  *hit_out = ctl[3] != 0.0;
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
