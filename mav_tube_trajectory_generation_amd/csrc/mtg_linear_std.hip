// mtg_linear_std.hip — batched linear solve (updateSegmentTimes +
// solveLinear + computeCost, linear_impl:277-379, 113-130) for the standard
// vertex pattern: start and end vertex fully fixed, intermediate vertices
// position only (createRandomVertices / makeStartOrEnd, vertex.cpp:27-82,
// 147-153; BASELINE configs 1, 2, 4 and 5).  One 64-lane workgroup per
// trajectory running stdp::Solver (mtg_std_device.h).  Other patterns run the
// generic kernel (mtg_kernels.hip).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>

#include "mtg_std_device.h"

namespace mtg {

size_t linear_std_lds_bytes(int N, int S, int D) {
  return sizeof(double) * static_cast<size_t>(stdp::layout(N, S, D).n);
}

template <int N, int R, int D>
__global__ __launch_bounds__(kWave) void linear_std_kernel(
    int S, const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    const double* __restrict__ times, double* __restrict__ coeffs, double* __restrict__ cost,
    double* __restrict__ free_vals, int32_t* __restrict__ status) {
  using Sv = stdp::Solver<N, R, D>;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int64_t b = blockIdx.x;
  MTG_STAMP(0);
  // Inputs: times, fixed values and the lane's two rows of H(1) are all
  // issued before the first use.
  Sv sv;
  sv.init(S, smem, nullptr);
  const int lane = sv.lane, nf = sv.nf;
  const double* tb = times + b * S;
  const double* fb = fixed_vals + b * D * nf;
  // Fixed values first, then the times, then the table rows: loads retire in
  // issue order, so the fixed values are stored to LDS while the times are
  // still in flight, and the powers wait only for the times.
  // Unconditional loads (clamped lanes re-read a valid element), so the
  // wait before the fixed-value stores covers the first load only.
  const double f_l = fb[lane < D * nf ? lane : D * nf - 1];
  const double t_raw = tb[lane < S ? lane : S - 1];
  const double t_l = lane < S ? t_raw : 1.0;
  sv.load_first_rows(tab);
  sv.clear_mid_terms();
  if (lane < D * nf) sv.put_fixed(lane, f_l);
  for (int i = lane + kWave; i < D * nf; i += kWave) sv.put_fixed(i, fb[i]);
  bool bad = lane < S ? sv.powers(lane, t_l) : false;
  for (int s = lane + kWave; s < S; s += kWave) bad = sv.powers(s, tb[s]) || bad;
  MTG_STAMP(7);
  const bool bad_time = __any(bad);
  __syncthreads();
  MTG_STAMP(1);

  const int64_t per = static_cast<int64_t>(S) * D * N;
  if (bad_time) {
    for (int i = lane; i < per; i += kWave) coeffs[b * per + i] = NAN;
    if (free_vals) {
      const int64_t nfv = static_cast<int64_t>(D) * (S - 1) * Sv::MF;
      for (int i = lane; i < nfv; i += kWave) free_vals[b * nfv + i] = NAN;
    }
    if (cost && lane == 0) cost[b] = NAN;
    if (status && lane == 0) status[b] = MTG_TRAJ_BAD_TIME;
    return;
  }
  sv.assemble(tab);
  __syncthreads();
  MTG_STAMP(2);
  const bool not_spd = sv.solve();
  const double J = sv.coeff_cost(coeffs + b * per);
  if (cost && lane == 0) cost[b] = J;
  if (free_vals) {
    const int np = (S - 1) * Sv::MF;
    for (int i = lane; i < D * np; i += kWave) {
      const int d = i / np, p = i % np;
      const int v = p / Sv::MF + 1, kk = p % Sv::MF + 1;
      free_vals[b * D * np + i] = sv.dv()[(v * D + d) * Sv::MP + kk];
    }
  }
  if (status && lane == 0) status[b] = not_spd ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK;
  MTG_STAMP(6);
}

template <int N, int R, int D>
static hipError_t launch_std_nrd(int S, int64_t B, const double* tab, const double* df,
                                 const double* times, double* coeffs, double* cost,
                                 double* free_vals, int32_t* status, hipStream_t st) {
  const size_t lds = linear_std_lds_bytes(N, S, D);
  hipLaunchKernelGGL((linear_std_kernel<N, R, D>), dim3(static_cast<unsigned>(B)), dim3(kWave),
                     lds, st, S, tab, df, times, coeffs, cost, free_vals, status);
  return hipGetLastError();
}

template <int N, int R>
static hipError_t launch_std_nr(int D, int S, int64_t B, const double* tab, const double* df,
                                const double* times, double* coeffs, double* cost,
                                double* free_vals, int32_t* status, hipStream_t st) {
  switch (D) {
    case 1: return launch_std_nrd<N, R, 1>(S, B, tab, df, times, coeffs, cost, free_vals, status, st);
    case 2: return launch_std_nrd<N, R, 2>(S, B, tab, df, times, coeffs, cost, free_vals, status, st);
    case 3: return launch_std_nrd<N, R, 3>(S, B, tab, df, times, coeffs, cost, free_vals, status, st);
    case 4: return launch_std_nrd<N, R, 4>(S, B, tab, df, times, coeffs, cost, free_vals, status, st);
    default: return hipErrorInvalidValue;
  }
}

template <int N>
static hipError_t launch_std_n(int r, int D, int S, int64_t B, const double* tab,
                               const double* df, const double* times, double* coeffs,
                               double* cost, double* free_vals, int32_t* status,
                               hipStream_t st) {
#define MTG_STD_R(RR)                                                                  \
  case RR:                                                                            \
    if constexpr (RR < N / 2)                                                         \
      return launch_std_nr<N, RR>(D, S, B, tab, df, times, coeffs, cost, free_vals,   \
                                  status, st);                                        \
    return hipErrorInvalidValue;
  switch (r) {
    MTG_STD_R(0)
    MTG_STD_R(1)
    MTG_STD_R(2)
    MTG_STD_R(3)
    MTG_STD_R(4)
    MTG_STD_R(5)
    default: return hipErrorInvalidValue;
  }
#undef MTG_STD_R
}

// MTG_STD_RUNTIME_S=1 (diagnostics): the runtime-S kernel below also where
// the compile-time-S kernel (mtg_linear_wave.hip) exists, for A/B runs.
static bool runtime_s_forced() {
  static const bool forced = [] {
    const char* e = std::getenv("MTG_STD_RUNTIME_S");
    return e && e[0] == '1';
  }();
  return forced;
}

hipError_t launch_linear_solve_std(const PlanDev& pl, int64_t B, const double* df,
                                   const double* times, double* coeffs, double* cost,
                                   double* free_vals, int32_t* status, hipStream_t st,
                                   const SelectArgs& sel) {
  // the wave kernel reduces a deferred selection in an extra workgroup; the
  // runtime-S kernel takes it as a launch of its own first
  if (has_linear_wave(pl) && !runtime_s_forced())
    return launch_linear_solve_wave(pl, B, sel, df, times, coeffs, cost, free_vals, status, st);
  if (sel.prev_out) {
    const hipError_t e = launch_select_local(sel.prev_cost, sel.prev_count, sel.prev_start,
                                             sel.rank, sel.prev_out, st);
    if (e != hipSuccess) return e;
  }
  switch (pl.N) {
    case 4: return launch_std_n<4>(pl.r, pl.D, pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 6: return launch_std_n<6>(pl.r, pl.D, pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 8: return launch_std_n<8>(pl.r, pl.D, pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 10: return launch_std_n<10>(pl.r, pl.D, pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    case 12: return launch_std_n<12>(pl.r, pl.D, pl.S, B, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg

#ifdef MTG_STAMPS
// Each HIP translation unit is its own code object: this kernel's stamps.
extern "C" int mtg_debug_stamps_std(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mtg_stamps),
                             sizeof(unsigned long long) * n) == hipSuccess ? 0 : -3;
}
#endif
