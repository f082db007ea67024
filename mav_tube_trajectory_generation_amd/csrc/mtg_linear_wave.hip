// mtg_linear_wave.hip — the standard-pattern linear solve (updateSegmentTimes
// + solveLinear + computeCost, linear_impl:277-379, 113-130; vertex pattern
// of createRandomVertices / makeStartOrEnd, vertex.cpp:27-82, 147-153) with
// the segment count S a compile-time constant: BASELINE config 2's kernel
// (N = 10, r = SNAP, D = 3, S = 2..16).  One 64-lane wavefront per
// trajectory running wave::Solver (mtg_wave_device.h); at one wave per SIMD
// the launch lasts one wave's instruction stream.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mtg_select_device.h"
#include "mtg_wave_device.h"

namespace mtg {
namespace wave {

// Trajectories (wavefronts) per workgroup; each wave owns its LDS region and
// runs independently (no workgroup barrier).  A/B builds: -DMTG_WAVE_WPB=n.
#ifndef MTG_WAVE_WPB
#define MTG_WAVE_WPB 1
#endif
constexpr int kWpb = MTG_WAVE_WPB;
static_assert(kWpb >= 1 && kWpb <= 4, "1 to 4 waves per workgroup");

// The problem count nb is an argument in the first 64 bytes (the first 56
// are preloaded into SGPRs; nb is the one scalar load before the first
// global load, as gridDim.x was in round 4), and kPrev (this launch carries
// the deferred selection's workgroup) a template parameter.  With the
// selection arguments appended, reading gridDim.x (a hidden argument after
// them, byte 128) and testing sel.prev_out in every workgroup measured
// 4.62 -> 4.99 us at C2, K = 200 (profiles/r05_kernarg_abl_c2.txt); moving nb
// into the preloaded bytes as well (free_vals after it) gave no gain
// (4.65 - 4.71 us, profiles/r05_kernarg_abl_c2_v2.txt).
template <int N, int R, int D, int S, bool kPrev>
__global__ __launch_bounds__(kWave * kWpb) void linear_wave_kernel(
    const double* __restrict__ tab, const double* __restrict__ fixed_vals,
    const double* __restrict__ times, double* __restrict__ coeffs, double* __restrict__ cost,
    double* __restrict__ free_vals, int32_t* __restrict__ status, int nb, SelectArgs sel) {
  using Sv = Solver<N, R, D, S>;
  using G = typename Sv::G;
  constexpr int MF = G::MF, MP = G::MP, NFIX = G::NFIX;
  __shared__ __attribute__((aligned(16))) double sm[kWpb * G::L_N];
  const int nblk = (nb + kWpb - 1) / kWpb;
  // The deferred selection (the previous step's costs) in one extra
  // workgroup after the solves: it runs beside them (about 1 us at
  // B = 1024 against a 3.4 us solve), so it costs no launch of its own.
  if (kPrev && static_cast<int>(blockIdx.x) == nblk) {
    if (threadIdx.x < kWave)
      select_reduce_block<kWave>(sel.prev_cost, sel.prev_count, sel.prev_start, sel.rank,
                                 sel.prev_out, nullptr, nullptr);
    return;
  }
  const int w = kWpb > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x / kWave) : 0;
  const int64_t b = xcd_problem(blockIdx.x, nblk) * kWpb + w;
  if (kWpb > 1 && b >= nb) return;
  Sv sv;
  sv.init(sm + w * G::L_N);
  const int lane = sv.lane;
  const double* fb = fixed_vals + b * D * NFIX;
  const double* tb = times + b * S;
  MTG_STAMP(0);
  // Inputs: each value loaded from HBM by one lane only (the four waves of a
  // CU share its L1 / TA path, which per-lane copies of the same values
  // saturated), all issued before the first use, then handed out through
  // LDS: d_f into the vertex table, H(1), the times.
  const double f0 = fb[lane < D * NFIX ? lane : D * NFIX - 1];
  double f1 = 0.0;
  if constexpr (D * NFIX > kWave) f1 = fb[lane + kWave < D * NFIX ? lane + kWave : D * NFIX - 1];
  const double t_own = tb[lane < S ? lane : S - 1];
  const double2 h_own = *reinterpret_cast<const double2*>(tab + 2 * (lane < N * N / 2 ? lane : 0));
  double* T = sv.aux();
  sv.store_constants(f0, f1, h_own);
  if (lane < S) T[lane] = t_own;
  lds_order();
  const bool bad = __any(lane < S && (!(t_own > 0.0) || !(t_own < 1e300)));
  MTG_STAMP(7);
  constexpr int64_t per = static_cast<int64_t>(S) * D * N;
  constexpr int NP = (S - 1) * MF;
  if (bad) {
    for (int i = lane; i < per; i += kWave) coeffs[b * per + i] = NAN;
    if (free_vals)
      for (int i = lane; i < D * NP; i += kWave) free_vals[b * D * NP + i] = NAN;
    if (cost && lane == 0) cost[b] = NAN;
    if (status && lane == 0) status[b] = MTG_TRAJ_BAD_TIME;
    return;
  }
  const bool not_spd = sv.solve(T);
  // The coefficients are staged in the chain slots (free after solve()) and
  // copied out with consecutive lanes on consecutive 16-byte pieces: three
  // stores over 19 cache lines instead of five over 95 (lane (s, d) writes
  // 80 bytes at an 80-byte stride).
  static_assert(2 * G::NSL * G::SLOT >= per, "coefficients fit the slots");
  double* stage = sv.slots;
#ifndef MTG_ABL_NOCOEF  // diagnostic ablation builds only (tools/gpu_r05_abl.sh)
  const double J = sv.coeff_cost(T, stage);
  lds_order();
  {
    copy_out16<kWave, per / 2>(reinterpret_cast<const double2*>(stage),
                               reinterpret_cast<double2*>(coeffs + b * per), lane);
  }
#else
  const double J = sv.dv[lane];
#endif
  if (lane == 0) {
    if (cost) cost[b] = J;
    if (status) status[b] = not_spd ? MTG_TRAJ_NOT_SPD : MTG_TRAJ_OK;
  }
  if (free_vals) {
    for (int i = lane; i < D * NP; i += kWave) {
      const int d = i / NP, p = i % NP;
      const int v = p / MF + 1, kk = p % MF + 1;
      free_vals[b * D * NP + i] = sv.dv[(v * D + d) * MP + kk];
    }
  }
  MTG_STAMP(6);
}

template <int S>
static hipError_t launch_wave_s(int64_t B, const SelectArgs& sel, const double* tab,
                                const double* df, const double* times, double* coeffs,
                                double* cost, double* free_vals, int32_t* status,
                                hipStream_t st) {
  const unsigned nblk = static_cast<unsigned>((B + kWpb - 1) / kWpb);
  if (sel.prev_out)
    hipLaunchKernelGGL((linear_wave_kernel<10, 4, 3, S, true>), dim3(nblk + 1),
                       dim3(kWave * kWpb), 0, st, tab, df, times, coeffs, cost, free_vals, status, static_cast<int>(B), sel);
  else
    hipLaunchKernelGGL((linear_wave_kernel<10, 4, 3, S, false>), dim3(nblk),
                       dim3(kWave * kWpb), 0, st, tab, df, times, coeffs, cost, free_vals, status, static_cast<int>(B), sel);
  return hipGetLastError();
}

}  // namespace wave

bool has_linear_wave(const PlanDev& pl) {
  return pl.std_pattern && pl.N == 10 && pl.r == 4 && pl.D == 3 && pl.S >= 2 && pl.S <= 16;
}

hipError_t launch_linear_solve_wave(const PlanDev& pl, int64_t B, const SelectArgs& sel,
                                    const double* df,
                                    const double* times, double* coeffs, double* cost,
                                    double* free_vals, int32_t* status, hipStream_t st) {
  switch (pl.S) {
#define MTG_WAVE_S(SS) \
  case SS: return wave::launch_wave_s<SS>(B, sel, pl.tab, df, times, coeffs, cost, free_vals, status, st);
    MTG_WAVE_S(2) MTG_WAVE_S(3) MTG_WAVE_S(4) MTG_WAVE_S(5) MTG_WAVE_S(6) MTG_WAVE_S(7)
    MTG_WAVE_S(8) MTG_WAVE_S(9) MTG_WAVE_S(10) MTG_WAVE_S(11) MTG_WAVE_S(12) MTG_WAVE_S(13)
    MTG_WAVE_S(14) MTG_WAVE_S(15) MTG_WAVE_S(16)
#undef MTG_WAVE_S
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg

#ifdef MTG_STAMPS
extern "C" int mtg_debug_stamps_wave(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mtg_stamps),
                             sizeof(unsigned long long) * n) == hipSuccess ? 0 : -3;
}
#endif
