// mtg_internal.h — shared between the host ABI (mtg_host.cpp) and the kernel
// launchers (mtg_kernels.hip, mtg_tube.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/mtg_hip.h"

namespace mtg {

constexpr int kMaxD = 4;  // spatial dimensions supported by the kernels

// Device view of a plan (mtg_plan_create).
struct PlanDev {
  int N, D, r, S;
  int nf, np;              // fixed / free derivatives per dimension
  const double* tab;       // H(1) then A(1)^-1, N*N each (device)
  const int* slots;        // (S+1)*M: fixed index f >= 0, or -(p+1) for free p
  const int* free_map;     // np: free index p -> v*M + k
  const int* fixed_map;    // nf: fixed index f -> v*M + k
  uint64_t fmask;          // bit v*M+k set iff fixed, valid when use_mask
  int use_mask;            // (S+1)*M <= 64
  int std_pattern;         // 1: standard pattern (start/end fully fixed,
                           // intermediate positions only), 2 <= S <= kMaxStdS
  int kernel;              // MTG_KERNEL_* choice (mtg_plan_set_kernel)
};

// Selection fused into a solve kernel's epilogue (mtg_select_device.h):
// the shard's (cost, start + index, rank) triple into out[3]; the lane
// kernels write per-workgroup partials (caller's workspace) that one small
// launch reduces.  out == nullptr: no selection.
struct SelectArgs {
  int64_t start = 0;
  int rank = 0;
  double* out = nullptr;
  double* part_cost = nullptr;
  int64_t* part_idx = nullptr;
  // Deferred selection (mtg_linear_solve_select_prev): the PREVIOUS step's
  // costs prev_cost[0 .. prev_count) (global indices prev_start ..) reduced
  // to the triple prev_out by one extra workgroup of this solve launch
  // (wave and lane-pair kernels; a separate launch before the others).
  const double* prev_cost = nullptr;
  int64_t prev_count = 0;
  int64_t prev_start = 0;
  double* prev_out = nullptr;
};
// Workgroups of the fused solve (the partial slots the workspace needs).
int64_t select_partials(const PlanDev& pl, int64_t B);

// Standard-pattern linear solve at compile-time S (mtg_linear_wave.hip):
// N = 10, r = 4, D = 3, 2 <= S <= 16, the kernel behind "standard" there.
bool has_linear_wave(const PlanDev& pl);
hipError_t launch_linear_solve_wave(const PlanDev& pl, int64_t B, const SelectArgs& sel,
                                    const double* df,
                                    const double* times, double* coeffs, double* cost,
                                    double* free_vals, int32_t* status, hipStream_t st);
// Standard-pattern linear solve (mtg_linear_std.hip).
constexpr int kMaxStdS = 64;
// Lane linear solve for large batches (mtg_linear_lane.hip): one
// (trajectory, dimension) per lane; standard pattern, N = 10, r = 4, D = 3,
// 2 <= S <= kMaxLaneS.  AUTO runs the two-lane variant (mtg_linear_lane2.hip)
// from kLaneMinBatch trajectories: the wave kernel holds at most two waves per
// SIMD up to 2048 trajectories (1024 SIMDs); with a third the lane-pair kernel
// is faster (S = 10: 2048 6.69 vs 7.09 us, 2560 8.03 vs 7.44 us,
// tools/gpu_r04_cross2.sh).
constexpr int kMaxLaneS = 12;
constexpr int64_t kLaneMinBatch = 2049;
// The lane-pair kernel stages its coefficients in LDS from this batch size.
constexpr int64_t kLane2StageMinBatch = 4096;
struct PlanDev;
bool has_linear_lane(const PlanDev& pl);
hipError_t launch_linear_solve_lane(const PlanDev& pl, int64_t B, const double* df,
                                    const double* times, double* coeffs, double* cost,
                                    double* free_vals, int32_t* status, hipStream_t st,
                                    const SelectArgs& sel = SelectArgs{});
int64_t lane_blocks(int64_t B);
// Two lanes per (trajectory, dimension), twisted elimination
// (mtg_linear_lane2.hip); same coverage as the lane kernel.
hipError_t launch_linear_solve_lane2(const PlanDev& pl, int64_t B, const double* df,
                                     const double* times, double* coeffs, double* cost,
                                     double* free_vals, int32_t* status, hipStream_t st,
                                     const SelectArgs& sel = SelectArgs{});
int64_t lane2_blocks(int64_t B);
int linear_kernel_for_batch(const PlanDev& pl, int64_t B);
hipError_t launch_linear_solve_std(const PlanDev& pl, int64_t B, const double* df,
                                   const double* times, double* coeffs, double* cost,
                                   double* free_vals, int32_t* status, hipStream_t st,
                                   const SelectArgs& sel = SelectArgs{});
size_t linear_std_lds_bytes(int N, int S, int D);
// Standard-pattern time kernels (mtg_time_std.hip): N = 10, r = 2..4, D = 1..3.
bool has_time_std(const PlanDev& pl);
hipError_t launch_time_cost_std(const PlanDev& pl, int64_t B, const double* df,
                                const double* times, const mtg_time_params& p, double* cost,
                                double* grad, int32_t* status, hipStream_t st);
hipError_t launch_time_optimize_std(const PlanDev& pl, int64_t B, const double* df,
                                    double* times, const mtg_time_params& p, int max_evals,
                                    double* cost, int32_t* evals, int32_t* solves,
                                    int32_t* result, int32_t* status, hipStream_t st);
size_t time_std_lds_bytes(int N, int S, int D, bool soft);

// Free-derivative objectives and optimiser (mtg_free.hip).
hipError_t launch_free_cost(const PlanDev& pl, int64_t B, const double* df, const double* dp,
                            const double* times, const mtg_time_params& p, int mode,
                            double* cost, double* grad, int32_t* status, hipStream_t st);
hipError_t launch_free_optimize(const PlanDev& pl, int64_t B, const double* df, double* dp,
                                const double* times, const double* lower, const double* upper,
                                const mtg_time_params& p, int max_evals, double* cost,
                                int32_t* evals, int32_t* status, hipStream_t st);
// p.optimizer 1: LN_SBPLX over [T; d_p] (result: nlopt_result codes).
hipError_t launch_time_free_optimize(const PlanDev& pl, int64_t B, const double* df, double* dp,
                                     double* times, const mtg_time_params& p, int max_evals,
                                     double* cost, int32_t* evals, int32_t* result,
                                     int32_t* status, hipStream_t st);
size_t free_lds_bytes(int N, int S, int D, int np, bool soft);
size_t free_sbplx_lds_bytes(int N, int S, int D, int np, bool soft);
inline bool use_std_kernel(const PlanDev& pl) {
  return pl.std_pattern && pl.kernel != MTG_KERNEL_GENERIC;
}

hipError_t launch_select_global_steps(const double* triples, int world, int G, int n,
                                      double* out, hipStream_t st);
hipError_t launch_linear_solve(const PlanDev& pl, int64_t B, const double* df,
                               const double* times, double* coeffs, double* cost,
                               double* free_vals, int32_t* status, hipStream_t st,
                               const SelectArgs& sel = SelectArgs{});
hipError_t launch_coeffs_from_constraints(const PlanDev& pl, int64_t B, const double* df,
                                          const double* dp, const double* times,
                                          double* coeffs, double* cost, int32_t* status,
                                          hipStream_t st);
hipError_t launch_time_cost(const PlanDev& pl, int64_t B, const double* df,
                            const double* times, const mtg_time_params& p,
                            double* cost, double* grad, int32_t* status,
                            hipStream_t st);
hipError_t launch_time_optimize(const PlanDev& pl, int64_t B, const double* df,
                                double* times, const mtg_time_params& p, int max_evals,
                                double* cost, int32_t* evals, int32_t* solves,
                                int32_t* result, int32_t* status, hipStream_t st);
hipError_t launch_segment_matrices(int N, int r, int64_t n, const double* tab,
                                   const double* times, double* Q, double* A,
                                   double* Ainv, double* H, hipStream_t st);
size_t linear_lds_bytes(int N, int S, int D);

// Tube QCQP (mtg_tube.hip).
struct TubeArgs {
  int N, r, S;
  int64_t B;
  const double* tab;        // H(1), A(1)^-1 for (N, r)
  const double* positions;  // B x (S+1) x 3
  const double* fixed_vals; // B x 3 x N
  const double* times_cp;   // B x S
  const double* times;      // B x S
  const double* radii;      // B x S x 2
  // Problems per trajectory: problem b takes its times from row b and its
  // geometry (positions, fixed values, times_cp, radii) from row b / rep
  // (the evaluation points of mtg_tube_time_cost / _optimize).
  int rep = 1;
  // Optional per-trajectory skip flags (indexed by problem / rep): a set flag
  // makes the problem's QCQP workgroup return without touching its outputs.
  const int32_t* skip = nullptr;
  // Optional warm-start state per problem (tube_warm_doubles(N, S) doubles
  // each: x, s, lam of its last usable solve) and its validity flags: a
  // problem with warm_ok set starts from that state, and every usable solve
  // stores its final state and sets the flag (mtg_tube_time.hip, LN_SBPLX).
  double* warm = nullptr;
  int32_t* warm_ok = nullptr;
  // Optional dispatch order: workgroup i solves problem order[i] (a
  // permutation of the B problems).  Results do not depend on it; the
  // LN_SBPLX time optimiser puts the trajectories whose previous solve took
  // the most iterations first (longest-processing-time first), so the
  // round's long solves do not form its tail.
  const int32_t* order = nullptr;
};
// Doubles of one problem's warm-start state.
int64_t tube_warm_doubles(int N, int S);
hipError_t launch_tube_residuals(const TubeArgs& a, const double* x, double* resid,
                                 hipStream_t st);
hipError_t launch_tube_solve(const TubeArgs& a, double tol, int max_iter, double* x,
                             double* coeffs, double* cost, int32_t* iters,
                             int32_t* status, hipStream_t st);
size_t tube_lds_bytes(int N, int S);
// Segment-time objective / optimiser with the QCQP inner solve
// (mtg_tube_time.hip); return MTG_* codes.
// All scratch comes from the caller's workspace (tube_time_workspace_bytes).
size_t tube_time_workspace_bytes(int N, int S, int64_t B, const mtg_time_params& p,
                                 bool optimiser);
// QCQP problems of one launch (B x evaluation points).
int64_t tube_time_problems(int S, int64_t B, const mtg_time_params& p, bool optimiser);
int tube_time_cost(const TubeArgs& a, double tol, int max_iter, const mtg_time_params& p,
                   double* cost, double* grad, int32_t* status, void* workspace,
                   size_t workspace_bytes, hipStream_t st);
int tube_time_optimize(const TubeArgs& a, double* times_io, double tol, int max_iter,
                       const mtg_time_params& p, int max_evals, double* cost, int32_t* evals,
                       int32_t* result, int32_t* status, void* workspace, size_t workspace_bytes,
                       hipStream_t st);

constexpr int kMaxLdsBytes = 160 * 1024;

// Trajectory sampling (mtg_sample.hip).
constexpr int kMaxSampleS = 64;  // segments staged in LDS per trajectory
hipError_t launch_sample(int N, int D, int S, int64_t B, const double* coeffs,
                         const double* times, double t_start, double t_end, double dt,
                         int n_max, int max_deriv, double* samples, double* sample_times,
                         int32_t* n_samples, hipStream_t st);

// Magnitude extrema and soft constraints (mtg_extrema.hip).
constexpr int kMaxExtremaDerivative = 4;  // POSITION..SNAP (nonlinear_impl:2697-2724)
constexpr int kMaxSoftConstraints = 8;
struct SoftLimits {
  int n;
  double value[kMaxSoftConstraints];
};
// Soft-constraint cost formed by the last constraint's launch:
// cost_b = sum_c min(maximum_cost, exp((max_bc - lim_c) / lim_c * weight)).
struct SoftCostArgs {
  double* cost;  // null: plain maximum search
  SoftLimits lim;
  double weight, maximum_cost;
  // Optional per-trajectory skip flags, indexed by trajectory / skip_rep: a
  // set flag makes the trajectory's lanes skip the search and leave its
  // outputs untouched (finished trajectories of the device optimisers).
  const int32_t* skip = nullptr;
  int skip_rep = 1;
};
// Collision cost over a dense occupancy grid (mtg_collision.hip).
size_t collision_lds_bytes(int N, int S);
// Near field of an occupancy map for the collision walk (mtg_coll_field,
// mtg_collision.hip): per voxel v, in kFieldSlots uint16 slots, the squared
// voxel distances from v and from its 6 axis neighbours (v - e_x, v + e_x,
// v - e_y, v + e_y, v - e_z, v + e_z) to the nearest occupied voxel of the
// box the walk scans around v, or kFieldNone when the box holds none:
// exactly the walk's minima m[0..6].
constexpr int kFieldSlots = 8;
constexpr unsigned kFieldNone = 0xFFFFu;
bool coll_field_supported(int side);
hipError_t launch_coll_field(const float* occ, int nx, int ny, int nz, int side,
                             uint16_t* field, hipStream_t st);
hipError_t launch_collision_cost(const PlanDev& pl, int64_t B, const double* coeffs,
                                 const double* times, const float* occ, int nx, int ny, int nz,
                                 const mtg_collision_params& p, double* cost, int32_t* coll,
                                 double* grad_coeffs, double* grad_free, hipStream_t st);

// Minimum outputs of mtg_min_max_magnitude (each nullable).
struct MinOut {
  double* time;
  double* value;
  int32_t* segment;
};
// All constraints of a soft-constraint evaluation in one launch
// (mtg_soft_constraint_cost): one workgroup per trajectory, one
// wave-aligned lane group per constraint, the cost formed in the workgroup.
constexpr int64_t kSoftOneLaunchMaxBatch = 4096;
struct SoftSpec {
  int n;
  int derivative[kMaxSoftConstraints];
  double limit[kMaxSoftConstraints];
  double weight, maximum_cost;
  const int32_t* skip = nullptr;  // as SoftCostArgs::skip
  int skip_rep = 1;
};
hipError_t launch_soft_cost(int N, int D, int S, int64_t B, const double* coeffs,
                            const double* times, const SoftSpec& spec, double* maxima,
                            double* cost, hipStream_t st);
hipError_t launch_soft_cost_any(int N, int D, int S, int64_t B, const double* coeffs,
                                const double* times, const SoftSpec& spec, double* maxima,
                                double* cost, hipStream_t st);
hipError_t launch_max_magnitude(int N, int D, int S, int64_t B, int derivative,
                                const double* coeffs, const double* times, double* max_time,
                                double* max_value, int32_t* max_segment, int value_stride,
                                int value_offset, const SoftCostArgs& soft, hipStream_t st,
                                const MinOut* mino = nullptr);
// Candidate lists of the magnitude extrema per segment (mtg_extrema.hip):
// n_seg = B * S segments, cap entries each.
hipError_t launch_magnitude_candidates(int N, int D, int64_t n_seg, int derivative,
                                       const double* coeffs, const double* times, int cap,
                                       double* cand_time, double* cand_value, int32_t* n_cand,
                                       hipStream_t st);

// Collision-driven objectives and their optimiser (mtg_coll_opt.hip); return
// MTG_* codes.  All scratch comes from the caller's workspace.
size_t coll_workspace_bytes(const PlanDev& pl, int64_t B, int mode, const mtg_coll_params& p,
                            bool optimiser);
int64_t coll_problems(const PlanDev& pl, int64_t B, int mode, const mtg_coll_params& p);
int coll_cost(const PlanDev& pl, int64_t B, int mode, const double* df, const double* x,
              const double* times, const float* occ, int nx, int ny, int nz,
              const uint16_t* field, const mtg_coll_params& p, const double* raise_ref, double* cost, double* grad,
              double* terms, int32_t* collision, int32_t* status, void* workspace,
              size_t workspace_bytes, hipStream_t st);
int coll_optimize(const PlanDev& pl, int64_t B, int mode, const double* df, double* x_io,
                  const double* times, const double* lower, const double* upper,
                  const double* initial_step, const float* occ, int nx, int ny, int nz,
                  const uint16_t* field, const mtg_coll_params& p, int max_evals, double* cost, int32_t* evals,
                  int32_t* result, int32_t* status, double* terms, double* x_history,
                  void* workspace, size_t workspace_bytes, hipStream_t st);

// Multi-GPU selection (mtg_select.hip).
hipError_t launch_select_local(const double* costs, int64_t count, int64_t start, int rank,
                               double* out, hipStream_t st);
// Reduction of n (cost, index) partials (idx == nullptr: index = position)
// to the triple of mtg_select_local over a shard of `count` trajectories.
hipError_t launch_select_reduce(const double* cost, const int64_t* idx, int64_t n, int64_t count,
                                int64_t start, int rank, double* out, hipStream_t st);
hipError_t launch_select_global(const double* triples, int world, double* out, hipStream_t st);

}  // namespace mtg
