// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU (FP64) restatement of the reference algorithm of
// NilsFunk/mav_tube_trajectory_generation for the hot path named in
// BASELINE.json `north_star` (linear minimum-derivative solve, tube QCQP
// constraint assembly, time-allocation cost callback).  Every function cites
// the reference file:line it follows (paths relative to the reference root;
// "linear_impl" = include/mav_tube_trajectory_generation/impl/
// polynomial_optimization_linear_impl.h, "qcqp_impl" / "nonlinear_impl"
// likewise).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this library, and only as the checker / CPU baseline: the product path
// (mav_tube_trajectory_generation_amd/, libmtg_hip.so) never links it.
//
// Parity pinning: the reference itself cannot be built here (Eigen, glog,
// NLopt, MOSEK and supereight are absent).  The linear
// restatement is pinned by the reference's own known-answer test
// (TwoVerticesSetup, test/test_polynomial_optimization.cpp:707-751) and its
// property tests (AMatrixInversion :695-705, ConstraintPacking :510-570,
// checkPath :113-172, checkCost :174-195) — see tests/test_oracle.py.  The
// QCQP solve (MOSEK in the reference) and the NLopt driver are "parity
// unpinned": MOSEK is replaced by the oracle's own primal-dual interior-point
// method, cross-checked against SciPy in tests.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Falling-factorial table base(n, i) = i!/(i-n)! (polynomial.cpp:145-161),
// n x n row-major.
int orc_base_coefficients(int n, double* out);

// Row `deriv` of the derivative basis at time t (polynomial.h:201-219).
int orc_base_coeffs_with_time(int N, int deriv, double t, double* out);

// Per-segment matrices for time T: Q (linear_impl:557-573), A
// (linear_impl:101-111), A^-1 by the Schur complement (linear_impl:132-169),
// H = A^-T Q A^-1 (linear_impl:318).  All N x N row-major; any may be NULL.
int orc_segment_matrices(int N, int r, double T, double* Q, double* A,
                         double* Ainv, double* H);

// createRandomVertices (vertex.cpp:27-82) with std::mt19937(seed) and
// std::uniform_real_distribution<double>.  Dense vertex form: mask[(v*K+k)]
// = 1 when vertex v carries a constraint on derivative k, values at
// vals[(v*K+k)*D + d].  K >= max_deriv+1.
int orc_random_vertices(int max_deriv, int S, int D, const double* pos_min,
                        const double* pos_max, uint64_t seed, int K,
                        uint8_t* mask, double* vals);

// estimateSegmentTimesNfabian (vertex.cpp:252-269; method 0) and
// estimateSegmentTimesVelocityRamp (vertex.cpp:233-250, 271-287; method 1).
// positions: (S+1) x D.
int orc_estimate_segment_times(int S, int D, const double* positions,
                               double v_max, double a_max, int method,
                               double magic_or_factor, double* times);

// Full linear path: setupFromVertices (linear_impl:46-99) + solveLinear
// (:337-379) + computeCost (:113-130).  Vertex constraints given in the dense
// form above with stride K (constraints of order > N/2-1 are dropped as in
// linear_impl:72-95).  Outputs (any may be NULL):
//   coeffs  S x D x N (segment, dimension, coefficient)
//   cost    scalar
//   df, dp  D x n_f, D x n_p compact fixed / free constraints
//   nf, np  counts
// Returns 0 on success, <0 on contract violation (the reference CHECK-aborts).
int orc_linear_solve(int N, int D, int r, int S, int K, const uint8_t* mask,
                     const double* vals, const double* times, double* coeffs,
                     double* cost, double* df, double* dp, int* nf, int* np);

// Accessors of the linear problem (linear_impl:489-555): dense R
// ((nf+np)^2), M (n_all x (nf+np)), A and A^-1 (NS x NS), M_pinv
// ((nf+np) x n_all).  Sizes via orc_linear_solve's nf/np (n_all = N*S).
int orc_linear_matrices(int N, int D, int r, int S, int K, const uint8_t* mask,
                        const double* vals, const double* times, double* R,
                        double* M, double* A, double* Ainv, double* Mpinv);

// Time-allocation objective of objectiveFunctionTime (nonlinear_impl:877-945)
// with w_c = 0 and no soft constraints, linear inner solve (upstream
// semantics): J = computeCost() + time_penalty * (sum T)^2.
// grad_mode 0: none; 1: getCostAndGradientTime (nonlinear_impl:2495-2584)
//   = w_d * dJd/dT_n + w_t, J_d = d^T R d with d held fixed (:1537-1606);
// 2: central differences of J itself (re-solved), increment and clamp rule of
//   nonlinear_impl:2525-2530.
int orc_time_cost(int N, int D, int r, int S, int K, const uint8_t* mask,
                  const double* vals, const double* times, double time_penalty,
                  int grad_mode, double increment, double w_d, double w_t,
                  double* cost, double* grad);

// PolynomialOptimization::computeMaximumOfMagnitude (linear_impl:455-487)
// on one trajectory (coeffs S x D x N, times S): the Extremum {time relative
// to its segment, value, segment}.  Roots by companion-matrix eigenvalues in
// place of Jenkins-Traub (see mtg_oracle.cpp).  -3 if N - derivative - 1 <= 0.
int orc_magnitude_candidates(int N, int D, int S, const double* coeffs, const double* times,
                             int derivative, int cap, double* cand_time, double* cand_value,
                             int* n_cand);
int orc_max_magnitude(int N, int D, int S, const double* coeffs, const double* times,
                      int derivative, double* time, double* value, int* segment,
                      int* n_candidates);
// All complex roots of the polynomial with increasing coefficients inc[0..n).
int orc_poly_roots(int n, const double* inc, double* re, double* im);
// evaluateMaximumMagnitudeAsSoftConstraint (nonlinear_impl:2735-2766).
int orc_soft_constraint_cost(int N, int D, int S, const double* coeffs, const double* times,
                             int n_constraints, const int* derivatives, const double* limits,
                             double weight, double maximum_cost, double* maxima,
                             double* cost);

// ---------------- tube QCQP (qcqp_impl) ----------------
// Inverse Bezier control-point map B^-1(T) with the 1e-5 zero-snap
// (qcqp_impl:267-319), N x N row-major.
int orc_control_point_map(int N, double T, double* Binv);

// Trajectory::evaluateRange (src/trajectory.cpp:74-134) on the trajectory
// given by coeffs (S x D x N) and segment times, for one derivative, exactly
// as the reference iterates (accumulated times by repeated addition).
// out: max_out x D samples, times_out: max_out (nullable); *count = number
// of samples the reference would produce (may exceed max_out; only the
// first max_out are written).  Returns 0, or -1 if t_start is out of range.
int orc_evaluate_range(int N, int D, int S, const double* coeffs, const double* times,
                       double t_start, double t_end, double dt, int derivative,
                       int max_out, double* out, double* times_out, int* count);

// Number of inequality constraints the tube problem builds
// (qcqp_impl:321-474): (S-1) spheres + S*(N-2) tubes + 2*S*(N-2) half-spaces.
int orc_tube_num_constraints(int N, int S);

// Assemble the tube QCQP exactly as setupFromVertices(radii) +
// setupControlPointConstraints (qcqp_impl:121-186, 321-474) and return it in
// dense form over the n_free_kDim = (S-1)*N/2*D free variables
// (dim-major, qcqp_impl:95-117):
//   P = 2 R_pp (n x n), q = 2 R_pf d_f (n), and per constraint k
//   quad_k (n x n), lin_k (n), cst_k: 0.5 x^T quad_k x + lin_k x + cst_k <= 0.
// times_cp = segment times used for the control-point maps (the reference
// builds them once at setup, qcqp_impl:152-157); times = current segment
// times (Q, A^-1).  Pass the same array twice for a fresh setup.
// radii: S x 2 (tube radius r1 = .first, sphere radius r2 = .second).
// Any output may be NULL; quad is large (ncon*n*n doubles).
int orc_tube_qcqp_assemble(int N, int D, int r, int S, int K,
                           const uint8_t* mask, const double* vals,
                           const double* times_cp, const double* times,
                           const double* radii, double* P, double* q,
                           double* quad, double* lin, double* cst, int* n_free);

// Residuals g_k(x) of the assembled constraints at free vector x
// (length n_free_kDim).  resid: ncon.
int orc_tube_residuals(int N, int D, int r, int S, int K, const uint8_t* mask,
                       const double* vals, const double* times_cp,
                       const double* times, const double* radii,
                       const double* x, double* resid);

// Solve the tube QCQP (replaces MSK_optimizetrm, qcqp_impl:476-788) with the
// oracle's primal-dual interior-point method, then recover coefficients
// (qcqp_impl:777-785 -> linear_impl:254-275) and the cost.
//   x_out: n_free_kDim; coeffs: S x D x N; cost: computeCost();
//   iters: IPM iterations; returns 0 converged, 1 max-iterations, <0 error.
int orc_tube_qcqp_solve(int N, int D, int r, int S, int K, const uint8_t* mask,
                        const double* vals, const double* times_cp,
                        const double* times, const double* radii, double tol,
                        int max_iter, double* x_out, double* coeffs,
                        double* cost, int* iters);

// objectiveFunctionTime with the QCQP inner solve (mtg_tube_time_cost):
// grad_mode 0 or 2; NaN cost where the QCQP fails.
int orc_tube_time_cost(int N, int D, int r, int S, int K, const uint8_t* mask,
                       const double* vals, const double* times_cp, const double* times,
                       const double* radii, double tol, int max_iter, double time_penalty,
                       int grad_mode, double increment, int n_soft,
                       const int* soft_derivatives, const double* soft_limits,
                       double soft_weight, double soft_maximum_cost, double* cost,
                       double* grad);
// The mtg_tube_time_optimize algorithm on that objective.
int orc_tube_time_optimize(int N, int D, int r, int S, int K, const uint8_t* mask,
                           const double* vals, const double* radii, double* times_io,
                           double tol, int max_iter, double time_penalty, double increment,
                           int max_evals, int n_soft, const int* soft_derivatives,
                           const double* soft_limits, double soft_weight,
                           double soft_maximum_cost, double* cost, int* evals);

// optimizeTime in the fork's QCQP form with LN_SBPLX (orc_sbplx.cpp): the
// reference's default kOptimizeTime path (nonlinear_impl:332-397, 877-945).
int orc_tube_time_optimize_sbplx(int N, int D, int r, int S, int K, const uint8_t* mask,
                                 const double* vals, const double* radii, double* times_io,
                                 double tol, int max_iter, double time_penalty, int max_evals,
                                 double f_rel, double f_abs, double step_rel, int n_soft,
                                 const int* soft_derivatives, const double* soft_limits,
                                 double soft_weight, double soft_maximum_cost, double* cost,
                                 int* evals, int* result, double* history);

// CPU baseline timing (bench.py cpu_baseline leg): repeat setupFromVertices +
// solveLinear + computeCost (the region polynomial_timing_evaluation.cpp:
// 93-110 times) over B trajectories given in dense vertex form
// (masks: B x (S+1) x K, vals: B x (S+1) x K x D, times: B x S), cycling
// until at least min_seconds have elapsed, on `threads` std::threads.
// Returns the number of solves and the wall seconds (steady_clock).
int orc_bench_linear(int N, int D, int r, int S, int K, int B, const uint8_t* masks,
                     const double* vals, const double* times, int threads,
                     double min_seconds, int64_t* solves, double* seconds);

// The batched optimiser of mtg_time_optimize (time_optimize_kernel),
// restated on the oracle objective (objectiveFunctionTime,
// nonlinear_impl:877-945, with central-difference gradients, grad_mode 2):
// projected scaled steepest descent in [0.1, 2 T0] (nonlinear_impl:350-378),
// step x1.5 on success / x0.5 on failure, at most max_evals objective
// evaluations.  times_io: S (in: T0, out: optimised times).
int orc_time_optimize(int N, int D, int r, int S, int K, const uint8_t* mask,
                      const double* vals, double* times_io, double time_penalty,
                      double increment, int max_evals, double* cost, int* evals);

// objectiveFunctionTime / the optimiser with soft magnitude constraints
// (use_soft_constraints, nonlinear_impl:907-913, 2735-2766): the objective
// adds orc_soft_constraint_cost on the solved coefficients.
int orc_time_cost_soft(int N, int D, int r, int S, int K, const uint8_t* mask,
                       const double* vals, const double* times, double time_penalty,
                       int grad_mode, double increment, double w_d, double w_t, int n_soft,
                       const int* soft_derivatives, const double* soft_limits,
                       double soft_weight, double soft_maximum_cost, double* cost,
                       double* grad);
// The optimiser with hard inequality constraints (use_soft_constraints =
// false, nonlinear_impl:861-872): g_c = max |p^(derivatives[c])| - limits[c]
// <= tolerance, accepted trials feasible-and-lower or less infeasible.
int orc_time_optimize_hard(int N, int D, int r, int S, int K, const uint8_t* mask,
                           const double* vals, double* times_io, double time_penalty,
                           double increment, int max_evals, int n_con, const int* derivatives,
                           const double* limits, double tolerance, double* cost, int* evals);
int orc_time_optimize_soft(int N, int D, int r, int S, int K, const uint8_t* mask,
                           const double* vals, double* times_io, double time_penalty,
                           double increment, int max_evals, int n_soft,
                           const int* soft_derivatives, const double* soft_limits,
                           double soft_weight, double soft_maximum_cost, double* cost,
                           int* evals);
// optimizeTime with the reference's default LN_SBPLX (orc_sbplx.cpp, NLopt
// restated; impl/polynomial_optimization_nonlinear_impl.h:95-101, 332-397,
// 877-945): bounds [0.1, 2 T0], initial step step_rel T0, maxeval
// max_evals, ftol_rel f_rel, ftol_abs f_abs.  result: the nlopt_result code.
int orc_time_optimize_sbplx(int N, int D, int r, int S, int K, const uint8_t* mask,
                            const double* vals, double* times_io, double time_penalty,
                            int max_evals, double f_rel, double f_abs, double step_rel,
                            int n_soft, const int* soft_derivatives, const double* soft_limits,
                            double soft_weight, double soft_maximum_cost, double* cost,
                            int* evals, int* result, double* history);
// The LN_SBPLX restatement on a fixed test objective (tests/test_sbplx.py).
int orc_sbplx_test(int n, const double* lb, const double* ub, double* x, const double* xstep,
                   int maxeval, double ftol_rel, double ftol_abs, double* minf, int* nevals,
                   double* history);

// CPU baseline for the other bench workloads, same cycling/threads/timing
// rules as orc_bench_linear.  kind 1: orc_time_optimize with max_evals =
// param_i; kind 2: tube QCQP solve (radii: B x S x 2, tol 1e-10, 100
// iterations); kind 3: evaluateRange for derivatives 0..param_i at
// dt = param_d over the whole trajectory, on coefficients solved once before
// the clock starts; kind 4: the soft-constraint cost of max |v| <= 3,
// max |a| <= 5 (two computeMaximumOfMagnitude searches) on coefficients
// solved before the clock starts; kind 5: orc_tube_time_cost with the
// grad_mode 2 gradient (2S + 1 QCQP solves, times_cp = times); kind 6:
// orc_time_optimize_sbplx with max_evals = param_i (f_rel 0.05, step 0.1); kind
// 7: orc_tube_time_optimize_sbplx with max_evals = param_i.  *units =
// optimisations (1), solves (2), samples (3, one sample = all derivatives of
// all dimensions at one time), trajectories (4) or evaluations (5).
int orc_bench_workload(int kind, int N, int D, int r, int S, int K, int B,
                       const uint8_t* masks, const double* vals, const double* times,
                       const double* radii, int param_i, double param_d, int threads,
                       double min_seconds, int64_t* units, double* seconds);

// Free-derivative objectives (see mtg_oracle.cpp):
// mode 0 objectiveFunctionFreeConstraints (nonlinear_impl:1021-1113, J_d and
// its gradient of :1537-1606), mode 1 objectiveFunctionTimeAndConstraints
// (:947-1019).  dp, grad: D x np.
int orc_free_cost(int N, int D, int r, int S, int K, const uint8_t* mask, const double* vals,
                  const double* times, const double* dp, int mode, double time_penalty,
                  int n_soft, const int* soft_derivatives, const double* soft_limits,
                  double soft_weight, double soft_maximum_cost, double* cost, double* grad);
// The mtg_free_optimize algorithm restated (projected Newton steps of J_d
// with backtracking on J_d + soft).  dp_io, lower, upper: D x np.
int orc_free_optimize(int N, int D, int r, int S, int K, const uint8_t* mask,
                      const double* vals, const double* times, double* dp_io,
                      const double* lower, const double* upper, int n_soft,
                      const int* soft_derivatives, const double* soft_limits,
                      double soft_weight, double soft_maximum_cost, int max_evals, double* cost,
                      int* evals);

// The mtg_time_free_optimize algorithm restated (optimizeTimeAndFreeConstraints
// with projected block-alternating steps).  dp_io: D x np, times_io: S.
int orc_time_free_optimize(int N, int D, int r, int S, int K, const uint8_t* mask,
                           const double* vals, double* dp_io, double* times_io,
                           double time_penalty, double increment, int n_soft,
                           const int* soft_derivatives, const double* soft_limits,
                           double soft_weight, double soft_maximum_cost, int max_evals,
                           double* cost, int* evals);

// optimizeTimeAndFreeConstraints with LN_SBPLX over [T; d_p] (the reference's
// default algorithm; see mtg_oracle.cpp).  dp_io: D x np, times_io: S.
int orc_time_free_optimize_sbplx(int N, int D, int r, int S, int K, const uint8_t* mask,
                                 const double* vals, double* dp_io, double* times_io,
                                 double time_penalty, int n_soft, const int* soft_derivatives,
                                 const double* soft_limits, double soft_weight,
                                 double soft_maximum_cost, int max_evals, double f_rel,
                                 double f_abs, double step_rel, double* cost, int* evals,
                                 int* result, double* history);

// Collision cost of getCostAndGradientCollision (nonlinear_impl:1609-1780)
// over a dense occupancy grid (see mtg_oracle.cpp).  dp: D x np (D = 3);
// params: res, min_bound[3], max_bound[3], epsilon, robot_radius,
// coll_pot_multiplier, coll_check_time_increment.  grad_coeffs S x D x N,
// grad_free D x np (nullable).
int orc_collision_cost(int N, int D, int r, int S, int K, const uint8_t* mask,
                       const double* vals, const double* times, const double* dp,
                       const float* occupancy, int nx, int ny, int nz, const double* params,
                       int box_side, double* cost, int* collision, double* grad_coeffs,
                       double* grad_free);

// Collision-driven objectives of the reference demo (mtg_coll_cost /
// mtg_coll_optimize; see mtg_oracle.cpp for the params / iparams layout):
// mode 0 objectiveFunctionFreeConstraintsAndCollision (nonlinear_impl:
// 1115-1272), x = d_p (D x np); mode 1 ...AndCollisionAndTime (:1274-1535),
// x = [T; d_p].  times: setup times (mode 0: the segment times).
// raise_ref: total_cost_iter0_ / last total for the collision raise rule.
// grad: nv, terms: 4 (nullable).
int orc_coll_cost(int N, int D, int r, int S, int K, const uint8_t* mask, const double* vals,
                  const double* times, int mode, const double* x, const float* occupancy, int nx,
                  int ny, int nz, const double* params, const int* iparams,
                  const int* soft_derivatives, const double* soft_limits, double raise_ref,
                  double* cost, double* grad, double* terms, int* collision);
// The mtg_coll_optimize algorithm (projected L-BFGS) on that objective.
int orc_coll_optimize(int N, int D, int r, int S, int K, const uint8_t* mask, const double* vals,
                      const double* times, int mode, const float* occupancy, int nx, int ny,
                      int nz, const double* params, const int* iparams,
                      const int* soft_derivatives, const double* soft_limits,
                      const double* lower, const double* upper, const double* initial_step,
                      int max_evals, double* x_io, double* cost, int* evals, int* result,
                      double* terms);

// CPU baseline of bench.py's collision workload (orc_coll_optimize mode 0
// over B starts X0 [B][nv], `threads` threads, >= min_seconds).
int orc_bench_coll(int N, int D, int r, int S, int K, const uint8_t* mask, const double* vals,
                   const double* times, const float* occupancy, int nx, int ny, int nz,
                   const double* params, const int* iparams, const int* soft_derivatives,
                   const double* soft_limits, int B, int nv, const double* X0, int max_evals,
                   int threads, double min_seconds, int64_t* units, double* seconds);

#ifdef __cplusplus
}
#endif
