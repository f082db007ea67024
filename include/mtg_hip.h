/*
 * mtg_hip.h — C ABI of the MI355X-native batched polynomial trajectory
 * optimizer (libmtg_hip.so, built from mav_tube_trajectory_generation_amd/
 * csrc/ for gfx950).
 *
 * This is the drop-in boundary for the hot path of
 * NilsFunk/mav_tube_trajectory_generation (BASELINE.json `north_star`).
 * The reference has no FFI: its boundary is the header-only C++ template API
 * PolynomialOptimization<N> / PolynomialOptimizationConstrained<N> /
 * PolynomialOptimizationNonLinear<N>.  Each entry point below
 * names the reference interface it replaces (file:line relative to the
 * reference root; "linear_impl" = include/mav_tube_trajectory_generation/
 * impl/polynomial_optimization_linear_impl.h, "qcqp_impl" / "nonlinear_impl"
 * likewise).  The C++ host mirror of that API lives in
 * include/mav_tube_trajectory_generation_amd/ and calls only this ABI.
 *
 * Conventions
 *  - All arithmetic is FP64.
 *  - int return = status: 0 ok, < 0 error (mtg_status_string).  No C++
 *    exceptions cross the ABI.  The reference CHECK-aborts on contract
 *    violations (linear_impl:50-55, 66-67, 281-283, 296); here they are
 *    reported as MTG_ERR_* codes, per trajectory where they depend on data.
 *  - "device" pointers are HIP device (HBM) pointers owned by the caller;
 *    "host" pointers are ordinary host memory.  Batched calls are
 *    stream-ordered on `stream` (hipStream_t, NULL = default stream) and do
 *    not synchronise.
 *  - Layouts are row-major; a batch of B independent trajectories is stored
 *    trajectory-major (trajectory b occupies one contiguous slice).
 *  - N = number of polynomial coefficients (even, 4..12); M = N/2 endpoint
 *    derivatives per vertex; D = spatial dimensions (1..4); S = segments;
 *    r = derivative to optimise (0..M-1).
 *  - A constraint pattern is a host byte array fixed_mask[(S+1) * M]:
 *    fixed_mask[v*M + k] != 0 iff vertex v constrains derivative k
 *    (Vertex::getConstraint, vertex.cpp:155-163).  Fixed constraints are
 *    numbered in (vertex, derivative) order, free ones likewise — the
 *    std::set<Constraint> order of linear_impl:171-252.
 */
#ifndef MTG_HIP_H_
#define MTG_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  MTG_OK = 0,
  MTG_ERR_INVALID_ARG = -1,  /* bad N/D/r/S/B or NULL pointer */
  MTG_ERR_NO_DEVICE = -2,    /* no HIP device / runtime error */
  MTG_ERR_HIP = -3,          /* HIP API call failed */
  MTG_ERR_UNSUPPORTED = -4,  /* size beyond the kernels' LDS budget */
  MTG_ERR_NUMERIC = -5       /* at least one trajectory failed (see status) */
};
/* HIP error state: an entry point that launches device work clears the
 * thread's pending HIP error (hipGetLastError) before it launches, so that a
 * failed call made earlier by the caller or another library is not reported
 * as this call's MTG_ERR_HIP; check your own HIP calls before calling one of
 * these.  Getters, size queries (*_workspace_bytes, mtg_coll_field_bytes,
 * mtg_tube_num_constraints), mtg_generate_random_problems and the create /
 * destroy calls leave the pending error untouched. */

/* Per-trajectory status codes written by batched kernels. */
enum {
  MTG_TRAJ_OK = 0,
  MTG_TRAJ_BAD_TIME = 1,     /* a segment time <= 0 (linear_impl:296) */
  MTG_TRAJ_NOT_SPD = 2,      /* free-derivative system not positive definite
                                (tube QCQP: its KKT system broke down twice,
                                plain and regularised, away from the optimum) */
  MTG_TRAJ_NOT_CONVERGED = 3, /* interior-point solve hit its iteration cap */
  MTG_TRAJ_NEAR_OPTIMAL = 4   /* interior-point solve stopped where its KKT
                                 system broke down, every residual within
                                 1e3 x tol: usable, not converged to tol */
};

typedef struct mtg_ctx mtg_ctx;
typedef struct mtg_plan mtg_plan;

const char* mtg_status_string(int status);
int mtg_version(void);

/* Context = one HIP device.  Replaces nothing in the reference (which has no
 * device); owns the cached constant tables and constraint patterns.
 * mtg_ctx_create makes `device` the calling thread's current device (the
 * C++ shim allocates its buffers there).  Allocating calls (plan create /
 * destroy, the constant tables, the host-memory solve's staging) run on the
 * context's device and restore the caller's current device; the launching
 * calls enqueue on the stream they are given (null: the current device's
 * null stream), whose device must be the context's. */
int mtg_ctx_create(int device, mtg_ctx** out);
int mtg_ctx_destroy(mtg_ctx* ctx);
int mtg_ctx_device(const mtg_ctx* ctx);

/* ------------------------------------------------------------------------
 * Plan = one (N, D, r, S, constraint pattern).  Replaces the batch-uniform
 * part of PolynomialOptimization<N>::setupFromVertices (linear_impl:46-99):
 * the constraint reordering of setupConstraintReorderingMatrix
 * (linear_impl:171-252) and the per-(N, r) base / cost tables
 * (polynomial.cpp:145-161, linear_impl:557-573).  Uploads to the device
 * synchronously; the solve calls below never allocate or synchronise.
 */
int mtg_plan_create(mtg_ctx* ctx, int N, int D, int r, int S,
                    const uint8_t* fixed_mask /* host (S+1)*M */,
                    mtg_plan** out);
int mtg_plan_destroy(mtg_plan* plan);
/* Kernel selection for mtg_linear_solve.  AUTO (default) runs the
 * standard-pattern kernels when the pattern is the reference's standard one
 * (start and end vertex fully fixed, intermediate vertices position only:
 * createRandomVertices / makeStartOrEnd, vertex.cpp:27-82, 147-153) and
 * 2 <= S <= 64, else the generic kernel.  Among the standard-pattern kernels
 * it picks by batch size: STANDARD (one wavefront per trajectory, lowest
 * latency) up to 2048 trajectories, LANE_PAIR above.  LANE gives each
 * (trajectory, dimension) one lane that walks the whole vertex chain;
 * LANE_PAIR gives it two lanes in two wavefronts of one workgroup that
 * eliminate the chain from both ends toward the middle vertex (a twisted
 * factorisation, Schur terms exchanged through LDS): half the chain per lane
 * (13.8 vs 15.6 us at B = 8192, equal at 65536).  Both cover N = 10, r = 4,
 * D = 3, 2 <= S <= 12.  GENERIC forces the generic kernel (parity
 * cross-checks); STANDARD / LANE / LANE_PAIR fail with MTG_ERR_UNSUPPORTED
 * where they do not apply.  mtg_plan_kernel returns the forced kernel, or
 * for AUTO the wavefront kernel (GENERIC or STANDARD);
 * mtg_plan_kernel_for_batch the kernel a solve of B trajectories runs.  The
 * time, free-derivative and sampling entry points treat LANE and LANE_PAIR
 * like STANDARD. */
enum {
  MTG_KERNEL_AUTO = 0,
  MTG_KERNEL_GENERIC = 1,
  MTG_KERNEL_STANDARD = 2,
  MTG_KERNEL_LANE = 3,
  MTG_KERNEL_LANE_PAIR = 4
};
int mtg_plan_set_kernel(mtg_plan* plan, int kernel);
int mtg_plan_kernel(const mtg_plan* plan);
int mtg_plan_kernel_for_batch(const mtg_plan* plan, int64_t B);

/* n_fixed / n_free per dimension (getNumberFixedConstraints /
 * getNumberFreeConstraints, polynomial_optimization_linear.h:224-226). */
int mtg_plan_counts(const mtg_plan* plan, int* n_fixed, int* n_free);

/* Batched linear solve.  Replaces, per trajectory b,
 *   updateSegmentTimes(times_b)            linear_impl:277-304
 *   solveLinear()                          linear_impl:337-379
 *     constructR (R = M^T blkdiag(A^-T Q A^-1) M)   linear_impl:306-335
 *     d_p = -R_pp^-1 R_pf d_f per dimension         linear_impl:359-375
 *     updateSegmentsFromCompactConstraints          linear_impl:254-275
 *   computeCost()                          linear_impl:113-130
 * Inputs (device):
 *   fixed_vals  B x D x n_fixed   fixed_constraints_compact_ per dimension
 *   times       B x S             segment times
 * Outputs (device; all but coeffs may be NULL):
 *   coeffs      B x S x D x N     segment polynomial coefficients,
 *                                 increasing powers (polynomial.h:33-37)
 *   cost        B                 computeCost() = 0.5 sum c^T Q c
 *   free_vals   B x D x n_free    free_constraints_compact_ (d_p)
 *   status      B                 MTG_TRAJ_*
 */
int mtg_linear_solve(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                     const double* times, double* coeffs, double* cost,
                     double* free_vals, int32_t* status, void* stream);

/* Same, host pointers in and out.  Used by the C++ single-trajectory shim
 * PolynomialOptimization<N>::solveLinear().  The plan keeps persistent
 * staging (a pinned, device-mapped host buffer, a device buffer and a
 * stream of its own, created on first use, grown when a larger B arrives): a
 * steady-state call of up to 64 KB of inputs and outputs (a single
 * trajectory) is one launch reading and writing the mapped host buffer, then
 * a wait on that stream; larger calls add one host-to-device and one
 * device-to-host copy.  No allocation, no device-wide synchronisation.  Calls on one plan are serialised (the staging is
 * shared); use separate plans for concurrent host threads. */
int mtg_linear_solve_host(const mtg_plan* plan, int64_t B,
                          const double* fixed_vals, const double* times,
                          double* coeffs, double* cost, double* free_vals,
                          int32_t* status);

/* Coefficients and cost from given fixed AND free derivatives (no solve):
 * setFreeConstraints -> updateSegmentsFromCompactConstraints
 * (linear_impl:254-275, 497-506) followed by computeCost (:113-130).
 * Inputs (device): fixed_vals B x D x n_fixed, free_vals B x D x n_free,
 * times B x S.  Outputs (device): coeffs B x S x D x N; cost B and status B
 * nullable. */
int mtg_coeffs_from_constraints(const mtg_plan* plan, int64_t B,
                                const double* fixed_vals, const double* free_vals,
                                const double* times, double* coeffs, double* cost,
                                int32_t* status, void* stream);

/* Per-segment matrices for a batch of n segment times (device), each N x N:
 * Q(T) = computeQuadraticCostJacobian (linear_impl:557-573),
 * A(T) = setupMappingMatrix (linear_impl:101-111),
 * A^-1(T) = invertMappingMatrix (linear_impl:132-169),
 * H(T) = A^-T Q A^-1 (linear_impl:318).  Any output may be NULL.
 * Backs getA / getAInverse / getR (linear_impl:503-544). */
int mtg_segment_matrices(mtg_ctx* ctx, int N, int r, int64_t n,
                         const double* times, double* Q, double* A,
                         double* Ainv, double* H, void* stream);

/* ------------------------------------------------------------------------
 * Time-allocation cost callback, batched.  Replaces
 * PolynomialOptimizationNonLinear<N>::objectiveFunctionTime
 * (nonlinear_impl:877-945) with w_c = 0 and a linear
 * inner solve (upstream semantics):
 *   J(T) = computeCost() + time_penalty * (sum_i T_i)^2 [+ soft]
 * soft (n_soft > 0, use_soft_constraints, :907-913) is
 * evaluateMaximumMagnitudeAsSoftConstraint (:2735-2766) over the
 * addMaximumMagnitudeConstraint list (:847-875): sum_c min(soft_maximum_cost,
 * exp((max_t |p^(soft_derivative[c])| - soft_limit[c]) / soft_limit[c] *
 * soft_weight)), with the maxima from the device extremum search of
 * mtg_max_magnitude.
 * hard_constraints = 1 (use_soft_constraints = false): the constraints are
 * the reference's NLopt inequality constraints g_c(T) = max_t
 * |p^(soft_derivative[c])| - soft_limit[c] <= hard_tolerance
 * (evaluateMaximumMagnitudeConstraint, :2687-2733); J carries no soft term
 * and mtg_time_optimize accepts a trial only if it is feasible and lowers J,
 * or, from an infeasible point, lowers the largest violation (feasibility
 * first).  Only mtg_time_cost / mtg_time_optimize accept it; every other
 * entry point returns MTG_ERR_INVALID_ARG for hard_constraints != 0.
 * grad_mode (grad may be NULL when 0):
 *   0  no gradient (objectiveFunctionTime is gradient-free, :881-882)
 *   1  getCostAndGradientTime (nonlinear_impl:2495-2584):
 *        grad_n = w_d * dJ_d/dT_n + w_t,  J_d = sum_dims d^T R(T) d with d
 *        held at the solution for T (getCostAndGradientDerivative,
 *        :1537-1606), central differences with step `increment`, clamped
 *        at 0.1 (:2525-2530)
 *   2  central differences of J itself (re-solved), same step and clamp.
 * Inputs/outputs are device pointers: fixed_vals B x D x n_fixed,
 * times B x S, cost B, grad B x S, status B.
 */
typedef struct mtg_time_params {
  double time_penalty; /* NonlinearOptimizationParameters::time_penalty (500) */
  double increment;    /* ::increment_time (0.1) */
  double w_d;          /* ::weights.w_d (0.1) */
  double w_t;          /* ::weights.w_t (1.0) */
  int grad_mode;       /* see above */
  int n_soft;          /* soft magnitude constraints, 0..8 (0: none) */
  int soft_derivative[8];   /* derivative order of constraint c, 0..4 */
  double soft_limit[8];     /* maximum_value of constraint c, > 0 */
  double soft_weight;       /* ::soft_constraint_weight (100) */
  double soft_maximum_cost; /* maximum_cost (1e12, header :576) */
  int hard_constraints;     /* 0: the n_soft constraints are soft costs
                               (use_soft_constraints = true, the default);
                               1: hard inequalities (use_soft_constraints =
                               false, nonlinear_impl:861-872) */
  double hard_tolerance;    /* ::inequality_constraint_tolerance (0.1) */
  /* The optimiser of mtg_time_optimize (round 5; a zero-filled struct keeps
   * the earlier behaviour):
   *   0  projected central-difference descent (below);
   *   1  LN_SBPLX, the reference's default algorithm (nlopt::LN_SBPLX,
   *      polynomial_optimization_nonlinear.h:61): NLopt's Subplex with its
   *      bounded Nelder-Mead restated on the device (mtg_sbplx_device.h),
   *      gradient-free, stopping at max_evals evaluations or at f_rel /
   *      f_abs (NLopt's ftol_rel / ftol_abs, nonlinear_impl:97-98; <= 0
   *      disables).  Soft constraints enter the objective; hard constraints
   *      are rejected (NLopt's SBPLX takes no inequality constraints). */
  int optimizer;
  double f_rel;                /* ::f_rel (0.05) */
  double f_abs;                /* ::f_abs (-1: disabled) */
  double initial_stepsize_rel; /* ::initial_stepsize_rel (0.1); <= 0 means 0.1 */
} mtg_time_params;

int mtg_time_cost(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                  const double* times, const mtg_time_params* params,
                  double* cost, double* grad, int32_t* status, void* stream);

/* Batched segment-time optimisation.  Replaces optimizeTime
 * (nonlinear_impl:332-397): bounds [0.1, 2 T0] per segment (:350-358,
 * 375-378), `max_evals` objective evaluations per trajectory (NLopt maxeval,
 * :101).  params->optimizer 0: a projected gradient method with
 * backtracking on the grad_mode 2 gradient; 1: LN_SBPLX (the reference's
 * default, restated: NLopt itself is absent).  Both run entirely on the
 * device (one workgroup per trajectory, no host round trips).
 *   times_io   B x S  in: initial times T0, out: optimised times
 *   cost       B      final objective
 *   evals      B      objective evaluations used (nullable)
 *   solves     B      inner solves run, gradient points included (nullable;
 *                     the work count behind the FP64 roofline of bench.py)
 */
int mtg_time_optimize(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                      double* times_io, const mtg_time_params* params,
                      int max_evals, double* cost, int32_t* evals,
                      int32_t* solves, int32_t* status, void* stream);
/* The same with the optimiser's stopping reason per trajectory (result, B,
 * nullable): NLopt's nlopt_result codes, as optimizeTime returns them
 * (nlopt::opt::optimize, nonlinear_impl:386): 3 FTOL_REACHED, 4 XTOL_REACHED
 * (the Subplex / Nelder-Mead simplex collapsed), 5 MAXEVAL_REACHED.  With
 * optimizer 0 the descent reports 5 when it used max_evals and 4 when its
 * step vanished.  times_io is the best point and cost its objective (NLopt's
 * x and opt_f). */
int mtg_time_optimize_ex(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                         double* times_io, const mtg_time_params* params, int max_evals,
                         double* cost, int32_t* evals, int32_t* solves, int32_t* result,
                         int32_t* status, void* stream);

/* ------------------------------------------------------------------------
 * Free-derivative objectives of PolynomialOptimizationNonLinear (the NLopt
 * callbacks of kOptimizeFreeConstraints / kOptimizeFreeConstraintsAndTime),
 * for any constraint pattern of the plan (the fork's nonlinear class uses the
 * tube pattern: start/end fully fixed, every intermediate derivative free,
 * qcqp_impl:95-117).  params: time_penalty and the soft-constraint fields of
 * mtg_time_params (increment, w_d, w_t, grad_mode unused).
 *   mode 0  objectiveFunctionFreeConstraints (nonlinear_impl:1021-1113):
 *           J = J_d [+ soft], J_d = sum_dim d^T R d (getCostAndGradientDerivative,
 *           :1537-1606) = 2 computeCost(); grad (nullable) = dJ_d/dd_p =
 *           2 (R_pf d_f + R_pp d_p) per dimension (:1591-1592; the soft term
 *           is not differentiated, :1100-1110).
 *   mode 1  objectiveFunctionTimeAndConstraints (:947-1019): with the given
 *           times and d_p (no re-solve), J = computeCost() + time_penalty
 *           (sum T)^2 [+ soft]; no gradient (the reference CHECKs it empty).
 * Inputs (device): fixed_vals B x D x n_fixed, free_vals B x D x n_free
 * (dimension-major, the x layout of :1040-1052), times B x S.
 * Outputs (device, nullable): cost B, grad B x D x n_free (mode 0), status B.
 */
int mtg_free_cost(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                  const double* free_vals, const double* times,
                  const mtg_time_params* params, int mode, double* cost, double* grad,
                  int32_t* status, void* stream);

/* Batched optimisation of the free derivatives (optimizeFreeConstraints,
 * nonlinear_impl:399-493, objective of mode 0).  NLopt is not available; the
 * device optimiser takes projected Newton steps of the quadratic J_d,
 * d <- clamp(d + alpha (d* - d), lower, upper) with d* = argmin J_d from the
 * linear solve, alpha = 1, x1.5 (capped at 1) on a decrease of J, x0.5
 * otherwise, until `max_evals` objective evaluations or a step below
 * 1e-13 (1 + |d|).  lower / upper: B x D x n_free bounds
 * (setFreeEndpointDerivativeHardConstraints, :2858-2905) or NULL.
 *   free_io  B x D x n_free   in: initial d_p, out: optimised d_p
 *   cost     B                final objective; evals B (nullable) */
int mtg_free_optimize(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                      double* free_io, const double* times, const double* lower,
                      const double* upper, const mtg_time_params* params, int max_evals,
                      double* cost, int32_t* evals, int32_t* status, void* stream);

/* Batched optimisation over segment times AND free derivatives
 * (optimizeTimeAndFreeConstraints, nonlinear_impl:610-706, objective mode 1
 * of mtg_free_cost = objectiveFunctionTimeAndConstraints, :947-1019) with
 * the reference's bounds T in [0.1, 2 |T0|], d_p in [-2 |d0|, 2 |d0|]
 * (:660-677).  NLopt's SBPLX is not available; the device optimiser
 * alternates projected steps, each trial one counted evaluation: a scaled
 * steepest-descent step in T (central-difference gradient in T with d_p held,
 * step params->increment, clamp rule of :2529-2530, not counted) and a
 * Newton step of the quadratic J in d_p toward the linear solve at the
 * current T; step sizes x1.5 (capped at 1) on a decrease of J, x0.5
 * otherwise (T starts at 0.1, d_p at 1); stops at `max_evals` evaluations,
 * both steps below 1e-9, or a round in which neither moves.
 *   free_io   B x D x n_free   in: d0 (the start solution), out: optimised d_p
 *   times_io  B x S            in: T0, out: optimised times
 *   cost B, evals B, status B (nullable) */
int mtg_time_free_optimize(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                           double* free_io, double* times_io, const mtg_time_params* params,
                           int max_evals, double* cost, int32_t* evals, int32_t* status,
                           void* stream);
/* The same with params->optimizer selecting the optimiser and the stopping
 * reason per trajectory (result, B, nullable; nlopt_result codes):
 *   0  the block-alternating descent above (result 5 / 4 as the time
 *      optimiser's descent; not reported: result untouched);
 *   1  LN_SBPLX, the reference's own algorithm for this objective (the
 *      default, polynomial_optimization_nonlinear.h:61): NLopt's Subplex
 *      restated on the device over all S + D n_free variables (its state in
 *      LDS sized by that count), bounds as above, initial steps
 *      initial_stepsize_rel |x0| (:664-675), maxeval max_evals, ftol f_rel /
 *      f_abs.  free_io / times_io out = NLopt's x, cost = opt_f.  A start
 *      with a zero entry (NLopt rejects a zero initial step) or a time below
 *      0.1 returns result -1 (nlopt::FAILURE) with no evaluation and x
 *      unchanged.  `increment` is not used. */
int mtg_time_free_optimize_ex(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                              double* free_io, double* times_io, const mtg_time_params* params,
                              int max_evals, double* cost, int32_t* evals, int32_t* result,
                              int32_t* status, void* stream);

/* ------------------------------------------------------------------------
 * Tube QCQP (PolynomialOptimizationConstrained<N>, qcqp_impl).  The tube
 * pattern is fixed by the reference: start and end vertices fully fixed
 * (derivatives 0..M-1), every intermediate derivative free, including
 * positions (setupConstraintReorderingMatrixkDim, qcqp_impl:18-118); D = 3
 * (hard-coded in qcqp_impl:377-384, 777-781).
 *
 * Inputs (device), per trajectory:
 *   positions   B x (S+1) x 3   vertex positions (tube geometry)
 *   fixed_vals  B x 3 x N       start derivatives 0..M-1 then end
 *                               derivatives 0..M-1, per dimension
 *                               (fixed_constraints_compact_, qcqp_impl:48-65)
 *   times_cp    B x S           times for the Bezier control-point maps
 *                               (built once at setup, qcqp_impl:152-157)
 *   times       B x S           current segment times (Q, A^-1)
 *   radii       B x S x 2       (tube radius r1, sphere radius r2)
 *
 * mtg_tube_residuals evaluates the (S-1) + 3 S (N-2) inequality residuals
 * g_k(x) = 0.5 x^T Q_k x + l_k x + c_k (feasible iff <= 0) of
 * compute_sphere/tube/tube_end_constraints (qcqp_impl:357-474) at the free
 * vector x (B x 3 (S-1) M, dimension-major as qcqp_impl:95-117), in the
 * reference's constraint order.  resid: B x n_con.
 *
 * mtg_tube_solve replaces solveQCQP (qcqp_impl:476-788): minimise
 * x^T R_pp x + 2 d_f^T R_fp x subject to g_k(x) <= 0 with a batched
 * primal-dual interior-point method (MOSEK in the reference), then recover
 * coefficients (qcqp_impl:777-785).  Outputs: x B x 3(S-1)M, coeffs
 * B x S x 3 x N, cost B (computeCost), iters B, status B (nullable except
 * coeffs).  Where a time is not positive (MTG_TRAJ_BAD_TIME) x, coeffs and
 * cost are NaN.  Where R_pp is numerically singular (very long segments) the
 * interior-point method starts on the tube axis instead of at the
 * unconstrained minimiser (intermediate vertices at their positions, higher
 * derivatives zero); a KKT factorisation with a non-positive pivot is
 * retried once with a 1e-10 relative diagonal regularisation before the
 * solve stops (MTG_TRAJ_NOT_SPD when away from the optimum).  B < 2^26 (one 64-lane workgroup per
 * trajectory).
 */
int mtg_tube_num_constraints(int N, int S);
int mtg_tube_residuals(mtg_ctx* ctx, int N, int r, int S, int64_t B,
                       const double* positions, const double* fixed_vals,
                       const double* times_cp, const double* times,
                       const double* radii, const double* x, double* resid,
                       void* stream);
int mtg_tube_solve(mtg_ctx* ctx, int N, int r, int S, int64_t B,
                   const double* positions, const double* fixed_vals,
                   const double* times_cp, const double* times,
                   const double* radii, double tol, int max_iter, double* x,
                   double* coeffs, double* cost, int32_t* iters,
                   int32_t* status, void* stream);

/* Segment-time objective with the QCQP inner solve: the fork's
 * objectiveFunctionTime (nonlinear_impl:877-945), which calls solveQCQP()
 * after updateSegmentTimes (:891-892; mtg_time_cost is the upstream,
 * linear-inner form).  J = computeCost() of the QCQP solution at `times`
 * + time_penalty (sum T)^2 [+ soft, as mtg_time_cost]; the control-point
 * maps use `times_cp` (the times at setup, qcqp_impl:152-157).  J is NaN
 * where the QCQP breaks down (status MTG_TRAJ_NOT_SPD) or a time is not
 * positive.  grad_mode 0 (none; the reference callback is gradient-free) or
 * 2 (central differences of the re-solved J, clamp rule of :2525-2530; 2S
 * extra QCQP solves per trajectory, all in the same launch); grad_mode 1 is
 * MTG_ERR_UNSUPPORTED.  tol / max_iter as mtg_tube_solve.  Outputs
 * (device): cost B, grad B x S (grad_mode 2), status B (nullable; the
 * QCQP status at `times`).
 *
 * Scratch: `workspace` is a caller-owned device buffer of at least
 * mtg_tube_time_workspace_bytes(N, S, B, params, 0) bytes (optimize = 1
 * for mtg_tube_time_optimize), used for the duration of the stream's work.
 * Neither call allocates or synchronises, so both can be captured in a HIP
 * graph.  The query returns < 0 (MTG_ERR_INVALID_ARG) for invalid sizes or
 * when B x (2S+1) problems would exceed one launch's grid (2^26 problems). */
int64_t mtg_tube_time_workspace_bytes(int N, int S, int64_t B,
                                      const mtg_time_params* params, int optimize);
int mtg_tube_time_cost(mtg_ctx* ctx, int N, int r, int S, int64_t B,
                       const double* positions, const double* fixed_vals,
                       const double* times_cp, const double* times, const double* radii,
                       double tol, int max_iter, const mtg_time_params* params,
                       double* cost, double* grad, int32_t* status,
                       void* workspace, size_t workspace_bytes, void* stream);

/* Batched segment-time optimisation over that objective (optimizeTime,
 * nonlinear_impl:332-397, in the fork's QCQP form), bounds [0.1, 2 T0],
 * max_evals counted evaluations.  params->optimizer selects the optimiser as
 * in mtg_time_optimize:
 *   1  LN_SBPLX, the reference's default (polynomial_optimization_nonlinear.h
 *      :61): NLopt's Subplex restated on the device (mtg_sbplx_device.h) on
 *      objectiveFunctionTime with solveQCQP() at every evaluation (:891-892),
 *      initial steps initial_stepsize_rel T0, ftol f_rel / f_abs.  Each round
 *      is one tube launch over B problems (one evaluation per trajectory);
 *      times_io is NLopt's x (the best point) and cost its value (opt_f).  A
 *      T0 below 0.1 is NLopt's invalid start: result -1 (nlopt::FAILURE, as
 *      optimizeTime returns it), no evaluation, times unchanged, cost NaN.
 *   0  the projected, scaled steepest descent of mtg_time_optimize on the
 *      grad_mode 2 gradient, stopping also at a non-finite gradient; each
 *      round is one tube launch over B x (2S+1) problems (every trial with
 *      its gradient points).
 * The call enqueues max_evals rounds; a trajectory that has stopped is
 * skipped by every later round on the device (its QCQP workgroups exit at
 * once), so there is no host round trip.
 *   times_io  B x S  in: T0 (also the control-point times), out: optimised
 *   cost B, evals B, status B (nullable); workspace as above (optimize = 1,
 *   with the same params: the LN_SBPLX workspace holds the machine states).
 * The _ex form adds result (B, nullable): the nlopt_result code as in
 * mtg_time_optimize_ex. */
int mtg_tube_time_optimize(mtg_ctx* ctx, int N, int r, int S, int64_t B,
                           const double* positions, const double* fixed_vals,
                           const double* radii, double* times_io, double tol, int max_iter,
                           const mtg_time_params* params, int max_evals, double* cost,
                           int32_t* evals, int32_t* status, void* workspace,
                           size_t workspace_bytes, void* stream);
int mtg_tube_time_optimize_ex(mtg_ctx* ctx, int N, int r, int S, int64_t B,
                              const double* positions, const double* fixed_vals,
                              const double* radii, double* times_io, double tol, int max_iter,
                              const mtg_time_params* params, int max_evals, double* cost,
                              int32_t* evals, int32_t* result, int32_t* status, void* workspace,
                              size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Batched trajectory sampling: Trajectory::evaluateRange (src/trajectory.cpp:
 * 74-134) for derivatives 0..max_derivative at once (the [t, p, v, a, j, s]
 * rows of printMatlabSampledTrajectory, nonlinear_impl:2907-3003).
 * Per trajectory b: samples start in the segment containing t_start, at
 * time-in-segment t_start - (segment start) + k dt, advancing to the next
 * segment while the time exceeds the segment time; they run while the
 * accumulated time (segment start + k dt) is < t_end, and stop at the first
 * sample past the last segment.  t_end < 0 means the trajectory's total time.
 * Device pointers: coeffs B x S x D x N (as mtg_linear_solve writes them),
 * times B x S; outputs samples B x ((max_derivative+1) * D) x n_max
 * (channel-major: channel = derivative * D + d), sample_times B x n_max (the
 * accumulated times, nullable), n_samples B (nullable).  Samples beyond
 * n_max are dropped.  1 <= S <= 64.  An n_max that is a multiple of 64 keeps
 * every channel row 512-byte aligned (full-line HBM writes).
 */
int mtg_sample_trajectories(int N, int D, int S, int64_t B, const double* coeffs,
                            const double* times, double t_start, double t_end,
                            double dt, int n_max, int max_derivative,
                            double* samples, double* sample_times,
                            int32_t* n_samples, void* stream);

/* ------------------------------------------------------------------------
 * Batched magnitude extrema: PolynomialOptimization::computeMaximumOfMagnitude
 * (polynomial_optimization_linear_impl.h:455-487, with
 * Segment::computeMinMaxMagnitudeCandidateTimes, src/segment.cpp:82-133, and
 * the candidate rules of Polynomial::selectMinMaxCandidatesFromRoots,
 * src/polynomial.cpp:32-63).  For each trajectory b: the maximum over all
 * segments s and t in [0, T_s] of |p_s^(derivative)(t)| (Euclidean norm over
 * the D dimensions), attained at t = 0, T_s or a real root of
 * d/dt |p^(derivative)|^2.  Outputs (device, each nullable): max_time B
 * (time relative to the segment start, Extremum::time), max_value B,
 * max_segment B.  Ties keep the first candidate in the reference's order
 * (segment ascending).  0 <= derivative <= 4 (POSITION..SNAP) and
 * derivative <= N - 2 (linear_impl:400); 1 <= S <= 256.  The reference's
 * optional candidate list is not produced.
 */
int mtg_max_magnitude(int N, int D, int S, int64_t B, const double* coeffs,
                      const double* times, int derivative, double* max_time,
                      double* max_value, int32_t* max_segment, void* stream);

/* The candidate lists behind those extrema: for every segment s of every
 * trajectory b, the candidates of Segment::computeMinMaxMagnitudeCandidates
 * (src/segment.cpp:82-161, all D dimensions; PolynomialOptimization::
 * computeSegmentMaximumMagnitudeCandidates, linear_impl:395-409, and the
 * optional candidate list of computeMaximumOfMagnitude, linear_impl:455-487):
 * t = 0, t = T_s, then the real roots in [0, T_s] of
 * f = sum_d p_d^(derivative) p_d^(derivative+1) ascending (for D = 1 the
 * roots of p^(derivative+1) alone, segment.cpp:123-129), each with
 * |p^(derivative)(t)| (Euclidean norm over D).  Roots are isolated by
 * Bernstein subdivision and refined as in mtg_max_magnitude; a multiple root
 * is listed once (the reference's RPOLY lists a multiple root's cluster, of
 * which its |Im| > DBL_EPSILON test keeps 0..m copies), and a root at
 * exactly t = 0 or t = T_s only as the endpoint.  Outputs (device):
 * cand_time / cand_value [B][S][max_candidates] (times relative to the
 * segment start), n_candidates [B][S] = the number of candidates found (if
 * it exceeds max_candidates only the first max_candidates are stored; 2 +
 * the degree of f, i.e. 2 (N - derivative) - 1, always suffices).  A
 * segment with T_s < 0 or NaN has none (the reference's t_start > t_end
 * warning).  0 <= derivative <= 4, derivative <= N - 2, max_candidates >= 2. */
int mtg_magnitude_candidates(int N, int D, int S, int64_t B, const double* coeffs,
                             const double* times, int derivative, int max_candidates,
                             double* cand_time, double* cand_value, int32_t* n_candidates,
                             void* stream);

/* Minimum and maximum of the magnitude: Trajectory::computeMinMaxMagnitude
 * (src/trajectory.cpp:184-220, candidates of Segment::
 * computeMinMaxMagnitudeCandidates, src/segment.cpp:82-161) over all D
 * dimensions of the coefficients given (a caller selecting dimensions passes
 * only those).  Same candidate search as mtg_max_magnitude; the minimum is
 * the first candidate with the smallest |p^(derivative)| (strict '<' from
 * +max in segment order, trajectory.cpp:201-214).  For D = 1 the candidates
 * include the zeros of p^(derivative) (the real minimum of |p|), where the
 * reference takes only the roots of p^(derivative+1) (segment.cpp:123-129),
 * so a 1-D minimum can be lower than the reference's; maxima agree.  Outputs
 * (device, each nullable): min_time / max_time B (relative to the segment
 * start), min_value / max_value B, min_segment / max_segment B. */
int mtg_min_max_magnitude(int N, int D, int S, int64_t B, const double* coeffs,
                          const double* times, int derivative, double* min_time,
                          double* min_value, int32_t* min_segment, double* max_time,
                          double* max_value, int32_t* max_segment, void* stream);

/* Soft-constraint cost of PolynomialOptimizationNonLinear
 * (evaluateMaximumMagnitudeAsSoftConstraint, nonlinear_impl:2735-2766; the
 * constraints of addMaximumMagnitudeConstraint, :847-875):
 *   cost_b = sum_c min(maximum_cost, exp((max_bc - limit_c) / limit_c * weight)).
 * derivatives and limits are HOST arrays of n_constraints (1..8) entries;
 * maxima (device, B x n_constraints) receives max_bc; cost (device, B).
 * Reference defaults: weight = soft_constraint_weight = 100
 * (polynomial_optimization_nonlinear.h:64), maximum_cost = 1e12 (:576). */
int mtg_soft_constraint_cost(int N, int D, int S, int64_t B, const double* coeffs,
                             const double* times, int n_constraints, const int* derivatives,
                             const double* limits, double weight, double maximum_cost,
                             double* maxima, double* cost, void* stream);

/* ------------------------------------------------------------------------
 * Collision cost over an occupancy map: getCostAndGradientCollision
 * (nonlinear_impl:1609-1780) with getCostAndGradientPotentialOctree
 * (:1782-1917), the nearest-occupied-voxel search of findOccupiedVoxels /
 * getDistanceOctree (:1920-2043) and getCostPotential (:2660-2684).  The
 * reference reads a supereight octree (absent; parity unpinned); here the
 * map is a caller-supplied dense grid `occupancy` (device, nx*ny*nz floats,
 * voxel (x, y, z) at (z*ny + y)*nx + x, occupied iff the log-odds value is
 * >= 0; voxels outside the grid are free).  A position maps to voxel
 * (position / map_resolution) truncated toward zero (:1815).
 * Per trajectory (D = 3): sample every coll_check_time_increment from each
 * segment's start; once the path length since the last evaluation reaches
 * map_resolution, add c(p) |v| time_sum, c = getCostPotential(distance to
 * the nearest occupied voxel in the box_side^3 box around p - robot_radius).
 * A collision (that distance <= 0, or p within one voxel of
 * [min_bound, max_bound]) stops the walk: cost 0, collision 1, zero
 * gradient.  Outputs (device, each nullable): cost B, collision B,
 * grad_coeffs B x S x 3 x N (dJ_c/dc, the eq. (14) terms per coefficient),
 * grad_free B x 3 x n_free (dJ_c/dd_p through L = A^-1 M, :1650-1656).
 * coeffs B x S x 3 x N and times B x S as mtg_linear_solve writes them. */
typedef struct mtg_collision_params {
  double map_resolution;            /* ::map_resolution (voxel edge, m) */
  double min_bound[3], max_bound[3]; /* ::min_bound / ::max_bound (m) */
  double epsilon;                   /* ::epsilon (0.5) obstacle clearance */
  double robot_radius;              /* ::robot_radius (0.5) */
  double coll_pot_multiplier;       /* ::coll_pot_multiplier (1.0) */
  double coll_check_time_increment; /* ::coll_check_time_increment (0.1) */
  int box_side;                     /* findOccupiedVoxels side (20, :1797) */
} mtg_collision_params;
int mtg_collision_cost(const mtg_plan* plan, int64_t B, const double* coeffs,
                       const double* times, const float* occupancy, int nx, int ny, int nz,
                       const mtg_collision_params* params, double* cost, int32_t* collision,
                       double* grad_coeffs, double* grad_free, void* stream);

/* ------------------------------------------------------------------------
 * Collision-driven objectives of PolynomialOptimizationNonLinear: the
 * reference demo's path (src/main.cpp:77, 104-105: kOptimizeFreeConstraints
 * AndCollision with NLopt LD_LBFGS).
 *   mode 0  objectiveFunctionFreeConstraintsAndCollision
 *           (nonlinear_impl:1115-1272), x = d_p (D x n_free, dimension-major,
 *           the x layout of :1130-1141), segment times from `times`;
 *   mode 1  objectiveFunctionFreeConstraintsAndCollisionAndTime
 *           (:1274-1535), x = [T (S); d_p (D x n_free)].
 * J = w_d J_d + w_c J_c + w_t J_t (mode 1) + w_sc J_sc with
 *   J_d  = sum_dim d^T R d (getCostAndGradientDerivative, :1537-1606),
 *          gradient 2 (R_pf d_f + R_pp d_p);
 *   J_c  = the collision walk of mtg_collision_cost (:1609-1780) with its
 *          eq. (14) gradient through L = A^-1 M; on a collision J_c = 0 and
 *          the gradient keeps the terms accumulated before it (the
 *          reference's zeroing loop at :1773-1777 works on copies);
 *   J_sc = evaluateMaximumMagnitudeAsSoftConstraint (:2735-2766) when
 *          n_soft > 0, gradient by central differences over every free
 *          variable with step coll.map_resolution
 *          (getCostAndGradientSoftConstraints, :2365-2432; mode 1 with
 *          simple_numgrad_constraints: forward differences,
 *          getCostAndGradientSoftConstraintsSimple :2434-2493);
 *   J_t  = sum T (mode 1; getCostAndGradientTime :2495-2584): gradient
 *          w_d dJ_d/dT_n + w_c dJ_c/dT_n + w_sc dJ_sc/dT_n + w_t by central
 *          (forward with simple_numgrad_time, :2586-2657) differences with
 *          step increment_time and the 0.1 clamp of :2529-2530, d held
 *          fixed; the perturbed J_c walks the coefficients of T over the
 *          perturbed segment times (L_ is not refreshed there) and dJ_sc/dT
 *          is 0 (updateSegmentTimes leaves the segments that
 *          computeMaximumOfMagnitude reads unchanged).
 * When the walk at x collides, J_d, J_sc and J_t are not evaluated (0, zero
 * gradients, :1171-1178) and with is_collision_safe the collision term is
 * raised so that J = raise_ref + add_coll_raise (:1207-1226); raise_ref is
 * the caller's total_cost_iter0_ (is_coll_raise_first_iter) or the previous
 * evaluation's total (NULL: 0, the reference's initial values).  Collisions
 * of the perturbed-time walks are ignored (J_c = 0 there; the reference
 * dereferences a null gradient vector in that case, :1773-1777).
 * terms (B x 4, nullable): w_d J_d, w_c J_c (after the raise), w_t J_t,
 * w_sc J_sc (OptimizationInfo cost_trajectory / collision / time /
 * soft_constraints).
 *
 * mtg_coll_optimize replaces the NLopt run of optimizeFreeConstraintsAnd
 * Collision (:495-607) / ...AndCollisionAndTime (:708-845): NLopt is absent,
 * and LD_LBFGS is replaced by a batched projected L-BFGS run on the device
 * (memory lbfgs_memory pairs; first direction -g scaled so its largest
 * entry moves max(initial_step); backtracking by safeguarded quadratic
 * interpolation on the Armijo condition, c1 = 1e-4, every trial one counted
 * evaluation; stops at max_evals evaluations (NLopt maxeval), NLopt's
 * ftol / xtol tests on an accepted step, or a projected gradient of zero).
 * The collision raise state follows the reference: total_cost_iter0_ is the
 * first evaluation's J, the "last iteration" is the previous evaluation.
 *   x_io          B x nx   in: start point, out: best point found
 *   lower, upper  B x nx   bounds (nullable: unbounded)
 *   initial_step  B x nx   NLopt initial step (nullable: 0.1 |x0|)
 *   cost B, evals B, result B (NLopt codes: 1 SUCCESS, 3 FTOL_REACHED,
 *   4 XTOL_REACHED, 5 MAXEVAL_REACHED, -1 FAILURE), status B (MTG_TRAJ_*),
 *   terms B x 4 (at the best point) — all nullable.
 * The optimiser enqueues max_evals rounds of a few launches; finished
 * trajectories are skipped on the device, nothing synchronises with the host
 * and nothing is allocated: scratch is the caller's `workspace` of at least
 * mtg_coll_workspace_bytes(plan, B, mode, params, optimize) bytes.
 * Requirements: D = 3 (the collision cost, :1796-1797), 1 <= n_free,
 * lbfgs_memory 1..16, n_soft 0..8; times > 0.
 */
typedef struct mtg_coll_params {
  mtg_collision_params coll;      /* map, potential and sampling parameters */
  double w_d, w_c, w_t, w_sc;     /* ::weights (0.1, 10, 1, 1) */
  int is_collision_safe;          /* ::is_collision_safe (1) */
  int is_coll_raise_first_iter;   /* ::is_coll_raise_first_iter (1) */
  double add_coll_raise;          /* ::add_coll_raise (0) */
  int simple_numgrad_time;        /* ::is_simple_numgrad_time (mode 1) */
  int simple_numgrad_constraints; /* ::is_simple_numgrad_constraints (mode 1) */
  double increment_time;          /* ::increment_time (0.1) */
  int n_soft;                     /* soft magnitude constraints 0..8 */
  int soft_derivative[8];         /* derivative order of constraint c, 0..4 */
  double soft_limit[8];           /* maximum_value of constraint c, > 0 */
  double soft_weight;             /* ::soft_constraint_weight (100) */
  double soft_maximum_cost;       /* 1e12 */
  double f_rel, f_abs, x_rel, x_abs; /* NLopt stopping tests (<= 0: off) */
  int lbfgs_memory;               /* history pairs (10) */
} mtg_coll_params;

/* Near field of an occupancy map for the collision walk.  For every voxel v
 * of the nx x ny x nz grid, 8 uint16 (7 used): the squared voxel distances
 * from v and from its 6 axis neighbours to the nearest occupied voxel of the
 * box_side^3 box the walk searches around v (0xFFFF: none) — the minima of
 * getCostAndGradientPotentialOctree's search (nonlinear_impl:1782-2018), so
 * a walk that reads them instead of scanning the box gives identical
 * results (the scan remains for samples whose voxel lies outside the grid).
 * It depends only on the occupancy and params->box_side: compute it once
 * per map (mtg_coll_field_bytes(nx, ny, nz) bytes, device) and pass it as
 * `near_field` to mtg_coll_cost / mtg_coll_optimize, whose walk then runs on
 * one thread per walk with one load per evaluated sample instead of a
 * workgroup-wide box scan and reduction per sample.  box_side <= 31. */
int64_t mtg_coll_field_bytes(int nx, int ny, int nz);
int mtg_coll_field(const float* occupancy, int nx, int ny, int nz,
                   const mtg_collision_params* params, uint16_t* field, void* stream);

int64_t mtg_coll_workspace_bytes(const mtg_plan* plan, int64_t B, int mode,
                                 const mtg_coll_params* params, int optimize);
/* near_field: mtg_coll_field of the same occupancy and box_side, or NULL
 * (every sample's box is scanned). */
int mtg_coll_cost(const mtg_plan* plan, int64_t B, int mode, const double* fixed_vals,
                  const double* x, const double* times, const float* occupancy, int nx,
                  int ny, int nz, const uint16_t* near_field, const mtg_coll_params* params,
                  const double* raise_ref,
                  double* cost, double* grad, double* terms, int32_t* collision,
                  int32_t* status, void* workspace, size_t workspace_bytes, void* stream);
int mtg_coll_optimize(const mtg_plan* plan, int64_t B, int mode, const double* fixed_vals,
                      double* x_io, const double* times, const double* lower,
                      const double* upper, const double* initial_step, const float* occupancy,
                      int nx, int ny, int nz, const uint16_t* near_field,
                      const mtg_coll_params* params, int max_evals,
                      double* cost, int32_t* evals, int32_t* result, int32_t* status,
                      double* terms, void* workspace, size_t workspace_bytes, void* stream);
/* mtg_coll_optimize with the evaluation history the reference keeps in
 * all_trajectories_ (one trajectory pushed per objective evaluation,
 * nonlinear_impl:1244, 1482; read by getAllTrajectories,
 * polynomial_optimization_nonlinear.h:316-331): x_history (device,
 * nullable) B x max_evals x nv doubles, where nv is the number of
 * optimisation variables (NOT the grid's nx): nv = D * n_free in mode 0
 * (x = d_p), S + D * n_free in mode 1 (x = [T; d_p]), n_free from
 * mtg_plan_counts.  Row k = the point of the (k+1)-th counted evaluation;
 * rows at or past evals[b] are not written. */
int mtg_coll_optimize_trace(const mtg_plan* plan, int64_t B, int mode, const double* fixed_vals,
                            double* x_io, const double* times, const double* lower,
                            const double* upper, const double* initial_step,
                            const float* occupancy, int nx, int ny, int nz,
                            const uint16_t* near_field, const mtg_coll_params* params,
                            int max_evals, double* cost, int32_t* evals, int32_t* result,
                            int32_t* status, double* terms, double* x_history, void* workspace,
                            size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Selection for the multi-GPU path (BASELINE config 4: the
 * shards solve independently and the ranks all-gather costs for
 * selection).  mtg_select_local reduces rank `rank`'s shard of `count`
 * costs (device), global indices start .. start+count-1, to the triple
 * out[3] = (cost, global index, rank) (device): NaN never wins, the lowest
 * index wins ties, an empty shard gives (+inf, -1, rank), all NaN / +inf
 * gives the shard's first index.  After the caller all-gathers the triples
 * (RCCL, 24 B per rank, rank order), mtg_select_global picks the winner of
 * `world` triples into out[3]: smallest cost, first rank on ties, empty
 * shards and NaN last, the first triple if none is finite.  One launch
 * each, stream-ordered, graph-capturable. */
int mtg_select_local(const double* costs, int64_t count, int64_t start, int rank, double* out,
                     void* stream);

/* The solve and the shard's selection: mtg_linear_solve, then
 * mtg_select_local's triple (cost, start + index, rank) in `triple` (device,
 * 3 doubles), with the same ordering rules.  The lane kernels write each
 * workgroup's best (cost, index) in their epilogue and one single-workgroup
 * launch reduces those partials; the wavefront kernels (one trajectory per
 * workgroup) are followed by the same reduction over the costs.  Two
 * stream-ordered launches, no atomics, graph-capturable.  `cost` must be
 * non-NULL.  workspace: caller-owned device memory of at least
 * mtg_select_workspace_bytes(plan, B) bytes (0 for the wavefront kernels;
 * NULL allowed then), no initialisation; one solve at a time may use it.  A
 * step of the multi-GPU path is then this call, the RCCL all-gather of the
 * triples, and mtg_select_global. */
int64_t mtg_select_workspace_bytes(const mtg_plan* plan, int64_t B);
int mtg_linear_solve_select(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                            const double* times, double* coeffs, double* cost,
                            double* free_vals, int32_t* status, int64_t start, int rank,
                            double* triple, void* workspace, size_t workspace_bytes,
                            void* stream);
int mtg_select_global(const double* triples, int world, double* out, void* stream);

/* The pipelined step (round 5): this step's solve (mtg_linear_solve) with
 * the PREVIOUS step's shard selection -- mtg_select_local of prev_cost
 * (device, prev_count costs, global indices prev_start ..) into prev_triple
 * (device, 3 doubles) -- in the same launch: the wave and lane-pair kernels
 * run it in one extra workgroup beside the solves, the others as a launch of
 * their own first.  prev_cost NULL: the plain solve.  prev_cost must not
 * alias this step's cost (alternate two output sets).  The selection never
 * feeds a solve, so it costs no launch on the step's critical path
 * (mav_tube_trajectory_generation_amd/shard.py SelectionPipeline). */
int mtg_linear_solve_select_prev(const mtg_plan* plan, int64_t B, const double* fixed_vals,
                                 const double* times, double* coeffs, double* cost,
                                 double* free_vals, int32_t* status, const double* prev_cost,
                                 int64_t prev_count, int64_t prev_start, int rank,
                                 double* prev_triple, void* stream);
/* The per-step winners of G steps at once: triples = the all-gather of every
 * rank's G triples (world x G x 3, rank-major), out = n x 3 (device), step
 * g's winner by mtg_select_global's rule, for g < n <= G. */
int mtg_select_global_steps(const double* triples, int world, int G, int n, double* out,
                            void* stream);

/* ------------------------------------------------------------------------
 * Host-side input generation (vertex.cpp:27-82, 228-269) for batches:
 * trajectory b uses createRandomVertices(max_derivative = M-1, S, +/-pos_bound,
 * seed = seed0 + b) and estimateSegmentTimes(v_max, a_max) (Nfabian, 6.5).
 * Writes the standard pattern's fixed_vals (B x D x n_fixed, n_fixed =
 * 2 M + (S-1)) and times (B x S); positions (B x (S+1) x D) nullable.
 * Bit-identical to the reference generator (std::mt19937 +
 * std::uniform_real_distribution<double> of libstdc++).
 */
int mtg_generate_random_problems(int N, int D, int S, int64_t B,
                                 uint64_t seed0, double pos_bound,
                                 double v_max, double a_max,
                                 uint8_t* fixed_mask /* (S+1)*M */,
                                 double* fixed_vals, double* times,
                                 double* positions);

#ifdef __cplusplus
}
#endif

#endif /* MTG_HIP_H_ */
