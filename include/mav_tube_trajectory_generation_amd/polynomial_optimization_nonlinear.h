// polynomial_optimization_nonlinear.h — PolynomialOptimizationNonLinear<N>,
// the segment-time optimisation of the reference
// (include/mav_tube_trajectory_generation/polynomial_optimization_nonlinear.h:
// 46-674, impl/polynomial_optimization_nonlinear_impl.h "nonlinear_impl"),
// restricted to the objectives on the hot path (SURVEY.md §8a T1-T6 and §8f
// rank 2): kOptimizeTime with the time-only cost callback
//   J(T) = computeCost() + time_penalty * (sum_i T_i)^2
// (objectiveFunctionTime, nonlinear_impl:877-945, w_c = 0, optional soft
// magnitude constraints).  Both the callback (evaluateTimeCost -> mtg_time_cost) and
// the whole optimisation loop (optimize -> mtg_time_optimize) run on the
// device.
//
// Semantics and deliberate differences:
//   * inner solve = the tube QCQP, as the fork does (solveQCQP in
//     objectiveFunctionTime, nonlinear_impl:892; mtg_tube_time_cost /
//     mtg_tube_time_optimize_ex) by default (round 6).  The build's
//     extension field `solve_time_with_qcqp = false` selects the linear solve
//     with the vertices' own constraint pattern instead (upstream
//     mav_trajectory_generation semantics; mtg_time_cost /
//     mtg_time_optimize_ex);
//   * NLopt (LN_SBPLX, nonlinear_impl:95-107) is absent.  kOptimizeTime with
//     the default algorithm LN_SBPLX runs the device restatement of NLopt's
//     Subplex (optimizer 1: bounds [0.1, 2 T0], :350-378, initial step
//     initial_stepsize_rel T0, maxeval max_iterations, :101, ftol f_rel /
//     f_abs, :97-98) over either inner solve, and
//     kOptimizeFreeConstraintsAndTime runs it over [T; d_p]
//     (mtg_time_free_optimize_ex); any other algorithm runs the projected
//     descents (optimizer 0).  NLopt itself is absent, so optimiser parity is
//     pinned to the oracle restatement only; the callback
//     value is pinned;
//   * the collision cost reads a dense occupancy grid (setOccupancyGrid) in
//     place of the supereight octree (setOctree).  kOptimizeFreeConstraints
//     AndCollision and kOptimizeFreeConstraintsAndCollisionAndTime (the
//     reference demo, src/main.cpp:77) run on the device (mtg_coll_optimize:
//     a batched projected L-BFGS in place of NLopt's LD_LBFGS, parity
//     unpinned); the time-only and free-derivative objectives ignore w_c
//     with a warning, as the reference's objectiveFunctionTime would
//     dereference a null octree there (§8a T6);
//   * addMaximumMagnitudeConstraint with use_soft_constraints (the default)
//     adds the soft cost of evaluateMaximumMagnitudeAsSoftConstraint
//     (:2735-2766) to the objective, evaluated on the device after every
//     inner solve (extremum search of mtg_max_magnitude); at most 8
//     constraints, derivatives POSITION..SNAP.  With use_soft_constraints =
//     false they are the NLopt inequality constraints of :861-872
//     (max |p^(k)| - value <= inequality_constraint_tolerance,
//     evaluateMaximumMagnitudeConstraint, :2687-2733): kOptimizeTime's
//     device optimiser then accepts only feasible improving trials
//     (feasibility first from an infeasible start, mtg_time_params
//     hard_constraints); the other objectives' device optimisers ignore hard
//     constraints with a warning.  As in the reference, the constraint is
//     only registered as an NLopt inequality when the selected algorithm
//     takes one (addMaximumMagnitudeConstraint returns false otherwise, e.g.
//     for the default LN_SBPLX, and the constraint then has no effect).
#ifndef MAV_TUBE_TRAJECTORY_GENERATION_AMD_POLYNOMIAL_OPTIMIZATION_NONLINEAR_H_
#define MAV_TUBE_TRAJECTORY_GENERATION_AMD_POLYNOMIAL_OPTIMIZATION_NONLINEAR_H_

#include <algorithm>
#include <chrono>
#include <cmath>
#include <fstream>
#include <map>
#include <ostream>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "mav_tube_trajectory_generation_amd/polynomial_optimization_qcqp.h"

// The NLopt names the reference's parameters and return codes use
// (nlopt.hpp is absent: only the enumerations, in NLopt's numbering, so that
// code such as main.cpp:104-105 `static_cast<nlopt::algorithm>(11)` and
// comparisons with nlopt::MAXEVAL_REACHED compile unchanged).
namespace nlopt {
enum algorithm {
  GN_DIRECT = 0, GN_DIRECT_L, GN_DIRECT_L_RAND, GN_DIRECT_NOSCAL, GN_DIRECT_L_NOSCAL,
  GN_DIRECT_L_RAND_NOSCAL, GN_ORIG_DIRECT, GN_ORIG_DIRECT_L, GD_STOGO, GD_STOGO_RAND,
  LD_LBFGS_NOCEDAL, LD_LBFGS, LN_PRAXIS, LD_VAR1, LD_VAR2, LD_TNEWTON, LD_TNEWTON_RESTART,
  LD_TNEWTON_PRECOND, LD_TNEWTON_PRECOND_RESTART, GN_CRS2_LM, GN_MLSL, GD_MLSL, GN_MLSL_LDS,
  GD_MLSL_LDS, LD_MMA, LN_COBYLA, LN_NEWUOA, LN_NEWUOA_BOUND, LN_NELDERMEAD, LN_SBPLX,
  LN_AUGLAG, LD_AUGLAG, LN_AUGLAG_EQ, LD_AUGLAG_EQ, LN_BOBYQA, GN_ISRES, AUGLAG, AUGLAG_EQ,
  G_MLSL, G_MLSL_LDS, LD_SLSQP, LD_CCSAQ, GN_ESCH, GN_AGS, NUM_ALGORITHMS
};
enum result {
  FAILURE = -1, INVALID_ARGS = -2, OUT_OF_MEMORY = -3, ROUNDOFF_LIMITED = -4, FORCED_STOP = -5,
  SUCCESS = 1, STOPVAL_REACHED = 2, FTOL_REACHED = 3, XTOL_REACHED = 4, MAXEVAL_REACHED = 5,
  MAXTIME_REACHED = 6
};
// Algorithms that accept inequality constraints (NLopt's add_inequality_
// constraint throws for the others).
inline bool takesInequalityConstraints(algorithm a) {
  switch (a) {
    case GN_ORIG_DIRECT: case GN_ORIG_DIRECT_L: case LD_MMA: case LN_COBYLA: case LN_AUGLAG:
    case LD_AUGLAG: case LN_AUGLAG_EQ: case LD_AUGLAG_EQ: case GN_ISRES: case AUGLAG:
    case AUGLAG_EQ: case LD_SLSQP: case LD_CCSAQ: case GN_AGS:
      return true;
    default:
      return false;
  }
}
}  // namespace nlopt

namespace mav_trajectory_generation {

// polynomial_optimization_nonlinear.h:46-210 (fields kept for source
// compatibility; the ones this build reads are marked).
struct NonlinearOptimizationParameters {
  enum OptimizationObjective {
    kOptimizeFreeConstraints,
    kOptimizeFreeConstraintsAndTime,
    kOptimizeTime,
    kOptimizeFreeConstraintsAndCollision,
    kOptimizeFreeConstraintsAndCollisionAndTime,
    kUnknown
  };
  struct cost_weights {
    cost_weights() : w_d(0.1), w_c(10.0), w_t(1.0), w_sc(1.0) {}
    double w_d;  // read (gradient mode 1)
    double w_c;
    double w_t;  // read (gradient mode 1)
    double w_sc;
  };

  double f_abs = -1;
  double f_rel = 0.05;
  double x_rel = -1;
  double x_abs = -1;
  double initial_stepsize_position = 0.05;
  double initial_stepsize_rel = 0.1;  // the device optimiser uses the default 0.1
  double equality_constraint_tolerance = 1.0e-3;
  double inequality_constraint_tolerance = 0.1;
  int max_iterations = 5;  // read: objective-evaluation budget
  double max_time = -1;
  double time_penalty = 500.0;  // read
  nlopt::algorithm algorithm = nlopt::LN_SBPLX;  // read: whether hard constraints are taken
  int random_seed = 0;
  bool use_soft_constraints = true;
  double soft_constraint_weight = 100.0;
  bool print_debug_info = false;
  OptimizationObjective objective = kOptimizeFreeConstraintsAndTime;  // read
  cost_weights weights;
  double map_resolution = 0.0;
  int side = 5;
  // Map bounds on the intermediate positions (read by the hard bounds of
  // kOptimizeFreeConstraints, nonlinear_impl:2876-2887; Eigen::Vector3d there).
  VectorXd min_bound = VectorXd::Zero(3);
  VectorXd max_bound = VectorXd::Zero(3);
  bool use_numeric_grad = false;
  // Build extension (not in the reference struct): kOptimizeTime's callback
  // re-solves the tube QCQP, as the fork does (solveQCQP in
  // objectiveFunctionTime, nonlinear_impl:892; the default, round 6), or
  // with false the linear problem (upstream mav_trajectory_generation
  // semantics, far cheaper).  Read.
  bool solve_time_with_qcqp = true;
  bool use_continous_distance = false;
  double increment_time = 0.1;  // read (gradient step)
  double epsilon = 0.5;
  double robot_radius = 0.5;
  double coll_pot_multiplier = 1.0;
  bool solve_with_position_constraint = false;
  bool is_collision_safe = true;
  bool is_simple_numgrad_time = false;
  bool is_simple_numgrad_constraints = false;
  double coll_check_time_increment = 0.1;
  bool is_coll_raise_first_iter = true;
  double add_coll_raise = 0.0;
  double use_esdf = 0.0;
  // Build extension: history pairs of the device L-BFGS that stands in for
  // NLopt's LD_LBFGS in the collision objectives.
  int lbfgs_memory = 10;
};

// polynomial_optimization_nonlinear.h:212-236.
class OptimizationInfo {
 public:
  void print(std::ostream& stream) const {
    stream << "--- optimization info ---" << std::endl;
    stream << "  optimization time:     " << optimization_time << std::endl;
    stream << "  n_iterations:          " << n_iterations << std::endl;
    stream << "  stopping reason:       " << stopping_reason << std::endl;
    stream << "  cost trajectory:       " << cost_trajectory << std::endl;
    stream << "  cost time:             " << cost_time << std::endl;
    stream << "  cost collision:        " << cost_collision << std::endl;
    stream << "  cost soft constraints: " << cost_soft_constraints << std::endl;
  }
  int n_iterations = 0;
  int stopping_reason = -1;  // nlopt::FAILURE
  double cost_trajectory = 0;
  double cost_collision = 0;
  double cost_time = 0;
  double cost_soft_constraints = 0;
  double optimization_time = 0;
  std::map<int, Extremum> maxima;  // per constrained derivative, after optimize()
};

template <int _N = 10>
class PolynomialOptimizationNonLinear {
  static_assert(_N % 2 == 0, "The number of coefficients has to be even.");

 public:
  enum { N = _N };

  PolynomialOptimizationNonLinear(size_t dimension,
                                  const NonlinearOptimizationParameters& parameters)
      : dimension_(dimension), params_(parameters), poly_opt_(dimension), linear_(dimension) {}

  // nonlinear_impl:57-110.
  bool setupFromVertices(const Vertex::Vector& vertices,
                         const std::vector<double>& segment_times,
                         const std::vector<std::pair<double, double>>& radii,
                         int derivative_to_optimize =
                             PolynomialOptimization<N>::kHighestDerivativeToOptimize) {
    vertices_ = vertices;
    bool ret = poly_opt_.setupFromVertices(vertices, segment_times, radii,
                                           derivative_to_optimize);
    ret = linear_.setupFromVertices(vertices, segment_times, derivative_to_optimize) && ret;
    return ret;
  }

  // nonlinear_impl:847-875.  The constraint is stored either way (it also
  // sets the free-derivative bounds of setFreeEndpointDerivativeHardConstraints,
  // :2890-2902); with use_soft_constraints = false it becomes an inequality
  // only if the algorithm takes one, else false is returned (NLopt throws in
  // add_inequality_constraint, :862-872) and the constraint is inactive.
  bool addMaximumMagnitudeConstraint(int derivative_order, double maximum_value) {
    MTG_CHECK(derivative_order >= 0, "derivative must be >= 0");
    MTG_CHECK(maximum_value >= 0.0, "maximum_value must be >= 0");
    if (soft_.size() >= 8 || derivative_order > derivative_order::SNAP ||
        N - derivative_order - 1 <= 0) {
      internal::warn("addMaximumMagnitudeConstraint: unsupported constraint ignored");
      return false;
    }
    soft_.push_back(std::make_pair(derivative_order, maximum_value));
    if (!params_.use_soft_constraints && !nlopt::takesInequalityConstraints(params_.algorithm))
      return false;
    return true;
  }

  int solveQCQP() { return poly_opt_.solveQCQP(); }
  bool solveLinear() { return linear_.solveLinear(); }

  // Time-only objective at `segment_times` (objectiveFunctionTime with the
  // linear inner solve).  grad_mode: 0 none, 1 getCostAndGradientTime
  // (nonlinear_impl:2495-2584), 2 central differences of J.  `gradient` is
  // resized to S when grad_mode != 0.
  double evaluateTimeCost(const std::vector<double>& segment_times, int grad_mode = 0,
                          std::vector<double>* gradient = nullptr) {
    const size_t S = linear_.getNumberSegments();
    MTG_CHECK(segment_times.size() == S, "segment_times has " << segment_times.size()
                                                              << " entries, need " << S);
    MTG_CHECK(grad_mode == 0 || gradient != nullptr, "gradient must not be null");
    warnCollision();
    if (params_.solve_time_with_qcqp) {
      MTG_CHECK(grad_mode != 1, "grad_mode 1 holds d fixed: not defined for the QCQP callback");
      return poly_opt_.evaluateTimeCostQCQP(segment_times, timeParams(grad_mode), gradient);
    }
    internal::DeviceBuffer<double> d_df, d_t, d_cost(1), d_g(S);
    d_df.upload(packFixed());
    d_t.upload(segment_times);
    const mtg_time_params p = timeParams(grad_mode, true);
    internal::checkStatus(mtg_time_cost(planOf(), 1, d_df.get(), d_t.get(), &p, d_cost.get(),
                                        grad_mode ? d_g.get() : nullptr, nullptr, nullptr),
                          "mtg_time_cost");
    internal::synchronize();
    double J = 0.0;
    d_cost.download(&J, 1);
    if (grad_mode) *gradient = d_g.download();
    return J;
  }

  // objectiveFunctionFreeConstraints (nonlinear_impl:1021-1113) on the
  // tube-pattern problem (poly_opt_): J_d = sum_dim d^T R d [+ soft], with
  // gradient dJ_d/dd_p per dimension when `gradient` is non-null.
  double evaluateFreeConstraintsCost(const std::vector<VectorXd>& free_constraints,
                                     std::vector<VectorXd>* gradient) {
    return freeCost(segmentTimesOfQcqp(), free_constraints, 0, gradient);
  }

  // objectiveFunctionTimeAndConstraints (nonlinear_impl:947-1019): segment
  // times and free derivatives given, J = computeCost() + time_penalty
  // (sum T)^2 [+ soft], no re-solve.
  double evaluateTimeAndFreeConstraintsCost(const std::vector<double>& segment_times,
                                            const std::vector<VectorXd>& free_constraints) {
    return freeCost(segment_times, free_constraints, 1, nullptr);
  }

  // Runs the optimisation: kOptimizeTime, kOptimizeFreeConstraints
  // (optimizeFreeConstraints, nonlinear_impl:399-493) or
  // kOptimizeFreeConstraintsAndTime (optimizeTimeAndFreeConstraints,
  // :610-706), each on the device.  Returns a positive NLopt-style success
  // code or a negative failure code.
  int optimize() {
    if (params_.objective == NonlinearOptimizationParameters::kOptimizeFreeConstraints)
      return optimizeFreeConstraints();
    if (params_.objective == NonlinearOptimizationParameters::kOptimizeFreeConstraintsAndTime)
      return optimizeTimeAndFreeConstraints();
    if (params_.objective == NonlinearOptimizationParameters::kOptimizeFreeConstraintsAndCollision)
      return optimizeCollision(false);
    if (params_.objective ==
        NonlinearOptimizationParameters::kOptimizeFreeConstraintsAndCollisionAndTime)
      return optimizeCollision(true);
    MTG_CHECK(params_.objective == NonlinearOptimizationParameters::kOptimizeTime,
              "unknown optimization objective (nonlinear_impl:305-307)");
    warnCollision();
    if (params_.solve_time_with_qcqp) return optimizeTimeQCQP();
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<double> times;
    linear_.getSegmentTimes(&times);
    linear_.solveLinear();  // initial solution (nonlinear_impl:341-349)
    linear_.getTrajectory(&trajectory_initial_);
    trajectory_initial_after_removing_pos_ = trajectory_initial_;  // :347-348, 416-417
    const size_t S = times.size();
    internal::DeviceBuffer<double> d_df, d_t, d_cost(1);
    internal::DeviceBuffer<int32_t> d_ev(1), d_st(1);
    d_df.upload(packFixed());
    d_t.upload(times);
    const mtg_time_params p = timeParams(0, true);
    const int budget = params_.max_iterations > 0 ? params_.max_iterations : 1000;
    internal::DeviceBuffer<int32_t> d_res(1);
    internal::checkStatus(mtg_time_optimize_ex(planOf(), 1, d_df.get(), d_t.get(), &p, budget,
                                               d_cost.get(), d_ev.get(), nullptr, d_res.get(),
                                               d_st.get(), nullptr),
                          "mtg_time_optimize_ex");
    internal::synchronize();
    d_t.download(times.data(), S);
    int32_t evals = 0, st = 0, res = 0;
    d_ev.download(&evals, 1);
    d_st.download(&st, 1);
    d_res.download(&res, 1);
    linear_.updateSegmentTimes(times);
    linear_.solveLinear();
    double tot = 0.0;
    for (double t : times) tot += t;
    optimization_info_.n_iterations = evals;
    optimization_info_.cost_trajectory = linear_.computeCost();
    optimization_info_.cost_time = tot * tot * params_.time_penalty;
    double J = 0.0;
    d_cost.download(&J, 1);
    optimization_info_.cost_soft_constraints =
        soft_.empty() ? 0.0
                      : J - optimization_info_.cost_trajectory - optimization_info_.cost_time;
    for (const auto& c : soft_)
      optimization_info_.maxima[c.first] =
          linear_.computeMaximumOfMagnitude(c.first, nullptr);
    optimization_info_.stopping_reason = st == MTG_TRAJ_OK ? res : -1;  // nlopt_result
    optimization_info_.optimization_time =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return optimization_info_.stopping_reason;
  }

  // The optimised trajectory: the linear problem's (kOptimizeTime) or the
  // tube-pattern problem's (after kOptimizeFreeConstraints, or kOptimizeTime
  // with solve_time_with_qcqp).
  void getTrajectory(Trajectory* trajectory) const {
    if (free_optimized_ || qcqp_time_optimized_)
      poly_opt_.getTrajectory(trajectory);
    else
      linear_.getTrajectory(trajectory);
  }
  void getQCQPTrajectory(Trajectory* trajectory) const { poly_opt_.getTrajectory(trajectory); }
  void getInitialSolutionTrajectory(Trajectory* trajectory) const {
    MTG_CHECK(trajectory != nullptr, "trajectory must not be null");
    MTG_CHECK(!trajectory_initial_.empty(), "optimize() has not run");
    *trajectory = trajectory_initial_;
  }
  void getFreeConstraints(std::vector<VectorXd>* free_constraints) const {
    linear_.getFreeConstraints(free_constraints);
  }
  // polynomial_optimization_nonlinear.h:293-295: the free derivatives as x, y,
  // z triples (D = 3), one per free derivative in the tube-pattern order of
  // poly_opt_ (the problem the free-derivative objectives optimise).
  void getFreeConstraints(std::vector<Vector3d>* free_constraints) const {
    MTG_CHECK(free_constraints != nullptr, "free_constraints must not be null");
    MTG_CHECK(dimension_ == 3, "Vector3d free constraints need dimension 3");
    std::vector<VectorXd> f;
    poly_opt_.getFreeConstraints(&f);
    free_constraints->clear();
    if (f.size() != 3) return;
    for (long i = 0; i < f[0].size(); ++i)
      free_constraints->push_back(Vector3d(f[0][i], f[1][i], f[2][i]));
  }
  // :307-314: the trajectory of the initial solution the optimiser starts
  // from (after the intermediate positions became free derivatives).
  void getInitialTrajectoryAfterRemovingPos(Trajectory* trajectory) const {
    MTG_CHECK(trajectory != nullptr, "trajectory must not be null");
    MTG_CHECK(!trajectory_initial_after_removing_pos_.empty(), "optimize() has not run");
    *trajectory = trajectory_initial_after_removing_pos_;
  }
  // :316-331: the trajectory of every objective evaluation of the collision
  // objectives (pushed at nonlinear_impl:1244, 1482; never cleared, as
  // there), appended to *trajectories.
  void getAllTrajectories(std::vector<Trajectory>* trajectories) const {
    MTG_CHECK(trajectories != nullptr, "trajectories must not be null");
    trajectories->reserve(trajectories->size() + all_trajectories_.size());
    for (const Trajectory& t : all_trajectories_) {
      MTG_CHECK(!t.empty(), "empty trajectory in the history");
      trajectories->push_back(t);
    }
  }
  // computeInitialSolutionWithPositionConstraints (nonlinear_impl:199-272):
  // solveQCQP, keep its trajectory as the initial one, then express it in
  // the pattern with the intermediate positions free.  The tube problem
  // (poly_opt_) already has every intermediate derivative free (the kDim
  // reordering, qcqp_impl:18-118), so re-deriving d_p from the coefficients
  // (M_pinv A p) returns the solve's own d_p, which is set back.
  bool computeInitialSolutionWithPositionConstraints() {
    poly_opt_.solveQCQP();
    poly_opt_.getTrajectory(&trajectory_initial_);
    std::vector<double> t;
    poly_opt_.getSegmentTimes(&t);
    trajectory_time_initial_ = 0.0;
    for (double ti : t) trajectory_time_initial_ += ti;  // computeTotalTrajectoryTime
    std::vector<VectorXd> free;
    poly_opt_.getFreeConstraints(&free);
    poly_opt_.setFreeConstraints(free);
    return true;
  }
  // Declared at polynomial_optimization_nonlinear.h:379; its definition is
  // commented out in the reference (nonlinear_impl:122-196) with the same
  // body as the WithPositionConstraints variant, which it runs here.
  bool computeInitialSolutionWithoutPositionConstraints() {
    return computeInitialSolutionWithPositionConstraints();
  }
  const PolynomialOptimization<N>& getPolynomialOptimizationRef() const { return linear_; }
  PolynomialOptimization<N>& getPolynomialOptimizationRef() { return linear_; }
  const PolynomialOptimizationConstrained<N>& getConstrainedOptimizationRef() const {
    return poly_opt_;
  }
  OptimizationInfo getOptimizationInfo() const { return optimization_info_; }

  // printMatlabSampledTrajectory (nonlinear_impl:2907-3003): the optimised
  // trajectory sampled every dt = 0.01 s from the start of each segment
  // (t = 0, dt, ... < T_i), one row per sample
  // [t_total, p(D), v(D), a(D), j(D), s(D), tm] where tm is the cumulative
  // time at the end of segment i written into row i only, zero rows padding
  // to sum_i (ceil(T_i / dt) + 1) rows, printed as Eigen's default matrix
  // stream format (6 significant digits, every column padded to the widest
  // entry, space separated).  The samples come from the device sampler
  // (mtg_sample_trajectories, one one-segment trajectory per segment); the
  // reference accumulates t by repeated addition where the sampler uses
  // k dt, which the 6-digit text does not resolve.
  void printMatlabSampledTrajectory(const std::string& file) const {
    Trajectory traj;
    getTrajectory(&traj);
    MTG_CHECK(!traj.empty(), "no trajectory to print");
    MTG_CHECK(N >= 5, "printMatlabSampledTrajectory needs derivatives up to snap (N >= 5)");
    const double dt = 0.01;
    const int S = traj.K(), D = traj.D(), K = derivative_order::SNAP;
    const std::vector<double> times = traj.getSegmentTimes();
    int total = 0, n_max = 1;
    for (double t : times) {
      const int n = static_cast<int>(std::ceil(t / dt)) + 1;
      total += n;
      n_max = std::max(n_max, n);
    }
    n_max = (n_max + 63) / 64 * 64;
    std::vector<double> coeffs(static_cast<size_t>(S) * D * N);
    for (int s = 0; s < S; ++s)
      for (int d = 0; d < D; ++d) {
        const VectorXd c = traj.segments()[s][d].getCoefficients(0);
        for (int k = 0; k < N; ++k) coeffs[(static_cast<size_t>(s) * D + d) * N + k] = c[k];
      }
    const int nch = (K + 1) * D;
    internal::DeviceBuffer<double> d_c, d_t, d_smp(static_cast<size_t>(S) * nch * n_max);
    internal::DeviceBuffer<int32_t> d_cnt(S);
    d_c.upload(coeffs);
    d_t.upload(times);
    internal::checkStatus(mtg_sample_trajectories(N, D, 1, S, d_c.get(), d_t.get(), 0.0, -1.0,
                                                  dt, n_max, K, d_smp.get(), nullptr,
                                                  d_cnt.get(), nullptr),
                          "mtg_sample_trajectories");
    internal::synchronize();
    const std::vector<double> smp = d_smp.download();
    const std::vector<int32_t> cnt = d_cnt.download();
    const int cols = 5 * D + 2;
    std::vector<double> out(static_cast<size_t>(total) * cols, 0.0);
    int row = 0;
    double seg_start = 0.0;
    for (int s = 0; s < S; ++s) {
      for (int k = 0; k < cnt[s] && row < total; ++k, ++row) {
        out[static_cast<size_t>(row) * cols] = k * dt + seg_start;
        for (int ch = 0; ch < nch; ++ch)
          out[static_cast<size_t>(row) * cols + 1 + ch] =
              smp[(static_cast<size_t>(s) * nch + ch) * n_max + k];
      }
      seg_start += times[s];
      out[static_cast<size_t>(s) * cols + cols - 1] = seg_start;
    }
    // Eigen's default IOFormat: one width for every entry.
    std::vector<std::string> txt(out.size());
    size_t width = 0;
    for (size_t i = 0; i < out.size(); ++i) {
      std::ostringstream os;
      os << out[i];
      txt[i] = os.str();
      width = std::max(width, txt[i].size());
    }
    std::ofstream fs(file);
    for (int r = 0; r < total; ++r) {
      if (r) fs << "\n";
      for (int c = 0; c < cols; ++c) {
        if (c) fs << " ";
        const std::string& t = txt[static_cast<size_t>(r) * cols + c];
        fs << std::string(width - t.size(), ' ') << t;
      }
    }
  }

  // setOctree (polynomial_optimization_nonlinear.h:357-363) is kept for
  // source compatibility: supereight is absent, so the octree is not read and
  // the map must be given to setOccupancyGrid.
  void setOctree(const void* octree) {
    if (octree)
      internal::warn("setOctree: supereight is not available; pass the map to setOccupancyGrid");
  }

  // Occupancy map for the collision cost (build extension standing in for
  // setOctree, polynomial_optimization_nonlinear.h:357-363; supereight is
  // absent): a dense grid of log-odds, voxel (x, y, z) at (z*ny + y)*nx + x,
  // occupied iff >= 0, uploaded once.
  void setOccupancyGrid(const std::vector<float>& occupancy, int nx, int ny, int nz) {
    MTG_CHECK(nx >= 0 && ny >= 0 && nz >= 0 &&
                  static_cast<size_t>(nx) * ny * nz == occupancy.size(),
              "grid size mismatch");
    occ_dims_[0] = nx;
    occ_dims_[1] = ny;
    occ_dims_[2] = nz;
    occupancy_.upload(occupancy);
    grid_set_ = true;
    field_side_ = -1;  // the near field is rebuilt for the new map
  }

  // The collision objective at x (objectiveFunctionFreeConstraintsAndCollision,
  // nonlinear_impl:1115-1272, x = d_p dimension-major; with the objective
  // kOptimizeFreeConstraintsAndCollisionAndTime :1274-1535, x = [T; d_p]) on
  // the tube-pattern problem, with the reference's collision raise state of
  // this object (total_cost_iter0_ set by the first evaluation, the last
  // evaluation's total).  `gradient` (nullable) is resized to x.size().
  double evaluateCollisionObjective(const std::vector<double>& x,
                                    std::vector<double>* gradient) {
    MTG_CHECK(grid_set_, "setOccupancyGrid first");
    const int mode = collisionMode();
    const size_t np = poly_opt_.getNumberFreeConstraints();
    const size_t S = poly_opt_.getNumberSegments();
    const size_t nv = (mode ? S : 0) + dimension_ * np;
    MTG_CHECK(x.size() == nv, "x has " << x.size() << " entries, need " << nv);
    const mtg_coll_params cp = collParams();
    const int64_t nb = mtg_coll_workspace_bytes(poly_opt_.getPlan(), 1, mode, &cp, 0);
    MTG_CHECK(nb > 0, "mtg_coll_workspace_bytes: " << mtg_status_string(static_cast<int>(nb)));
    internal::DeviceBuffer<double> d_df, d_x, d_t, d_ref, d_cost(1), d_g(nv), d_terms(4);
    internal::DeviceBuffer<int32_t> d_coll(1), d_st(1);
    internal::DeviceBuffer<unsigned char> ws(static_cast<size_t>(nb));
    d_df.upload(packFixedQcqp());
    d_x.upload(x);
    d_t.upload(segmentTimesOfQcqp());
    const double ref = params_.is_coll_raise_first_iter ? total_cost_iter0_ : last_total_;
    d_ref.upload(&ref, 1);
    internal::checkStatus(
        mtg_coll_cost(poly_opt_.getPlan(), 1, mode, d_df.get(), d_x.get(), d_t.get(),
                      occupancy_.get(), occ_dims_[0], occ_dims_[1], occ_dims_[2],
                      nearField(cp.coll), &cp,
                      d_ref.get(), d_cost.get(), gradient ? d_g.get() : nullptr, d_terms.get(),
                      d_coll.get(), d_st.get(), ws.get(), static_cast<size_t>(nb), nullptr),
        "mtg_coll_cost");
    internal::synchronize();
    double J = 0.0;
    d_cost.download(&J, 1);
    if (gradient) *gradient = d_g.download();
    if (is_iter0_) {  // nonlinear_impl:1253-1257
      total_cost_iter0_ = J;
      is_iter0_ = false;
    }
    last_total_ = J;
    return J;
  }

  // getCostAndGradientCollision (nonlinear_impl:1609-1780) of the tube-pattern
  // problem's current solution (poly_opt_, as the reference) on the device
  // (mtg_collision_cost); gradient (nullable) w.r.t. its free derivatives.
  double getCostAndGradientCollision(std::vector<VectorXd>* gradients, bool* is_collision) {
    MTG_CHECK(is_collision != nullptr, "is_collision must not be null");
    MTG_CHECK(grid_set_, "setOccupancyGrid first");
    Trajectory traj;
    poly_opt_.getTrajectory(&traj);
    const int S = traj.K(), D = traj.D();
    MTG_CHECK(D == 3, "the collision cost is 3-D (nonlinear_impl:1796-1797)");
    std::vector<double> coeffs(static_cast<size_t>(S) * D * N);
    for (int s = 0; s < S; ++s)
      for (int d = 0; d < D; ++d) {
        const VectorXd c = traj.segments()[s][d].getCoefficients(0);
        for (int k = 0; k < N; ++k) coeffs[(static_cast<size_t>(s) * D + d) * N + k] = c[k];
      }
    const mtg_collision_params cp = collisionParams();
    const size_t np = poly_opt_.getNumberFreeConstraints();
    internal::DeviceBuffer<double> d_c, d_t, d_cost(1), d_g(np ? D * np : 1);
    internal::DeviceBuffer<int32_t> d_coll(1);
    d_c.upload(coeffs);
    d_t.upload(traj.getSegmentTimes());
    internal::checkStatus(
        mtg_collision_cost(poly_opt_.getPlan(), 1, d_c.get(), d_t.get(), occupancy_.get(),
                           occ_dims_[0], occ_dims_[1], occ_dims_[2], &cp, d_cost.get(),
                           d_coll.get(), nullptr, (gradients && np) ? d_g.get() : nullptr,
                           nullptr),
        "mtg_collision_cost");
    internal::synchronize();
    double J = 0.0;
    int32_t coll = 0;
    d_cost.download(&J, 1);
    d_coll.download(&coll, 1);
    *is_collision = coll != 0;
    if (gradients) {
      gradients->assign(D, VectorXd(static_cast<long>(np)));
      if (np) {
        const std::vector<double> g = d_g.download();
        for (int d = 0; d < D; ++d)
          for (size_t i = 0; i < np; ++i) (*gradients)[d][i] = g[d * np + i];
      }
    }
    return J;
  }

  // nonlinear_impl:2768-2774.
  static double computeTotalTrajectoryTime(const std::vector<double>& segment_times) {
    double t = 0.0;
    for (double s : segment_times) t += s;
    return t;
  }

 private:
  mtg_collision_params collisionParams() const {
    mtg_collision_params cp;
    cp.map_resolution = params_.map_resolution;
    for (int k = 0; k < 3; ++k) {
      cp.min_bound[k] = params_.min_bound[k];
      cp.max_bound[k] = params_.max_bound[k];
    }
    cp.epsilon = params_.epsilon;
    cp.robot_radius = params_.robot_radius;
    cp.coll_pot_multiplier = params_.coll_pot_multiplier;
    cp.coll_check_time_increment = params_.coll_check_time_increment;
    cp.box_side = 20;  // findOccupiedVoxels side (nonlinear_impl:1798)
    return cp;
  }

  int collisionMode() const {
    return params_.objective ==
                   NonlinearOptimizationParameters::kOptimizeFreeConstraintsAndCollisionAndTime
               ? 1
               : 0;
  }

  mtg_coll_params collParams() const {
    mtg_coll_params p;
    p.coll = collisionParams();
    p.w_d = params_.weights.w_d;
    p.w_c = params_.weights.w_c;
    p.w_t = params_.weights.w_t;
    p.w_sc = params_.weights.w_sc;
    p.is_collision_safe = params_.is_collision_safe ? 1 : 0;
    p.is_coll_raise_first_iter = params_.is_coll_raise_first_iter ? 1 : 0;
    p.add_coll_raise = params_.add_coll_raise;
    p.simple_numgrad_time = params_.is_simple_numgrad_time ? 1 : 0;
    p.simple_numgrad_constraints = params_.is_simple_numgrad_constraints ? 1 : 0;
    p.increment_time = params_.increment_time;
    // Soft costs only with use_soft_constraints (:1174-1177); otherwise the
    // constraints would be NLopt inequalities, which LD_LBFGS does not take.
    p.n_soft = params_.use_soft_constraints ? static_cast<int>(soft_.size()) : 0;
    for (int c = 0; c < 8; ++c) {
      p.soft_derivative[c] = c < p.n_soft ? soft_[c].first : 0;
      p.soft_limit[c] = c < p.n_soft ? soft_[c].second : 1.0;
    }
    p.soft_weight = params_.soft_constraint_weight;
    p.soft_maximum_cost = 1.0e12;
    p.f_rel = params_.f_rel;
    p.f_abs = params_.f_abs;
    p.x_rel = params_.x_rel;
    p.x_abs = params_.x_abs;
    p.lbfgs_memory = params_.lbfgs_memory;
    return p;
  }

  // setFreeEndpointDerivativeHardConstraints (nonlinear_impl:2858-2905) over
  // the free derivatives x (dimension-major), including the reference's
  // stride of derivative_to_optimize per vertex when
  // solve_with_position_constraint is set (:2879-2880).  Indices are
  // unsigned int and every write goes through .at(), as in the reference: a
  // position-magnitude constraint with solve_with_position_constraint wraps
  // (derivative - 1) and a derivative past the vertex stride runs off the
  // end; both throw std::out_of_range instead of writing out of bounds.
  void freeEndpointBounds(size_t n, std::vector<double>* lo, std::vector<double>* hi) const {
    const size_t np = poly_opt_.getNumberFreeConstraints();
    const size_t S = poly_opt_.getNumberSegments();
    lo->assign(n, -HUGE_VAL);
    hi->assign(n, HUGE_VAL);
    const int r = poly_opt_.getDerivativeToOptimize();
    for (size_t k = 0; k < dimension_; ++k)
      for (size_t v = 0; v + 1 < S; ++v) {
        unsigned int start;
        if (params_.solve_with_position_constraint) {
          start = static_cast<unsigned int>(k * np + v * r);
        } else {
          start = static_cast<unsigned int>(k * np + v * (r + 1));
          lo->at(start) = params_.min_bound[static_cast<long>(k)];
          hi->at(start) = params_.max_bound[static_cast<long>(k)];
        }
        for (const auto& c : soft_) {
          const unsigned int deriv = params_.solve_with_position_constraint
                                         ? static_cast<unsigned int>(c.first - 1)
                                         : static_cast<unsigned int>(c.first);
          lo->at(static_cast<size_t>(start) + deriv) = -std::abs(c.second);
          hi->at(static_cast<size_t>(start) + deriv) = std::abs(c.second);
        }
      }
  }

  // optimizeFreeConstraintsAndCollision (nonlinear_impl:495-607) and
  // optimizeFreeConstraintsAndCollisionAndTime (:708-845): initial solution
  // from the tube QCQP (with solve_with_position_constraint directly; else
  // computeInitialSolutionWithPositionConstraints, :199-272, which rebuilds
  // the same all-intermediates-free pattern and recovers the same d_p), the
  // reference's bounds and initial steps, then the device L-BFGS of
  // mtg_coll_optimize in place of NLopt (max_iterations evaluations, f_rel /
  // f_abs / x_rel / x_abs).  The problem keeps the best point found.
  int optimizeCollision(bool with_time) {
    MTG_CHECK(grid_set_, "setOccupancyGrid first: the collision objectives need a map");
    MTG_CHECK(dimension_ == 3, "the collision objectives are 3-D (nonlinear_impl:1796-1797)");
    const auto t0 = std::chrono::steady_clock::now();
    poly_opt_.solveQCQP();
    poly_opt_.getTrajectory(&trajectory_initial_);
    trajectory_initial_after_removing_pos_ = trajectory_initial_;  // :347-348, 416-417
    std::vector<VectorXd> free;
    poly_opt_.getFreeConstraints(&free);
    MTG_CHECK(!free.empty() && free.front().size() > 0, "no free constraints (:516-517)");
    const std::vector<double> d0 = packFree(free);
    std::vector<double> times = segmentTimesOfQcqp();
    const size_t S = times.size(), np = poly_opt_.getNumberFreeConstraints();
    const size_t off = with_time ? S : 0, nv = off + d0.size();
    std::vector<double> x(nv), lo(nv), hi(nv), step(nv);
    for (size_t i = 0; i < S && with_time; ++i) {
      x[i] = times[i];
      lo[i] = 0.1;  // :785-789
      hi[i] = HUGE_VAL;
    }
    std::vector<double> lod, hid;
    freeEndpointBounds(d0.size(), &lod, &hid);
    for (size_t i = 0; i < d0.size(); ++i) {
      x[off + i] = d0[i];
      lo[off + i] = lod[i];
      hi[off + i] = hid[i];
    }
    for (size_t i = 0; i < nv; ++i) {  // :559-567 (position steps) and :800-805
      const double a = std::abs(x[i]);
      step[i] = (!with_time && a > 5) ? params_.initial_stepsize_position
                                      : params_.initial_stepsize_rel * a;
    }
    const int mode = with_time ? 1 : 0;
    const mtg_coll_params cp = collParams();
    const int64_t nb = mtg_coll_workspace_bytes(poly_opt_.getPlan(), 1, mode, &cp, 1);
    MTG_CHECK(nb > 0, "mtg_coll_workspace_bytes: " << mtg_status_string(static_cast<int>(nb)));
    internal::DeviceBuffer<double> d_df, d_x, d_t, d_lo, d_hi, d_step, d_cost(1), d_terms(4);
    internal::DeviceBuffer<int32_t> d_ev(1), d_res(1), d_st(1);
    internal::DeviceBuffer<unsigned char> ws(static_cast<size_t>(nb));
    const std::vector<double> fixed = packFixedQcqp();
    d_df.upload(fixed);
    d_x.upload(x);
    d_t.upload(times);
    d_lo.upload(lo);
    d_hi.upload(hi);
    d_step.upload(step);
    const int budget = params_.max_iterations > 0 ? params_.max_iterations : 1000;
    internal::DeviceBuffer<double> d_hist(static_cast<size_t>(budget) * nv);
    internal::checkStatus(
        mtg_coll_optimize_trace(poly_opt_.getPlan(), 1, mode, d_df.get(), d_x.get(), d_t.get(),
                                d_lo.get(), d_hi.get(), d_step.get(), occupancy_.get(),
                                occ_dims_[0], occ_dims_[1], occ_dims_[2], nearField(cp.coll), &cp,
                                budget, d_cost.get(), d_ev.get(), d_res.get(), d_st.get(),
                                d_terms.get(), d_hist.get(), ws.get(), static_cast<size_t>(nb),
                                nullptr),
        "mtg_coll_optimize_trace");
    internal::synchronize();
    x = d_x.download();
    int32_t evals = 0, res = 0, st = 0;
    d_ev.download(&evals, 1);
    d_res.download(&res, 1);
    d_st.download(&st, 1);
    appendHistory(d_hist, evals, nv, with_time, fixed, times);
    double terms[4] = {0, 0, 0, 0};
    d_terms.download(terms, 4);
    if (with_time) {
      for (size_t i = 0; i < S; ++i) times[i] = x[i];
      poly_opt_.updateSegmentTimes(times);
    }
    for (size_t d = 0; d < dimension_; ++d)
      for (size_t i = 0; i < np; ++i) free[d][i] = x[off + d * np + i];
    poly_opt_.setFreeConstraints(free);
    optimization_info_.n_iterations = evals;
    optimization_info_.cost_trajectory = terms[0];
    optimization_info_.cost_collision = terms[1];
    optimization_info_.cost_time = terms[2];
    optimization_info_.cost_soft_constraints = terms[3];
    optimization_info_.stopping_reason = st == MTG_TRAJ_OK ? res : nlopt::FAILURE;
    optimization_info_.optimization_time =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    free_optimized_ = true;
    return optimization_info_.stopping_reason;
  }

  // optimizeTime in the fork's form: initial QCQP solve (nonlinear_impl:
  // 341-349), device optimiser over the QCQP objective, final QCQP solve at
  // the optimised times.
  int optimizeTimeQCQP() {
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<double> times = segmentTimesOfQcqp();
    poly_opt_.solveQCQP();
    poly_opt_.getTrajectory(&trajectory_initial_);
    trajectory_initial_after_removing_pos_ = trajectory_initial_;  // :347-348, 416-417
    const int budget = params_.max_iterations > 0 ? params_.max_iterations : 1000;
    double J = 0.0;
    int32_t evals = 0;
    // LN_SBPLX (the default algorithm) runs NLopt's Subplex restated on the
    // device over the QCQP objective; any other algorithm the descent
    const mtg_time_params tp = timeParams(2);
    int32_t res = 0;
    const int st = poly_opt_.optimizeTimeQCQP(tp, budget, &times, &J, &evals, 1e-10, 100, &res);
    poly_opt_.updateSegmentTimes(times);
    poly_opt_.solveQCQP();
    qcqp_time_optimized_ = true;
    double tot = 0.0;
    for (double t : times) tot += t;
    optimization_info_.n_iterations = evals;
    optimization_info_.cost_trajectory = poly_opt_.computeCost();
    optimization_info_.cost_time = tot * tot * params_.time_penalty;
    optimization_info_.cost_soft_constraints =
        soft_.empty() ? 0.0
                      : J - optimization_info_.cost_trajectory - optimization_info_.cost_time;
    for (const auto& c : soft_)
      optimization_info_.maxima[c.first] = poly_opt_.computeMaximumOfMagnitude(c.first, nullptr);
    optimization_info_.stopping_reason = st == MTG_TRAJ_OK ? res : -1;  // nlopt_result
    optimization_info_.optimization_time =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return optimization_info_.stopping_reason;
  }

  // all_trajectories_ (nonlinear_impl:1241-1244, 1479-1482): the trajectory
  // of every counted evaluation, in order.  The evaluated points come from
  // the device optimiser's history; their coefficients from one batched
  // mtg_coeffs_from_constraints over the tube-pattern plan.
  void appendHistory(const internal::DeviceBuffer<double>& d_hist, int evals, size_t nv,
                     bool with_time, const std::vector<double>& fixed,
                     const std::vector<double>& times0) {
    if (evals <= 0) return;
    const size_t S = times0.size(), off = with_time ? S : 0, nd = nv - off;
    const size_t ne = static_cast<size_t>(evals), D = dimension_;
    std::vector<double> hx(ne * nv);
    d_hist.download(hx.data(), hx.size());
    std::vector<double> df, dp, tt;
    for (size_t e = 0; e < ne; ++e) {
      df.insert(df.end(), fixed.begin(), fixed.end());
      for (size_t i = 0; i < nd; ++i) dp.push_back(hx[e * nv + off + i]);
      for (size_t i = 0; i < S; ++i) tt.push_back(with_time ? hx[e * nv + i] : times0[i]);
    }
    internal::DeviceBuffer<double> d_df, d_dp, d_t, d_c(ne * S * D * N);
    d_df.upload(df);
    d_dp.upload(dp);
    d_t.upload(tt);
    internal::checkStatus(mtg_coeffs_from_constraints(poly_opt_.getPlan(),
                                                      static_cast<int64_t>(ne), d_df.get(),
                                                      d_dp.get(), d_t.get(), d_c.get(), nullptr,
                                                      nullptr, nullptr),
                          "mtg_coeffs_from_constraints");
    internal::synchronize();
    const std::vector<double> c = d_c.download();
    for (size_t e = 0; e < ne; ++e) {
      Segment::Vector segs(S, Segment(N, static_cast<int>(D)));
      for (size_t s = 0; s < S; ++s) {
        segs[s].setTime(tt[e * S + s]);
        for (size_t d = 0; d < D; ++d) {
          VectorXd cd(N);
          for (int k = 0; k < N; ++k) cd[k] = c[((e * S + s) * D + d) * N + k];
          segs[s][static_cast<int>(d)] = Polynomial(N, cd);
        }
      }
      Trajectory t;
      t.setSegments(segs);
      all_trajectories_.push_back(t);
    }
  }

  std::vector<double> segmentTimesOfQcqp() const {
    std::vector<double> t;
    poly_opt_.getSegmentTimes(&t);
    return t;
  }

  std::vector<double> packFree(const std::vector<VectorXd>& free_constraints) const {
    const size_t np = poly_opt_.getNumberFreeConstraints();
    MTG_CHECK(free_constraints.size() == dimension_,
              "free constraints: need " << dimension_ << " dimensions");
    std::vector<double> out;
    for (const VectorXd& v : free_constraints) {
      MTG_CHECK(static_cast<size_t>(v.size()) == np, "free constraints: need " << np
                                                         << " entries per dimension");
      for (long i = 0; i < v.size(); ++i) out.push_back(v[i]);
    }
    return out;
  }

  std::vector<double> packFixedQcqp() const {
    std::vector<VectorXd> df;
    poly_opt_.getFixedConstraints(&df);
    std::vector<double> out;
    for (const VectorXd& v : df)
      for (long i = 0; i < v.size(); ++i) out.push_back(v[i]);
    return out;
  }

  double freeCost(const std::vector<double>& segment_times,
                  const std::vector<VectorXd>& free_constraints, int mode,
                  std::vector<VectorXd>* gradient) {
    const size_t np = poly_opt_.getNumberFreeConstraints();
    MTG_CHECK(segment_times.size() == poly_opt_.getNumberSegments(), "segment_times size");
    warnCollision();
    const std::vector<double> dp = packFree(free_constraints);
    internal::DeviceBuffer<double> d_df, d_dp, d_t, d_cost(1), d_g(dp.size() ? dp.size() : 1);
    d_df.upload(packFixedQcqp());
    d_dp.upload(dp);
    d_t.upload(segment_times);
    const mtg_time_params p = timeParams(0);
    internal::checkStatus(
        mtg_free_cost(poly_opt_.getPlan(), 1, d_df.get(), d_dp.get(), d_t.get(), &p, mode,
                      d_cost.get(), (gradient && mode == 0) ? d_g.get() : nullptr, nullptr,
                      nullptr),
        "mtg_free_cost");
    internal::synchronize();
    double J = 0.0;
    d_cost.download(&J, 1);
    if (gradient && mode == 0) {
      const std::vector<double> g = d_g.download();
      gradient->assign(dimension_, VectorXd(static_cast<long>(np)));
      for (size_t d = 0; d < dimension_; ++d)
        for (size_t i = 0; i < np; ++i) (*gradient)[d][i] = g[d * np + i];
    }
    return J;
  }

  // optimizeFreeConstraints (nonlinear_impl:399-493): initial solution from
  // the tube QCQP (:405-416; the fork's
  // computeInitialSolutionWithPositionConstraints rebuilds the same tube
  // pattern and recovers the same d_p), hard bounds of
  // setFreeEndpointDerivativeHardConstraints (:2858-2905), then the device
  // optimiser of mtg_free_optimize in place of NLopt with max_iterations
  // objective evaluations.
  int optimizeFreeConstraints() {
    warnCollision();
    const auto t0 = std::chrono::steady_clock::now();
    poly_opt_.solveQCQP();
    poly_opt_.getTrajectory(&trajectory_initial_);
    trajectory_initial_after_removing_pos_ = trajectory_initial_;  // :347-348, 416-417
    std::vector<VectorXd> free;
    poly_opt_.getFreeConstraints(&free);
    const std::vector<double> x0 = packFree(free);
    const size_t np = poly_opt_.getNumberFreeConstraints();
    std::vector<double> lo, hi;
    freeEndpointBounds(x0.size(), &lo, &hi);
    internal::DeviceBuffer<double> d_df, d_dp, d_t, d_lo, d_hi, d_cost(1);
    internal::DeviceBuffer<int32_t> d_ev(1), d_st(1);
    d_df.upload(packFixedQcqp());
    d_dp.upload(x0);
    d_t.upload(segmentTimesOfQcqp());
    d_lo.upload(lo);
    d_hi.upload(hi);
    const mtg_time_params p = timeParams(0);
    const int budget = params_.max_iterations > 0 ? params_.max_iterations : 1000;
    internal::checkStatus(mtg_free_optimize(poly_opt_.getPlan(), 1, d_df.get(), d_dp.get(),
                                            d_t.get(), d_lo.get(), d_hi.get(), &p, budget,
                                            d_cost.get(), d_ev.get(), d_st.get(), nullptr),
                          "mtg_free_optimize");
    internal::synchronize();
    const std::vector<double> x = d_dp.download();
    for (size_t d = 0; d < dimension_; ++d)
      for (size_t i = 0; i < np; ++i) free[d][i] = x[d * np + i];
    poly_opt_.setFreeConstraints(free);
    int32_t evals = 0, st = 0;
    d_ev.download(&evals, 1);
    d_st.download(&st, 1);
    double J = 0.0;
    d_cost.download(&J, 1);
    optimization_info_.n_iterations = evals;
    optimization_info_.cost_trajectory = 2.0 * poly_opt_.computeCost();  // J_d
    optimization_info_.cost_soft_constraints =
        soft_.empty() ? 0.0 : J - optimization_info_.cost_trajectory;
    optimization_info_.stopping_reason = st == MTG_TRAJ_OK ? 5 /* MAXEVAL_REACHED */ : -1;
    optimization_info_.optimization_time =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    free_optimized_ = true;
    return optimization_info_.stopping_reason;
  }

  // optimizeTimeAndFreeConstraints (nonlinear_impl:610-706): initial
  // solution from the tube QCQP (:617-622), x = [T; d_p] with the bounds of
  // :660-677, then the device optimiser of mtg_time_free_optimize in place of
  // NLopt (max_iterations objective evaluations of
  // objectiveFunctionTimeAndConstraints, :947-1019).
  int optimizeTimeAndFreeConstraints() {
    warnCollision();
    const auto t0 = std::chrono::steady_clock::now();
    poly_opt_.solveQCQP();
    poly_opt_.getTrajectory(&trajectory_initial_);
    trajectory_initial_after_removing_pos_ = trajectory_initial_;  // :347-348, 416-417
    std::vector<VectorXd> free;
    poly_opt_.getFreeConstraints(&free);
    MTG_CHECK(!free.empty() && free.front().size() > 0, "no free constraints (:619-621)");
    const std::vector<double> x0 = packFree(free);
    std::vector<double> times = segmentTimesOfQcqp();
    const size_t np = poly_opt_.getNumberFreeConstraints();
    internal::DeviceBuffer<double> d_df, d_dp, d_t, d_cost(1);
    internal::DeviceBuffer<int32_t> d_ev(1), d_res(1), d_st(1);
    d_df.upload(packFixedQcqp());
    d_dp.upload(x0);
    d_t.upload(times);
    // LN_SBPLX (the default) runs NLopt's Subplex restated on the device over
    // all S + D n_p variables (:610-706); any other algorithm the
    // block-alternating descent
    const mtg_time_params p = timeParams(0);
    const int budget = params_.max_iterations > 0 ? params_.max_iterations : 1000;
    internal::checkStatus(mtg_time_free_optimize_ex(poly_opt_.getPlan(), 1, d_df.get(),
                                                    d_dp.get(), d_t.get(), &p, budget,
                                                    d_cost.get(), d_ev.get(), d_res.get(),
                                                    d_st.get(), nullptr),
                          "mtg_time_free_optimize_ex");
    internal::synchronize();
    const std::vector<double> x = d_dp.download();
    d_t.download(times.data(), times.size());
    for (size_t d = 0; d < dimension_; ++d)
      for (size_t i = 0; i < np; ++i) free[d][i] = x[d * np + i];
    poly_opt_.updateSegmentTimes(times);
    poly_opt_.setFreeConstraints(free);
    int32_t evals = 0, st = 0, res = 0;
    d_ev.download(&evals, 1);
    d_st.download(&st, 1);
    d_res.download(&res, 1);
    double J = 0.0, tot = 0.0;
    d_cost.download(&J, 1);
    for (double t : times) tot += t;
    optimization_info_.n_iterations = evals;
    optimization_info_.cost_trajectory = poly_opt_.computeCost();
    optimization_info_.cost_time = tot * tot * params_.time_penalty;
    optimization_info_.cost_soft_constraints =
        soft_.empty() ? 0.0
                      : J - optimization_info_.cost_trajectory - optimization_info_.cost_time;
    // nlopt_result of the device Subplex; the descent reports MAXEVAL_REACHED
    const int code = p.optimizer == 1 ? res : 5;
    optimization_info_.stopping_reason = st == MTG_TRAJ_OK ? code : -1;
    optimization_info_.optimization_time =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    free_optimized_ = true;
    return optimization_info_.stopping_reason;
  }

  // hard_ok: the entry point takes hard constraints (mtg_time_cost /
  // mtg_time_optimize); elsewhere hard constraints are dropped with a warning.
  mtg_time_params timeParams(int grad_mode, bool hard_ok = false) const {
    mtg_time_params p{};
    // LN_SBPLX (the default) is restated on the device; it takes no
    // inequality constraints, so use_soft_constraints = false leaves the
    // magnitude constraints without effect, as NLopt does
    // (nonlinear_impl:861-872 registers them only for algorithms taking them)
    const bool sbplx = params_.algorithm == nlopt::LN_SBPLX;
    p.optimizer = sbplx ? 1 : 0;
    p.f_rel = params_.f_rel;
    p.f_abs = params_.f_abs;
    p.initial_stepsize_rel = params_.initial_stepsize_rel;
    p.time_penalty = params_.time_penalty;
    p.increment = params_.increment_time;
    p.w_d = params_.weights.w_d;
    p.w_t = params_.weights.w_t;
    p.grad_mode = grad_mode;
    const bool hard = !params_.use_soft_constraints;
    if (hard && !hard_ok && !soft_.empty())
      internal::warn("hard magnitude constraints are only applied by kOptimizeTime with the "
                     "linear inner solve; ignored here");
    const bool take_hard = hard && hard_ok && !sbplx;
    p.n_soft = (!hard || take_hard) ? static_cast<int>(soft_.size()) : 0;
    p.hard_constraints = take_hard ? 1 : 0;
    p.hard_tolerance = params_.inequality_constraint_tolerance;
    for (int c = 0; c < 8; ++c) {
      p.soft_derivative[c] = c < p.n_soft ? soft_[c].first : 0;
      p.soft_limit[c] = c < p.n_soft ? soft_[c].second : 1.0;
    }
    p.soft_weight = params_.soft_constraint_weight;
    p.soft_maximum_cost = 1.0e12;  // evaluateMaximumMagnitudeAsSoftConstraint default
    return p;
  }
  void warnCollision() const {
    if (params_.weights.w_c > 0.0)
      internal::warn("this objective has no collision term here (w_c > 0 ignored; "
                     "kOptimizeFreeConstraintsAndCollision(AndTime) use it)");
  }
  std::vector<double> packFixed() const {
    std::vector<VectorXd> df;
    linear_.getFixedConstraints(&df);
    std::vector<double> out;
    for (const VectorXd& v : df)
      for (long i = 0; i < v.size(); ++i) out.push_back(v[i]);
    return out;
  }
  const mtg_plan* planOf() const { return linear_.getPlan(); }

  size_t dimension_;
  NonlinearOptimizationParameters params_;
  PolynomialOptimizationConstrained<N> poly_opt_;
  PolynomialOptimization<N> linear_;
  Vertex::Vector vertices_;
  double trajectory_time_initial_ = 0.0;
  Trajectory trajectory_initial_;
  Trajectory trajectory_initial_after_removing_pos_;
  std::vector<Trajectory> all_trajectories_;
  OptimizationInfo optimization_info_;
  std::vector<std::pair<int, double>> soft_;  // (derivative, maximum_value)
  internal::DeviceBuffer<float> occupancy_;
  int occ_dims_[3] = {0, 0, 0};
  bool grid_set_ = false;
  // Near field of the map (mtg_coll_field) for the current box side, built
  // on first use and kept until the map or the box side changes.
  internal::DeviceBuffer<uint16_t> field_;
  int field_side_ = -1;

  const uint16_t* nearField(const mtg_collision_params& cp) {
    if (field_side_ == cp.box_side) return field_.get();
    const int64_t n = mtg_coll_field_bytes(occ_dims_[0], occ_dims_[1], occ_dims_[2]);
    if (n <= 0) return nullptr;
    field_.resize(static_cast<size_t>(n) / sizeof(uint16_t));
    if (mtg_coll_field(occupancy_.get(), occ_dims_[0], occ_dims_[1], occ_dims_[2], &cp,
                       field_.get(), nullptr) != MTG_OK)
      return nullptr;  // box side beyond the field's range: the walk scans
    field_side_ = cp.box_side;
    return field_.get();
  }
  // Collision raise state (polynomial_optimization_nonlinear.h:672-673, and
  // the optimization_info_ totals of the last evaluation, :1216-1219).
  double total_cost_iter0_ = 0.0;
  double last_total_ = 0.0;
  bool is_iter0_ = true;
  bool free_optimized_ = false;
  bool qcqp_time_optimized_ = false;
};

}  // namespace mav_trajectory_generation

#endif  // MAV_TUBE_TRAJECTORY_GENERATION_AMD_POLYNOMIAL_OPTIMIZATION_NONLINEAR_H_
