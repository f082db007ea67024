// polynomial_optimization_qcqp.h — PolynomialOptimizationConstrained<N>, the
// tube-constrained QCQP of the reference
// (include/mav_tube_trajectory_generation/polynomial_optimization_qcqp.h:
// 24-82, impl/polynomial_optimization_qcqp_impl.h "qcqp_impl"), as a shim
// over the gfx950 tube kernels (mtg_tube_solve / mtg_tube_residuals).
//
// Pattern (setupConstraintReorderingMatrixkDim, qcqp_impl:18-118): start and
// end vertex fix derivatives 0..N/2-1, every derivative of an intermediate
// vertex is free (intermediate positions only define the tube geometry).
// The per-dimension compact vectors use the reference's layout: d_f[d] =
// [start derivs; end derivs], d_p[d] = intermediate (vertex, derivative).
//
// solveQCQP replaces the MOSEK solve (qcqp_impl:476-788) with the batched
// primal-dual interior-point method of mtg_tube_solve (B = 1).  It returns 0
// when the device reports convergence and the MTG_TRAJ_* status otherwise
// (the reference returns MOSEK's MSKrescodee, 0 = MSK_RES_OK).  Control-point
// maps use the segment times given to setupFromVertices, as the reference
// does (built once at setup, qcqp_impl:152-157); Q and A^-1 use the current
// times.  Dimension must be 3 (hard-coded in qcqp_impl:377-384, 777-781).
//
// Deliberate difference: the reference's solveLinear override assigns
// -R_pf d_f instead of the solution to the free derivatives
// (qcqp_impl:246-247); here solveLinear returns the unconstrained minimiser
// for the tube pattern (the QCQP without inequality constraints).
#ifndef MAV_TUBE_TRAJECTORY_GENERATION_AMD_POLYNOMIAL_OPTIMIZATION_QCQP_H_
#define MAV_TUBE_TRAJECTORY_GENERATION_AMD_POLYNOMIAL_OPTIMIZATION_QCQP_H_

#include <utility>
#include <vector>

#include "mav_tube_trajectory_generation_amd/polynomial_optimization_linear.h"

namespace mav_trajectory_generation {

template <int _N = 10>
class PolynomialOptimizationConstrained : public PolynomialOptimization<_N> {
  typedef PolynomialOptimization<_N> Base;

 public:
  using Base::N;
  using Base::kHighestDerivativeToOptimize;

  explicit PolynomialOptimizationConstrained(size_t dimension) : Base(dimension) {
    MTG_CHECK(dimension == 3, "the tube QCQP is three-dimensional (qcqp_impl:377-384)");
  }

  // qcqp_impl:122-186.
  bool setupFromVertices(const Vertex::Vector& vertices, const std::vector<double>& times,
                         const std::vector<std::pair<double, double>>& radii,
                         int derivative_to_optimize) {
    MTG_CHECK(vertices.size() == radii.size() + 1,
              "Size of radii must be one less than positions.");
    MTG_CHECK(vertices.size() >= 2, "need at least two vertices");
    segment_radii_ = radii;
    times_cp_ = times;
    Base::setupFromVertices(vertices, times, derivative_to_optimize);
    // The base class built the vertices' own pattern; replace it by the
    // tube pattern.
    const int M = N / 2;
    std::vector<uint8_t> mask((this->n_segments_ + 1) * M, 0);
    for (int k = 0; k < M; ++k) {
      mask[k] = 1;
      mask[this->n_segments_ * M + k] = 1;
    }
    for (size_t v = 0; v < this->n_vertices_; ++v)
      MTG_CHECK(this->vertices_[v].hasConstraint(derivative_order::POSITION),
                "vertex " << v << " needs a position (tube geometry)");
    this->setupPattern(mask);
    return true;
  }
  // Single-pattern setup without radii is not meaningful for the tube class;
  // keep the base overload reachable for code that calls it explicitly.
  using Base::setupFromVertices;

  // Tube QCQP on the device (qcqp_impl:476-788).  The reference returns
  // MOSEK's response code (0 = MSK_RES_OK); this returns the device status
  // (include/mtg_hip.h MTG_TRAJ_*):
  //   0 MTG_TRAJ_OK             converged to tol;
  //   4 MTG_TRAJ_NEAR_OPTIMAL   the interior-point KKT system broke down with
  //                             every residual within 1e3 x tol: the solution
  //                             is written and usable (callers that test for 0
  //                             only must also accept 4, see qcqpUsable);
  //   2, 3                      not SPD / iteration cap: the point is written
  //                             but is not an optimum.
  // Since round 3 the IPM's complementarity floor turns most
  // former breakdowns into status 0; the remaining near-optimal stops are 4
  // (2 of the 4,096 config-3 problems with round 6's scaled start, DESIGN.md
  // 5.3).
  static bool qcqpUsable(int status) {
    return status == MTG_TRAJ_OK || status == MTG_TRAJ_NEAR_OPTIMAL;
  }
  int solveQCQP(double tol = 1e-10, int max_iter = 100) {
    const int S = static_cast<int>(this->n_segments_);
    const int M = N / 2;
    std::vector<double> pos, df, radii;
    packTubeInputs(&pos, &df, &radii);
    const size_t nx = static_cast<size_t>(3) * (S - 1) * M;
    internal::DeviceBuffer<double> d_pos, d_df, d_tcp, d_t, d_r, d_x(nx ? nx : 1),
        d_c(static_cast<size_t>(S) * 3 * N), d_cost(1);
    internal::DeviceBuffer<int32_t> d_it(1), d_st(1);
    d_pos.upload(pos);
    d_df.upload(df);
    d_tcp.upload(times_cp_);
    d_t.upload(this->segment_times_);
    d_r.upload(radii);
    internal::checkStatus(
        mtg_tube_solve(internal::defaultContext(), N, this->derivative_to_optimize_, S, 1,
                       d_pos.get(), d_df.get(), d_tcp.get(), d_t.get(), d_r.get(), tol,
                       max_iter, d_x.get(), d_c.get(), d_cost.get(), d_it.get(), d_st.get(),
                       nullptr),
        "mtg_tube_solve");
    internal::synchronize();
    const std::vector<double> x = d_x.download();
    for (int d = 0; d < 3; ++d) {
      VectorXd v(static_cast<long>(this->n_free_constraints_));
      for (size_t p = 0; p < this->n_free_constraints_; ++p)
        v[p] = x[d * this->n_free_constraints_ + p];
      this->free_constraints_compact_[d] = v;
    }
    this->setSegmentsFrom(d_c.download());
    d_cost.download(&this->cost_, 1);
    this->cost_valid_ = true;
    d_it.download(&iterations_, 1);
    int32_t st = 0;
    d_st.download(&st, 1);
    return st;
  }

  // Inequality residuals g_k(x) (feasible iff <= 0) at the current free
  // derivatives, in the reference's constraint order (qcqp_impl:357-474).
  std::vector<double> getConstraintResiduals() const {
    const int S = static_cast<int>(this->n_segments_);
    const int n_con = mtg_tube_num_constraints(N, S);
    MTG_CHECK(n_con >= 0, "invalid tube size");
    std::vector<double> pos, df, radii, x;
    packTubeInputs(&pos, &df, &radii);
    for (int d = 0; d < 3; ++d) {
      const VectorXd& v = this->free_constraints_compact_[d];
      MTG_CHECK(static_cast<size_t>(v.size()) == this->n_free_constraints_,
                "no free derivatives yet: call solveQCQP or setFreeConstraints");
      for (long p = 0; p < v.size(); ++p) x.push_back(v[p]);
    }
    internal::DeviceBuffer<double> d_pos, d_df, d_tcp, d_t, d_r, d_x, d_res(n_con ? n_con : 1);
    d_pos.upload(pos);
    d_df.upload(df);
    d_tcp.upload(times_cp_);
    d_t.upload(this->segment_times_);
    d_r.upload(radii);
    d_x.upload(x);
    internal::checkStatus(
        mtg_tube_residuals(internal::defaultContext(), N, this->derivative_to_optimize_, S, 1,
                           d_pos.get(), d_df.get(), d_tcp.get(), d_t.get(), d_r.get(),
                           d_x.get(), d_res.get(), nullptr),
        "mtg_tube_residuals");
    internal::synchronize();
    std::vector<double> res = d_res.download();
    res.resize(n_con);
    return res;
  }

  // objectiveFunctionTime in the fork's form (nonlinear_impl:877-945, with
  // solveQCQP at :892): J(T) = computeCost() of the QCQP at T + time_penalty
  // (sum T)^2 [+ soft] (mtg_tube_time_cost; params.grad_mode 0 or 2).
  // Control-point maps stay at the setup times.
  double evaluateTimeCostQCQP(const std::vector<double>& segment_times,
                              const mtg_time_params& params, std::vector<double>* gradient,
                              int32_t* status = nullptr, double tol = 1e-10,
                              int max_iter = 100) const {
    const size_t S = this->n_segments_;
    MTG_CHECK(segment_times.size() == S, "segment_times has " << segment_times.size()
                                                              << " entries, need " << S);
    MTG_CHECK(params.grad_mode == 0 || gradient != nullptr, "gradient must not be null");
    std::vector<double> pos, df, radii;
    packTubeInputs(&pos, &df, &radii);
    internal::DeviceBuffer<double> d_pos, d_df, d_tcp, d_t, d_r, d_cost(1), d_g(S);
    internal::DeviceBuffer<int32_t> d_st(1);
    internal::DeviceBuffer<unsigned char> d_ws(
        workspaceBytes(static_cast<int>(S), params, 0));
    d_pos.upload(pos);
    d_df.upload(df);
    d_tcp.upload(times_cp_);
    d_t.upload(segment_times);
    d_r.upload(radii);
    internal::checkStatus(
        mtg_tube_time_cost(internal::defaultContext(), N, this->derivative_to_optimize_,
                           static_cast<int>(S), 1, d_pos.get(), d_df.get(), d_tcp.get(),
                           d_t.get(), d_r.get(), tol, max_iter, &params, d_cost.get(),
                           params.grad_mode ? d_g.get() : nullptr, d_st.get(), d_ws.get(),
                           d_ws.size(), nullptr),
        "mtg_tube_time_cost");
    internal::synchronize();
    double J = 0.0;
    d_cost.download(&J, 1);
    if (params.grad_mode) *gradient = d_g.download();
    if (status) d_st.download(status, 1);
    return J;
  }

  // optimizeTime over that objective (mtg_tube_time_optimize_ex): `times`
  // in = the setup times (also the control-point times), out = optimised
  // (NLopt's x with params.optimizer 1, LN_SBPLX).  *result (nullable): the
  // nlopt_result code.  Returns the trajectory status (MTG_TRAJ_*).
  int optimizeTimeQCQP(const mtg_time_params& params, int max_evals, std::vector<double>* times,
                       double* cost, int32_t* evals, double tol = 1e-10, int max_iter = 100,
                       int32_t* result = nullptr) const {
    MTG_CHECK(times != nullptr && times->size() == this->n_segments_, "times size");
    std::vector<double> pos, df, radii;
    packTubeInputs(&pos, &df, &radii);
    internal::DeviceBuffer<double> d_pos, d_df, d_t, d_r, d_cost(1);
    internal::DeviceBuffer<int32_t> d_ev(1), d_res(1), d_st(1);
    internal::DeviceBuffer<unsigned char> d_ws(
        workspaceBytes(static_cast<int>(this->n_segments_), params, 1));
    d_pos.upload(pos);
    d_df.upload(df);
    d_t.upload(*times);
    d_r.upload(radii);
    internal::checkStatus(
        mtg_tube_time_optimize_ex(internal::defaultContext(), N, this->derivative_to_optimize_,
                                  static_cast<int>(this->n_segments_), 1, d_pos.get(),
                                  d_df.get(), d_r.get(), d_t.get(), tol, max_iter, &params,
                                  max_evals, d_cost.get(), d_ev.get(), d_res.get(), d_st.get(),
                                  d_ws.get(), d_ws.size(), nullptr),
        "mtg_tube_time_optimize_ex");
    internal::synchronize();
    d_t.download(times->data(), times->size());
    if (cost) d_cost.download(cost, 1);
    if (evals) d_ev.download(evals, 1);
    if (result) d_res.download(result, 1);
    int32_t st = 0;
    d_st.download(&st, 1);
    return st;
  }

  void getSegmentRadii(std::vector<std::pair<double, double>>* segment_radii) const {
    MTG_CHECK(segment_radii != nullptr, "segment_radii must not be null");
    *segment_radii = segment_radii_;
  }
  // Interior-point iterations of the last solveQCQP.
  int getIterations() const { return iterations_; }

 private:
  static size_t workspaceBytes(int S, const mtg_time_params& params, int optimize) {
    const int64_t n = mtg_tube_time_workspace_bytes(N, S, 1, &params, optimize);
    internal::checkStatus(n < 0 ? static_cast<int>(n) : MTG_OK, "mtg_tube_time_workspace_bytes");
    return static_cast<size_t>(n);
  }

  // Device layouts of mtg_tube_*: positions (S+1) x 3, fixed values 3 x N
  // (start then end derivatives per dimension), radii S x 2.
  void packTubeInputs(std::vector<double>* pos, std::vector<double>* df,
                      std::vector<double>* radii) const {
    const int S = static_cast<int>(this->n_segments_);
    pos->assign(static_cast<size_t>(S + 1) * 3, 0.0);
    df->assign(static_cast<size_t>(3) * N, 0.0);
    radii->assign(static_cast<size_t>(S) * 2, 0.0);
    for (int v = 0; v <= S; ++v) {
      VectorXd p;
      this->vertices_[v].getConstraint(derivative_order::POSITION, &p);
      for (int d = 0; d < 3; ++d) (*pos)[v * 3 + d] = p[d];
    }
    for (int d = 0; d < 3; ++d)
      for (int j = 0; j < N; ++j) (*df)[d * N + j] = this->fixed_constraints_compact_[d][j];
    for (int s = 0; s < S; ++s) {
      (*radii)[2 * s] = segment_radii_[s].first;
      (*radii)[2 * s + 1] = segment_radii_[s].second;
    }
  }

  std::vector<std::pair<double, double>> segment_radii_;
  std::vector<double> times_cp_;
  int32_t iterations_ = 0;
};

}  // namespace mav_trajectory_generation

#endif  // MAV_TUBE_TRAJECTORY_GENERATION_AMD_POLYNOMIAL_OPTIMIZATION_QCQP_H_
