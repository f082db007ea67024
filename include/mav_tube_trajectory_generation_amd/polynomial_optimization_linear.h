// polynomial_optimization_linear.h — PolynomialOptimization<N>, the
// single-trajectory C++ API of the reference
// (include/mav_tube_trajectory_generation/polynomial_optimization_linear.h:
// 45-285, impl/polynomial_optimization_linear_impl.h "linear_impl"), as a
// shim over the gfx950 batched solver (include/mtg_hip.h).
//
// Same class / method names, argument meaning and error behaviour (MTG_CHECK
// aborts where the reference CHECK-aborts).  What runs where:
//   * constraint bookkeeping (setupConstraintReorderingMatrix, linear_impl:
//     171-252) — host, index work only; it defines the plan's pattern;
//   * solveLinear (R assembly, R_pp solve, coefficients, cost,
//     linear_impl:306-379, 254-275, 113-130) — one mtg_linear_solve launch;
//   * setFreeConstraints -> coefficients (linear_impl:497-506, 254-275) —
//     one mtg_coeffs_from_constraints launch;
//   * getA / getAInverse / getR (linear_impl:509-544) — per-segment blocks
//     from mtg_segment_matrices, scattered through M on the host;
//   * the static helpers setupMappingMatrix / invertMappingMatrix /
//     computeQuadraticCostJacobian (linear_impl:101-111, 132-169, 557-573)
//     are host utilities on one N x N matrix, as in the reference; the solve
//     path never calls them.
// There is no CPU solve: without a HIP device solveLinear fails its check.
//
// Differences from the reference, all deliberate:
//   * Eigen types are replaced by VectorXd / MatrixXd of linalg.h
//     (SquareMatrix is an N x N MatrixXd);
//   * the unconditional debug prints of updateSegmentTimes / solveLinear
//     (linear_impl:287-292, 370) are not reproduced;
//   * setupFromPositons (header :79) is declared but never defined in the
//     reference and is not provided;
//   * computeMaximumOfMagnitude (linear_impl:449-487) runs on the device:
//     mtg_max_magnitude, or with a candidate list mtg_magnitude_candidates
//     (per segment 0, T, then the real roots ascending; a multiple root
//     once, where RPOLY's cluster passes the |Im| test 0..m times).  The
//     static per-segment helpers computeSegmentMaximumMagnitudeCandidates
//     (BySampling) (:389-447) are host arithmetic on one Segment, as in
//     the reference.
#ifndef MAV_TUBE_TRAJECTORY_GENERATION_AMD_POLYNOMIAL_OPTIMIZATION_LINEAR_H_
#define MAV_TUBE_TRAJECTORY_GENERATION_AMD_POLYNOMIAL_OPTIMIZATION_LINEAR_H_

#include <cmath>
#include <cstdint>
#include <memory>
#include <ostream>
#include <utility>
#include <vector>

#include "mav_tube_trajectory_generation_amd/device.h"
#include "mav_tube_trajectory_generation_amd/extremum.h"
#include "mav_tube_trajectory_generation_amd/polynomial.h"
#include "mav_tube_trajectory_generation_amd/segment.h"
#include "mav_tube_trajectory_generation_amd/trajectory.h"
#include "mav_tube_trajectory_generation_amd/vertex.h"

namespace mav_trajectory_generation {

namespace internal {
struct PlanDeleter {
  void operator()(mtg_plan* p) const {
    if (p) mtg_plan_destroy(p);
  }
};
typedef std::shared_ptr<mtg_plan> PlanPtr;

inline PlanPtr makePlan(int N, int D, int r, int S, const std::vector<uint8_t>& mask) {
  mtg_plan* p = nullptr;
  checkStatus(mtg_plan_create(defaultContext(), N, D, r, S, mask.data(), &p),
              "mtg_plan_create");
  return PlanPtr(p, PlanDeleter());
}

// Inverse by partial-pivot LU and one triangular solve pair per column (the
// method of Eigen's fixed-size inverse() used at linear_impl:160-161).
inline MatrixXd smallInverse(const MatrixXd& a) {
  const long n = a.rows();
  MatrixXd lu(a);
  std::vector<long> perm(n);
  for (long i = 0; i < n; ++i) perm[i] = i;
  for (long k = 0; k < n; ++k) {
    long p = k;
    for (long i = k + 1; i < n; ++i)
      if (std::fabs(lu(i, k)) > std::fabs(lu(p, k))) p = i;
    if (p != k) {
      for (long j = 0; j < n; ++j) std::swap(lu(k, j), lu(p, j));
      std::swap(perm[k], perm[p]);
    }
    for (long i = k + 1; i < n; ++i) {
      lu(i, k) /= lu(k, k);
      for (long j = k + 1; j < n; ++j) lu(i, j) -= lu(i, k) * lu(k, j);
    }
  }
  MatrixXd inv(n, n);
  std::vector<double> y(n);
  for (long c = 0; c < n; ++c) {
    for (long i = 0; i < n; ++i) {
      double s = perm[i] == c ? 1.0 : 0.0;
      for (long j = 0; j < i; ++j) s -= lu(i, j) * y[j];
      y[i] = s;
    }
    for (long i = n - 1; i >= 0; --i) {
      double s = y[i];
      for (long j = i + 1; j < n; ++j) s -= lu(i, j) * y[j];
      y[i] = s / lu(i, i);
    }
    for (long i = 0; i < n; ++i) inv(i, c) = y[i];
  }
  return inv;
}
}  // namespace internal

template <int _N = 10>
class PolynomialOptimization {
  static_assert(_N % 2 == 0, "The number of coefficients has to be even.");

 public:
  enum { N = _N };
  static constexpr int kHighestDerivativeToOptimize = N / 2 - 1;
  typedef MatrixXd SquareMatrix;  // N x N
  typedef std::vector<SquareMatrix> SquareMatrixVector;

  explicit PolynomialOptimization(size_t dimension)
      : dimension_(dimension),
        derivative_to_optimize_(derivative_order::INVALID),
        n_vertices_(0),
        n_segments_(0),
        n_all_constraints_(0),
        n_fixed_constraints_(0),
        n_free_constraints_(0) {
    MTG_CHECK(dimension >= 1 && dimension <= 4,
              "dimension " << dimension << " not supported (1..4)");
    fixed_constraints_compact_.resize(dimension_);
    free_constraints_compact_.resize(dimension_);
  }
  virtual ~PolynomialOptimization() {}

  // linear_impl:46-99.
  virtual bool setupFromVertices(const Vertex::Vector& vertices,
                                 const std::vector<double>& segment_times,
                                 int derivative_to_optimize = kHighestDerivativeToOptimize) {
    MTG_CHECK(derivative_to_optimize >= 0 &&
                  derivative_to_optimize <= kHighestDerivativeToOptimize,
              "You tried to optimize the " << derivative_to_optimize
                                           << "th derivative of position on a " << N
                                           << "th order polynomial.");
    derivative_to_optimize_ = derivative_to_optimize;
    vertices_ = vertices;
    segment_times_ = segment_times;
    n_vertices_ = vertices.size();
    n_segments_ = n_vertices_ - 1;
    segments_.assign(n_segments_, Segment(N, static_cast<int>(dimension_)));
    MTG_CHECK(n_vertices_ == segment_times.size() + 1,
              "Size of times must be one less than positions.");
    for (size_t v = 0; v < n_vertices_; ++v) {
      Vertex& vertex = vertices_[v];
      MTG_CHECK(static_cast<size_t>(vertex.D()) == dimension_,
                "vertex " << v << " has dimension " << vertex.D());
      bool valid = true;
      Vertex tmp(dimension_);
      for (auto it = vertex.cBegin(); it != vertex.cEnd(); ++it) {
        if (it->first > kHighestDerivativeToOptimize) {
          valid = false;
          std::ostringstream os;
          os << "Invalid constraint on vertex " << v << ": maximum possible derivative is "
             << kHighestDerivativeToOptimize << ", but was set to " << it->first
             << ". Ignoring constraint";
          internal::warn(os.str());
        } else {
          tmp.addConstraint(it->first, it->second);
        }
      }
      if (!valid) vertex = tmp;
    }
    updateSegmentTimes(segment_times);
    setupConstraintReorderingMatrix();
    return true;
  }

  // A = [A(t=0); A(t=T)], rows = baseCoeffsWithTime (linear_impl:101-111).
  static void setupMappingMatrix(double segment_time, SquareMatrix* A) {
    MTG_CHECK(A != nullptr, "A must not be null");
    A->resize(N, N);
    for (int i = 0; i < N / 2; ++i) {
      const VectorXd r0 = Polynomial::baseCoeffsWithTime(N, i, 0.0);
      const VectorXd rT = Polynomial::baseCoeffsWithTime(N, i, segment_time);
      for (int j = 0; j < N; ++j) {
        (*A)(i, j) = r0[j];
        (*A)(i + N / 2, j) = rT[j];
      }
    }
  }

  // Schur-complement inverse [diag^-1 0; -D^-1 C diag^-1 D^-1]
  // (linear_impl:132-169).
  static void invertMappingMatrix(const SquareMatrix& A, SquareMatrix* Ainv) {
    MTG_CHECK(Ainv != nullptr, "Ainv must not be null");
    MTG_CHECK(A.rows() == N && A.cols() == N, "mapping matrix must be N x N");
    const int M = N / 2;
    MatrixXd C(M, M), Dm(M, M);
    for (int i = 0; i < M; ++i)
      for (int j = 0; j < M; ++j) {
        C(i, j) = A(M + i, j);
        Dm(i, j) = A(M + i, M + j);
      }
    const MatrixXd Dinv = internal::smallInverse(Dm);
    Ainv->resize(N, N);
    for (int i = 0; i < M; ++i) (*Ainv)(i, i) = 1.0 / A(i, i);
    for (int i = 0; i < M; ++i)
      for (int j = 0; j < M; ++j) {
        double s = 0.0;
        for (int k = 0; k < M; ++k) s += Dinv(i, k) * C(k, j);
        (*Ainv)(M + i, j) = -s / A(j, j);
        (*Ainv)(M + i, M + j) = Dinv(i, j);
      }
  }

  // 0.5 * sum_s sum_d c^T Q_s c with the current coefficients and times
  // (linear_impl:113-130).
  double computeCost() const {
    MTG_CHECK(n_segments_ == segments_.size(), "setupFromVertices not called");
    if (cost_valid_) return cost_;
    // Times changed since the coefficients were computed: Q(T) from the
    // device, quadratic form here (S * D dot products).
    std::vector<double> Q = segmentMatrices(0);
    double cost = 0.0;
    for (size_t s = 0; s < n_segments_; ++s)
      for (size_t d = 0; d < dimension_; ++d) {
        const VectorXd c = segments_[s][d].getCoefficients(derivative_order::POSITION);
        const double* q = Q.data() + s * N * N;
        for (int i = 0; i < N; ++i)
          for (int j = 0; j < N; ++j) cost += c[i] * q[i * N + j] * c[j];
      }
    return 0.5 * cost;
  }

  // linear_impl:277-304.
  void updateSegmentTimes(const std::vector<double>& segment_times) {
    MTG_CHECK(segment_times.size() == n_segments_,
              "Number of segment times (" << segment_times.size()
                                          << ") does not match number of segments ("
                                          << n_segments_ << ")");
    for (double t : segment_times)
      MTG_CHECK(t > 0, "Segment times need to be greater than zero");
    segment_times_ = segment_times;
    cost_valid_ = false;
  }

  // linear_impl:337-379 (+ computeCost, cached).  Returns false only when the
  // device reports a non-positive pivot (R_pp not SPD).
  bool solveLinear() {
    MTG_CHECK(derivative_to_optimize_ >= 0 &&
                  derivative_to_optimize_ <= kHighestDerivativeToOptimize,
              "setupFromVertices not called");
    if (n_free_constraints_ == 0) {
      internal::warn(
          "No free constraints set in the vertices. Polynomial can not be optimized. "
          "Outputting fully constrained polynomial.");
      updateSegmentsFromCompactConstraints();
      return true;
    }
    const int D = static_cast<int>(dimension_);
    const std::vector<double> df = packFixed();
    std::vector<double> coeffs(n_segments_ * D * N), dp(D * n_free_constraints_);
    double cost = 0.0;
    int32_t st = 0;
    const int rc = mtg_linear_solve_host(plan_.get(), 1, df.data(), segment_times_.data(),
                                         coeffs.data(), &cost, dp.data(), &st);
    MTG_CHECK(rc == MTG_OK || rc == MTG_ERR_NUMERIC,
              "mtg_linear_solve_host failed: " << mtg_status_string(rc));
    for (int d = 0; d < D; ++d) {
      VectorXd v(static_cast<long>(n_free_constraints_));
      for (size_t p = 0; p < n_free_constraints_; ++p) v[p] = dp[d * n_free_constraints_ + p];
      free_constraints_compact_[d] = v;
    }
    setSegmentsFrom(coeffs);
    cost_ = cost;
    cost_valid_ = true;
    return st == MTG_TRAJ_OK;
  }

  // Candidate times of the maximum magnitude of one segment over all its
  // dimensions (linear_impl:389-409): Segment::
  // computeMinMaxMagnitudeCandidateTimes on dimensions 0 .. D-1.
  template <int Derivative>
  static bool computeSegmentMaximumMagnitudeCandidates(const Segment& segment, double t_start,
                                                       double t_stop,
                                                       std::vector<double>* candidates) {
    return computeSegmentMaximumMagnitudeCandidates(Derivative, segment, t_start, t_stop,
                                                    candidates);
  }
  static bool computeSegmentMaximumMagnitudeCandidates(int derivative, const Segment& segment,
                                                       double t_start, double t_stop,
                                                       std::vector<double>* candidates) {
    MTG_CHECK(candidates != nullptr, "candidates must not be null");
    MTG_CHECK(N - derivative - 1 > 0, "N-Derivative-1 has to be greater 0");
    std::vector<int> dimensions;
    for (int i = 0; i < segment.D(); ++i) dimensions.push_back(i);
    return segment.computeMinMaxMagnitudeCandidateTimes(derivative, t_start, t_stop, dimensions,
                                                        candidates);
  }

  // The same candidates by sampling every dt (linear_impl:411-447): a change
  // of the sign of d|p^(Derivative)|/dt between samples with
  // |p^(Derivative+1)| < 1e-2 at the earlier sample appends that sample's
  // time.  A debugging / test helper, as in the reference.
  template <int Derivative>
  static void computeSegmentMaximumMagnitudeCandidatesBySampling(
      const Segment& segment, double t_start, double t_stop, double dt,
      std::vector<double>* candidates) {
    MTG_CHECK(candidates != nullptr, "candidates must not be null");
    const VectorXd value_start = segment.evaluate(t_start - dt, Derivative);
    VectorXd value_old = segment.evaluate(t_start, Derivative);
    // the direction from t_start - dt to t_start: t_start itself may be an
    // extremum (start and end vertices)
    double direction = value_old.norm() - value_start.norm();
    for (double t = t_start + dt; t < t_stop + dt; t += dt) {
      const VectorXd value_new = segment.evaluate(t, Derivative);
      const double direction_new = value_new.norm() - value_old.norm();
      if (std::signbit(direction) != std::signbit(direction_new)) {
        const VectorXd value_deriv = segment.evaluate(t - dt, Derivative + 1);
        if (value_deriv.norm() < 1e-2) candidates->push_back(t - dt);
      }
      value_old = value_new;
      direction = direction_new;
    }
  }

  // linear_impl:449-487: the maximum of |p^(Derivative)| over all segments,
  // by the device extremum search (mtg_max_magnitude); with `candidates`,
  // the device candidate lists (mtg_magnitude_candidates) in the
  // reference's order — per segment (0, T, roots...) with its index, then
  // the last segment's end once more — and the first largest of them.
  template <int Derivative>
  Extremum computeMaximumOfMagnitude(std::vector<Extremum>* candidates) const {
    return computeMaximumOfMagnitude(Derivative, candidates);
  }
  Extremum computeMaximumOfMagnitude(int derivative, std::vector<Extremum>* candidates) const {
    MTG_CHECK(N - derivative - 1 > 0, "N-Derivative-1 has to be greater 0");
    if (candidates != nullptr) return maximumWithCandidates(derivative, candidates);
    const int D = static_cast<int>(dimension_);
    const int S = static_cast<int>(n_segments_);
    std::vector<double> coeffs(static_cast<size_t>(S) * D * N);
    std::vector<double> times(S);
    for (int s = 0; s < S; ++s) {
      times[s] = segments_[s].getTime();
      for (int d = 0; d < D; ++d) {
        const VectorXd c = segments_[s][d].getCoefficients(0);
        for (int k = 0; k < N; ++k) coeffs[(static_cast<size_t>(s) * D + d) * N + k] = c[k];
      }
    }
    internal::DeviceBuffer<double> d_c, d_t, d_time(1), d_value(1);
    internal::DeviceBuffer<int32_t> d_seg(1);
    d_c.upload(coeffs);
    d_t.upload(times);
    internal::checkStatus(mtg_max_magnitude(N, D, S, 1, d_c.get(), d_t.get(), derivative,
                                            d_time.get(), d_value.get(), d_seg.get(), nullptr),
                          "mtg_max_magnitude");
    internal::synchronize();
    Extremum e;
    int32_t seg = 0;
    d_time.download(&e.time, 1);
    d_value.download(&e.value, 1);
    d_seg.download(&seg, 1);
    e.segment_idx = seg;
    return e;
  }

  Extremum maximumWithCandidates(int derivative, std::vector<Extremum>* candidates) const {
    candidates->clear();
    const int D = static_cast<int>(dimension_);
    const int S = static_cast<int>(n_segments_);
    const int C = 2 * (N - derivative) - 1;  // 2 + the degree of f: never overflows
    std::vector<double> coeffs(static_cast<size_t>(S) * D * N);
    std::vector<double> times(S);
    for (int s = 0; s < S; ++s) {
      times[s] = segments_[s].getTime();
      for (int d = 0; d < D; ++d) {
        const VectorXd c = segments_[s][d].getCoefficients(0);
        for (int k = 0; k < N; ++k) coeffs[(static_cast<size_t>(s) * D + d) * N + k] = c[k];
      }
    }
    internal::DeviceBuffer<double> d_c, d_t, d_ct(static_cast<size_t>(S) * C),
        d_cv(static_cast<size_t>(S) * C);
    internal::DeviceBuffer<int32_t> d_n(S);
    d_c.upload(coeffs);
    d_t.upload(times);
    internal::checkStatus(mtg_magnitude_candidates(N, D, S, 1, d_c.get(), d_t.get(), derivative,
                                                   C, d_ct.get(), d_cv.get(), d_n.get(),
                                                   nullptr),
                          "mtg_magnitude_candidates");
    internal::synchronize();
    const std::vector<double> ct = d_ct.download(), cv = d_cv.download();
    const std::vector<int32_t> n = d_n.download();
    Extremum extremum;
    for (int s = 0; s < S; ++s)
      for (int k = 0; k < n[s] && k < C; ++k) {
        const Extremum c(ct[static_cast<size_t>(s) * C + k], cv[static_cast<size_t>(s) * C + k], s);
        if (extremum < c) extremum = c;
        candidates->push_back(c);
      }
    // the last segment's end once more (linear_impl:477-484)
    const Segment& last = segments_.back();
    const Extremum c(last.getTime(), last.evaluate(last.getTime(), derivative).norm(), S - 1);
    if (extremum < c) extremum = c;
    candidates->push_back(c);
    return extremum;
  }

  void getTrajectory(Trajectory* trajectory) const {
    MTG_CHECK(trajectory != nullptr, "trajectory must not be null");
    trajectory->setSegments(segments_);
  }

  void getVertices(Vertex::Vector* vertices) const {
    MTG_CHECK(vertices != nullptr, "vertices must not be null");
    *vertices = vertices_;
  }
  void getSegments(Segment::Vector* segments) const {
    MTG_CHECK(segments != nullptr, "segments must not be null");
    *segments = segments_;
  }
  void getSegmentTimes(std::vector<double>* segment_times) const {
    MTG_CHECK(segment_times != nullptr, "segment_times must not be null");
    *segment_times = segment_times_;
  }
  void getFreeConstraints(std::vector<VectorXd>* free_constraints) const {
    MTG_CHECK(free_constraints != nullptr, "free_constraints must not be null");
    *free_constraints = free_constraints_compact_;
  }
  // linear_impl:497-506.
  void setFreeConstraints(const std::vector<VectorXd>& free_constraints) {
    MTG_CHECK(free_constraints.size() == dimension_, "one vector per dimension");
    for (const VectorXd& v : free_constraints)
      MTG_CHECK(static_cast<size_t>(v.size()) == n_free_constraints_,
                "free constraint vector has size " << v.size());
    free_constraints_compact_ = free_constraints;
    updateSegmentsFromCompactConstraints();
  }
  void getFixedConstraints(std::vector<VectorXd>* fixed_constraints) const {
    MTG_CHECK(fixed_constraints != nullptr, "fixed_constraints must not be null");
    *fixed_constraints = fixed_constraints_compact_;
  }

  // Q_ij = 2 base(r,i) base(r,j) t^(i+j-2r+1) / (i+j-2r+1)
  // (linear_impl:557-573).
  static void computeQuadraticCostJacobian(int derivative, double t,
                                           SquareMatrix* cost_jacobian) {
    MTG_CHECK(cost_jacobian != nullptr, "cost_jacobian must not be null");
    MTG_CHECK(derivative < N, "derivative " << derivative << " >= N");
    cost_jacobian->resize(N, N);
    const MatrixXd& base = Polynomial::baseCoefficients();
    for (int col = 0; col < N - derivative; ++col)
      for (int row = 0; row < N - derivative; ++row) {
        const double exponent = (N - 1 - derivative) * 2 + 1 - row - col;
        (*cost_jacobian)(N - 1 - row, N - 1 - col) =
            base(derivative, N - 1 - row) * base(derivative, N - 1 - col) *
            std::pow(t, exponent) * 2.0 / exponent;
      }
  }

  size_t getDimension() const { return dimension_; }
  size_t getNumberSegments() const { return n_segments_; }
  size_t getNumberAllConstraints() const { return n_all_constraints_; }
  size_t getNumberFixedConstraints() const { return n_fixed_constraints_; }
  size_t getNumberFreeConstraints() const { return n_free_constraints_; }
  int getDerivativeToOptimize() const { return derivative_to_optimize_; }

  // Block-diagonal A^-1 (linear_impl:509-518); blocks from the device.
  void getAInverse(MatrixXd* A_inv) const {
    MTG_CHECK(A_inv != nullptr, "A_inv must not be null");
    *A_inv = blockDiagonal(segmentMatrices(2));
  }
  // Dense reordering matrix M (linear_impl:520-523).
  void getM(MatrixXd* M) const {
    MTG_CHECK(M != nullptr, "M must not be null");
    M->resize(static_cast<long>(n_all_constraints_),
              static_cast<long>(n_fixed_constraints_ + n_free_constraints_));
    for (size_t row = 0; row < n_all_constraints_; ++row) (*M)(row, column_of_row_[row]) = 1.0;
  }
  // R = M^T blkdiag(A^-T Q A^-1) M (linear_impl:306-335, 525-532); H blocks
  // from the device, scattered through M here.
  void getR(MatrixXd* R) const {
    MTG_CHECK(R != nullptr, "R must not be null");
    const std::vector<double> H = segmentMatrices(3);
    const long n = static_cast<long>(n_fixed_constraints_ + n_free_constraints_);
    R->resize(n, n);
    for (size_t s = 0; s < n_segments_; ++s)
      for (int a = 0; a < N; ++a)
        for (int b = 0; b < N; ++b)
          (*R)(column_of_row_[s * N + a], column_of_row_[s * N + b]) +=
              H[(s * N + a) * N + b];
  }
  // Block-diagonal A (linear_impl:534-549); blocks from the device.
  void getA(MatrixXd* A) const {
    MTG_CHECK(A != nullptr, "A must not be null");
    *A = blockDiagonal(segmentMatrices(1));
  }
  // Row-normalised M^T (linear_impl:551-560).
  void getMpinv(MatrixXd* M_pinv) const {
    MTG_CHECK(M_pinv != nullptr, "M_pinv must not be null");
    MatrixXd M;
    getM(&M);
    *M_pinv = M.transpose();
    for (long i = 0; i < M_pinv->rows(); ++i) {
      double s = 0.0;
      for (long j = 0; j < M_pinv->cols(); ++j) s += (*M_pinv)(i, j);
      for (long j = 0; j < M_pinv->cols(); ++j) (*M_pinv)(i, j) /= s;
    }
  }

  void printReorderingMatrix(std::ostream& stream) const {
    MatrixXd M;
    getM(&M);
    stream << "Mapping matrix:\n";
    for (long i = 0; i < M.rows(); ++i) {
      for (long j = 0; j < M.cols(); ++j) stream << (j ? " " : "") << M(i, j);
      stream << "\n";
    }
  }

  // Constraint pattern of the plan: mask[v * N/2 + k] != 0 iff vertex v fixes
  // derivative k.  Batched callers (mtg_plan_create) use the same layout.
  const std::vector<uint8_t>& getFixedMask() const { return mask_; }
  // The device plan of that pattern (valid after setupFromVertices).
  const mtg_plan* getPlan() const { return plan_.get(); }

 protected:
  // The reference's std::set<Constraint> ordering by (vertex, derivative)
  // (linear_impl:171-252, header :288-305): fixed columns first, then free.
  void setupConstraintReorderingMatrix() {
    const int M = N / 2;
    std::vector<uint8_t> mask(n_vertices_ * M, 0);
    for (size_t v = 0; v < n_vertices_; ++v)
      for (int k = 0; k < M; ++k) mask[v * M + k] = vertices_[v].hasConstraint(k) ? 1 : 0;
    setupPattern(mask);
  }

  // M, d_f and the device plan for a given fixed pattern; fixed values come
  // from the vertices' constraints.
  void setupPattern(const std::vector<uint8_t>& mask) {
    const int M = N / 2;
    const size_t V = n_vertices_;
    mask_ = mask;
    std::vector<int> col_of(V * M, -1);
    n_fixed_constraints_ = 0;
    for (size_t v = 0; v < V; ++v)
      for (int k = 0; k < M; ++k)
        if (mask_[v * M + k]) col_of[v * M + k] = static_cast<int>(n_fixed_constraints_++);
    n_free_constraints_ = 0;
    for (size_t v = 0; v < V; ++v)
      for (int k = 0; k < M; ++k)
        if (!mask_[v * M + k])
          col_of[v * M + k] = static_cast<int>(n_fixed_constraints_ + n_free_constraints_++);
    // all_constraints: vertex v once at the ends, twice in between; row
    // s*N + k is vertex s, row s*N + M + k vertex s+1.
    n_all_constraints_ = N * n_segments_;
    column_of_row_.assign(n_all_constraints_, 0);
    for (size_t s = 0; s < n_segments_; ++s)
      for (int k = 0; k < M; ++k) {
        column_of_row_[s * N + k] = col_of[s * M + k];
        column_of_row_[s * N + M + k] = col_of[(s + 1) * M + k];
      }
    for (size_t d = 0; d < dimension_; ++d) {
      VectorXd df(static_cast<long>(n_fixed_constraints_));
      long f = 0;
      for (size_t v = 0; v < V; ++v)
        for (int k = 0; k < M; ++k)
          if (mask_[v * M + k]) {
            VectorXd value;
            MTG_CHECK(vertices_[v].getConstraint(k, &value),
                      "vertex " << v << " has no constraint on derivative " << k);
            df[f++] = value[d];
          }
      fixed_constraints_compact_[d] = df;
    }
    plan_ = internal::makePlan(N, static_cast<int>(dimension_), derivative_to_optimize_,
                               static_cast<int>(n_segments_), mask_);
  }

  // Coefficients (and cost) from the current d_f, d_p on the device
  // (linear_impl:254-275).
  void updateSegmentsFromCompactConstraints() {
    const int D = static_cast<int>(dimension_);
    const std::vector<double> df = packFixed();
    std::vector<double> dp(D * n_free_constraints_, 0.0);
    for (int d = 0; d < D; ++d) {
      const VectorXd& v = free_constraints_compact_[d];
      if (static_cast<size_t>(v.size()) != n_free_constraints_) continue;  // unsolved: zeros
      for (size_t p = 0; p < n_free_constraints_; ++p) dp[d * n_free_constraints_ + p] = v[p];
    }
    internal::DeviceBuffer<double> d_df, d_dp, d_t, d_c, d_cost;
    d_df.upload(df);
    d_dp.upload(dp);
    d_t.upload(segment_times_);
    d_c.resize(n_segments_ * D * N);
    d_cost.resize(1);
    internal::checkStatus(
        mtg_coeffs_from_constraints(plan_.get(), 1, d_df.get(), d_dp.get(), d_t.get(),
                                    d_c.get(), d_cost.get(), nullptr, nullptr),
        "mtg_coeffs_from_constraints");
    internal::synchronize();
    setSegmentsFrom(d_c.download());
    d_cost.download(&cost_, 1);
    cost_valid_ = true;
  }

  std::vector<double> packFixed() const {
    std::vector<double> df(dimension_ * n_fixed_constraints_);
    for (size_t d = 0; d < dimension_; ++d)
      for (size_t f = 0; f < n_fixed_constraints_; ++f)
        df[d * n_fixed_constraints_ + f] = fixed_constraints_compact_[d][f];
    return df;
  }

  void setSegmentsFrom(const std::vector<double>& coeffs) {
    const int D = static_cast<int>(dimension_);
    for (size_t s = 0; s < n_segments_; ++s) {
      Segment& seg = segments_[s];
      seg.setTime(segment_times_[s]);
      for (int d = 0; d < D; ++d) {
        VectorXd c(N);
        for (int k = 0; k < N; ++k) c[k] = coeffs[(s * D + d) * N + k];
        seg[d] = Polynomial(N, c);
      }
    }
  }

  // Per-segment Q (which=0), A (1), A^-1 (2) or H (3) at the current times,
  // S x N x N, computed by mtg_segment_matrices.
  std::vector<double> segmentMatrices(int which) const {
    MTG_CHECK(derivative_to_optimize_ >= 0, "setupFromVertices not called");
    const size_t n = n_segments_;
    internal::DeviceBuffer<double> d_t, d_out(n * N * N);
    d_t.upload(segment_times_);
    double* out[4] = {nullptr, nullptr, nullptr, nullptr};
    out[which] = d_out.get();
    internal::checkStatus(mtg_segment_matrices(internal::defaultContext(), N,
                                               derivative_to_optimize_, static_cast<int64_t>(n),
                                               d_t.get(), out[0], out[1], out[2], out[3],
                                               nullptr),
                          "mtg_segment_matrices");
    internal::synchronize();
    return d_out.download();
  }

  MatrixXd blockDiagonal(const std::vector<double>& blocks) const {
    MatrixXd m(static_cast<long>(N * n_segments_), static_cast<long>(N * n_segments_));
    for (size_t s = 0; s < n_segments_; ++s)
      for (int a = 0; a < N; ++a)
        for (int b = 0; b < N; ++b) m(s * N + a, s * N + b) = blocks[(s * N + a) * N + b];
    return m;
  }

  size_t dimension_;
  int derivative_to_optimize_;
  size_t n_vertices_;
  size_t n_segments_;
  size_t n_all_constraints_;
  size_t n_fixed_constraints_;
  size_t n_free_constraints_;
  Vertex::Vector vertices_;
  Segment::Vector segments_;
  std::vector<double> segment_times_;
  std::vector<VectorXd> fixed_constraints_compact_;
  std::vector<VectorXd> free_constraints_compact_;
  std::vector<uint8_t> mask_;
  std::vector<int> column_of_row_;  // M as a row -> column map
  internal::PlanPtr plan_;
  double cost_ = 0.0;
  bool cost_valid_ = false;
};

}  // namespace mav_trajectory_generation

#endif  // MAV_TUBE_TRAJECTORY_GENERATION_AMD_POLYNOMIAL_OPTIMIZATION_LINEAR_H_
