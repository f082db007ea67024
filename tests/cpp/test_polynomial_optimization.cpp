// C++ API tests: the reference's own test strategy
// (test/test_polynomial_optimization.cpp) run against the
// MI355X shims in include/mav_tube_trajectory_generation_amd/.  The checker
// is the oracle (oracle/mtg_oracle.h, liboracle.so): test infrastructure,
// never the thing under test.
//
//   test_polynomial_optimization host   -> tests that need no GPU (static
//        host utilities, generators, and that the solve path fails loudly
//        without a device)
//   test_polynomial_optimization gpu    -> the parity tests proper
#define MTG_CHECK_THROWS 1

#include <algorithm>
#include <chrono>
#include <fstream>
#include <random>
#include <sstream>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "mav_tube_trajectory_generation_amd/polynomial_optimization_nonlinear.h"
#include "mtg_oracle.h"

using namespace mav_trajectory_generation;

namespace {

int g_failures = 0;
int g_checks = 0;

#define EXPECT_TRUE(cond)                                                            \
  do {                                                                               \
    ++g_checks;                                                                      \
    if (!(cond)) {                                                                   \
      ++g_failures;                                                                  \
      std::fprintf(stderr, "  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);       \
    }                                                                                \
  } while (0)

#define EXPECT_LE(a, b)                                                              \
  do {                                                                               \
    ++g_checks;                                                                      \
    const double va_ = (a), vb_ = (b);                                               \
    if (!(va_ <= vb_)) {                                                             \
      ++g_failures;                                                                  \
      std::fprintf(stderr, "  FAILED %s:%d: %s = %.6g > %s = %.6g\n", __FILE__,     \
                   __LINE__, #a, va_, #b, vb_);                                      \
    }                                                                                \
  } while (0)

#define EXPECT_THROW(stmt)                                                           \
  do {                                                                               \
    ++g_checks;                                                                      \
    bool thrown_ = false;                                                            \
    try {                                                                            \
      stmt;                                                                          \
    } catch (const std::logic_error&) {                                              \
      thrown_ = true;                                                                \
    }                                                                                \
    if (!thrown_) {                                                                  \
      ++g_failures;                                                                  \
      std::fprintf(stderr, "  FAILED %s:%d: %s did not throw\n", __FILE__, __LINE__, \
                   #stmt);                                                           \
    }                                                                                \
  } while (0)

struct TestCase {
  const char* group;
  const char* name;
  std::function<void()> fn;
};
std::vector<TestCase>& registry() {
  static std::vector<TestCase> r;
  return r;
}
struct Register {
  Register(const char* g, const char* n, std::function<void()> f) {
    registry().push_back({g, n, f});
  }
};
#define TEST(group, name)                                             \
  static void test_##group##_##name();                                \
  static Register reg_##group##_##name(#group, #name, test_##group##_##name); \
  static void test_##group##_##name()

// Normwise relative difference ||a - b|| / max(||b||, 1e-300).
double relErr(const std::vector<double>& a, const std::vector<double>& b) {
  double num = 0.0, den = 0.0;
  for (size_t i = 0; i < a.size(); ++i) {
    num += (a[i] - b[i]) * (a[i] - b[i]);
    den += b[i] * b[i];
  }
  return std::sqrt(num) / std::max(std::sqrt(den), 1e-300);
}
double relErr(double a, double b) { return std::fabs(a - b) / std::max(std::fabs(b), 1e-300); }

// Row-major copy of a (column-major, as Eigen) MatrixXd, the oracle's order.
std::vector<double> rowMajor(const MatrixXd& m) {
  std::vector<double> r;
  for (long i = 0; i < m.rows(); ++i)
    for (long j = 0; j < m.cols(); ++j) r.push_back(m(i, j));
  return r;
}

// Dense oracle vertex form (mask[v*K+k], vals[(v*K+k)*D+d]).
struct Dense {
  int S, D, K;
  std::vector<uint8_t> mask;
  std::vector<double> vals;
};
Dense toDense(const Vertex::Vector& vs, int K) {
  Dense o{static_cast<int>(vs.size()) - 1, vs.front().D(), K, {}, {}};
  o.mask.assign(vs.size() * K, 0);
  o.vals.assign(vs.size() * K * o.D, 0.0);
  for (size_t v = 0; v < vs.size(); ++v)
    for (int k = 0; k < K; ++k) {
      VectorXd val;
      if (vs[v].getConstraint(k, &val)) {
        o.mask[v * K + k] = 1;
        for (int d = 0; d < o.D; ++d) o.vals[(v * K + k) * o.D + d] = val[d];
      }
    }
  return o;
}

std::vector<double> coeffsOf(const Segment::Vector& segs, int N) {
  std::vector<double> c;
  for (const Segment& s : segs)
    for (int d = 0; d < s.D(); ++d) {
      const VectorXd v = s[d].getCoefficients();
      for (int k = 0; k < N; ++k) c.push_back(v[k]);
    }
  return c;
}

// checkPath (test_polynomial_optimization.cpp:113-172).
void checkPath(const Vertex::Vector& vs, const Segment::Vector& segs, int N) {
  const int M = N / 2;
  for (size_t s = 0; s < segs.size(); ++s) {
    for (int end = 0; end < 2; ++end) {
      const Vertex& v = vs[s + end];
      const double t = end ? segs[s].getTime() : 0.0;
      for (int k = 0; k < M; ++k) {
        VectorXd want;
        if (!v.getConstraint(k, &want)) continue;
        const VectorXd got = segs[s].evaluate(t, k);
        for (long d = 0; d < want.size(); ++d)
          EXPECT_LE(std::fabs(got[d] - want[d]), 1e-6 * std::max(1.0, std::fabs(want[d])));
      }
    }
    if (s > 0)
      for (int k = 0; k < M; ++k) {
        const VectorXd a = segs[s - 1].evaluate(segs[s - 1].getTime(), k);
        const VectorXd b = segs[s].evaluate(0.0, k);
        for (long d = 0; d < a.size(); ++d)
          EXPECT_LE(std::fabs(a[d] - b[d]), 1e-6 * std::max(1.0, std::fabs(a[d])));
      }
  }
}

// computeCostNumeric (test_utils.h:56-64) vs computeCost, 10 % (checkCost,
// test_polynomial_optimization.cpp:174-195).
void checkCost(const Segment::Vector& segs, int r, double cost) {
  double num = 0.0;
  const double dt = 1e-3;
  for (const Segment& s : segs)
    for (double t = 0.0; t < s.getTime(); t += dt) {
      const VectorXd v = s.evaluate(t, r);
      num += v.squaredNorm() * dt;
    }
  EXPECT_LE(std::fabs(num - cost), 0.1 * std::fabs(num));
}

// getMaximumMagnitude (test_utils.h:43-54): the sampled maximum of |p^(k)|,
// dt = 0.01.
double getMaximumMagnitude(const Trajectory& trajectory, int derivative, double dt = 0.01) {
  double maximum = -1e9;
  for (double ts = 0; ts < trajectory.getMaxTime(); ts += dt) {
    const double v = trajectory.evaluate(ts, derivative).norm();
    if (v > maximum) maximum = v;
  }
  return maximum;
}

struct Fixture {
  int D, r, S;
  unsigned seed;
  double vmax, amax;
};
// The reference's OptimizationParams instances
// (test_polynomial_optimization.cpp:753-812).
const Fixture kFixtures[] = {
    {1, 4, 1, 100, 3.0, 5.0},  // segment_1_dim_1
    {1, 4, 10, 102, 3.0, 5.0}, // segment_10_dim_1
    {1, 4, 50, 103, 3.0, 5.0}, // segment_50_dim_1
    {3, 4, 1, 104, 3.0, 5.0},  // segment_1_dim_3
    {3, 4, 10, 105, 3.0, 5.0}, // segment_10_dim_3
    {3, 4, 50, 106, 3.0, 5.0}, // segment_50_dim_3
    {3, 4, 75, 106, 3.0, 5.0}, // segment_75_dim_3
    {1, 2, 5, 107, 1.0, 2.0},  // deriv_accel_1
    {3, 2, 1, 108, 1.0, 2.0},  // deriv_accel_3_1
    {3, 2, 5, 109, 1.0, 2.0},  // deriv_accel
    {3, 3, 5, 110, 1.0, 2.0},  // deriv_jerk
};
const Fixture& kSeg10Dim3 = kFixtures[4];

Vertex::Vector fixtureVertices(const Fixture& f, int N) {
  return createRandomVertices(N / 2 - 1, f.S, VectorXd::Constant(f.D, -10.0),
                              VectorXd::Constant(f.D, 10.0), f.seed);
}

// ---------------------------------------------------------------- host tests

TEST(host, AMatrixInversion) {
  // test_polynomial_optimization.cpp:695-705: Schur inverse vs a general
  // dense inverse at 1e-10 (Eigen's partial-pivot LU there and here).
  for (double t = 1; t <= 60; t += 1) {
    PolynomialOptimization<10>::SquareMatrix A, Ai;
    PolynomialOptimization<10>::setupMappingMatrix(t, &A);
    PolynomialOptimization<10>::invertMappingMatrix(A, &Ai);
    const MatrixXd full = internal::smallInverse(A);  // dense 10 x 10 LU inverse
    for (int i = 0; i < 10; ++i)
      for (int j = 0; j < 10; ++j)
        EXPECT_LE(std::fabs(Ai(i, j) - full(i, j)), 1e-10);
  }
}

// MatrixXd stores column-major as Eigen's default MatrixXd does: data()
// lists column 0 first, so Eigen-style .data() copies keep their meaning.
TEST(host, MatrixXdColumnMajor) {
  MatrixXd m(2, 3);
  for (long i = 0; i < 2; ++i)
    for (long j = 0; j < 3; ++j) m(i, j) = 10.0 * i + j;
  const double want[6] = {0, 10, 1, 11, 2, 12};
  for (int k = 0; k < 6; ++k) EXPECT_TRUE(m.data()[k] == want[k]);
  const MatrixXd t = m.transpose();
  EXPECT_TRUE(t.rows() == 3 && t.cols() == 2 && t(2, 1) == 12.0 && t.data()[1] == 1.0);
  // the mapping matrix A(T) (linear_impl:132-150): row 0 is (1, 0, ..., 0)
  // and column 0 is (1, 0, 0, 0, 0, 1, 0, 0, 0, 0) at T = 1, so data()[0..9]
  // is column 0
  PolynomialOptimization<10>::SquareMatrix A;
  PolynomialOptimization<10>::setupMappingMatrix(1.0, &A);
  for (int i = 0; i < 10; ++i) EXPECT_TRUE(A.data()[i] == A(i, 0));
  EXPECT_TRUE(A.data()[5] == 1.0 && A.data()[10] == 0.0);
}

TEST(host, QuadraticCostJacobianMatchesOracle) {
  for (int r = 0; r < 5; ++r)
    for (double t : {0.1, 1.0, 3.7, 12.0}) {
      PolynomialOptimization<10>::SquareMatrix Q;
      PolynomialOptimization<10>::computeQuadraticCostJacobian(r, t, &Q);
      std::vector<double> q(100), got = rowMajor(Q);
      orc_segment_matrices(10, r, t, q.data(), nullptr, nullptr, nullptr);
      EXPECT_LE(relErr(got, q), 1e-14);
    }
}

TEST(host, MappingMatrixMatchesOracle) {
  for (double t : {0.1, 1.0, 3.7, 12.0}) {
    PolynomialOptimization<10>::SquareMatrix A, Ai;
    PolynomialOptimization<10>::setupMappingMatrix(t, &A);
    PolynomialOptimization<10>::invertMappingMatrix(A, &Ai);
    std::vector<double> a(100), ai(100);
    orc_segment_matrices(10, 4, t, nullptr, a.data(), ai.data(), nullptr);
    EXPECT_LE(relErr(rowMajor(A), a), 0.0);
    EXPECT_LE(relErr(rowMajor(Ai), ai), 1e-13);
  }
}

TEST(host, RandomVerticesBitIdentical) {
  for (const Fixture& f : kFixtures) {
    const Vertex::Vector vs = fixtureVertices(f, 10);
    const Dense d = toDense(vs, 5);
    std::vector<double> lo(f.D, -10.0), hi(f.D, 10.0);
    std::vector<uint8_t> mask((f.S + 1) * 5);
    std::vector<double> vals((f.S + 1) * 5 * f.D);
    orc_random_vertices(4, f.S, f.D, lo.data(), hi.data(), f.seed, 5, mask.data(),
                        vals.data());
    EXPECT_TRUE(mask == d.mask);
    EXPECT_TRUE(vals == d.vals);  // bit-identical
  }
}

TEST(host, SolveFailsLoudlyWithoutDevice) {
  // No CPU fallback: the plan cannot be created without a HIP device.  (On a
  // GPU host there is a device, and the gpu group covers the solve.)
  int n_dev = 0;
  if (hipGetDeviceCount(&n_dev) == hipSuccess && n_dev > 0) return;
  const Vertex::Vector vs = fixtureVertices(kSeg10Dim3, 10);
  PolynomialOptimization<10> opt(3);
  EXPECT_THROW(opt.setupFromVertices(vs, estimateSegmentTimes(vs, 3.0, 5.0), 4));
}

TEST(host, ContractChecks) {
  // linear_impl:50-55, 66-67: derivative out of range, size mismatch.
  const Vertex::Vector vs = fixtureVertices(kSeg10Dim3, 10);
  PolynomialOptimization<10> opt(3);
  EXPECT_THROW(opt.setupFromVertices(vs, estimateSegmentTimes(vs, 3.0, 5.0), 5));
  EXPECT_THROW(opt.setupFromVertices(vs, std::vector<double>(2, 1.0), 4));
}

// ----------------------------------------------------------------- gpu tests

TEST(gpu, TwoVerticesSetup) {
  // test_polynomial_optimization.cpp:707-751 (Matlab solution).
  Vertex start(1);
  for (int k = 0; k <= 4; ++k) start.addConstraint(k, 0.0);
  Vertex goal = start;
  goal.addConstraint(derivative_order::POSITION, 5.0);
  PolynomialOptimization<10> opt(1);
  Vertex::Vector vs{start, goal};
  opt.setupFromVertices(vs, {5.0}, derivative_order::SNAP);
  EXPECT_TRUE(opt.solveLinear());
  Segment::Vector segs;
  opt.getSegments(&segs);
  checkPath(vs, segs, 10);
  const double matlab[10] = {-0.000000000000004, 0.000000000000004, -0.000000000000006,
                             0.000000000000003,  -0.000000000000001, 0.201600000000015,
                             -0.134400000000012, 0.034560000000004,  -0.004032000000000,
                             0.000179200000000};
  const VectorXd c = segs[0][0].getCoefficients();
  for (int k = 0; k < 10; ++k) EXPECT_LE(std::fabs(c[k] - matlab[k]), 1e-13);
}

template <int N>
void runFixture(const Fixture& f) {
  const Vertex::Vector vs = fixtureVertices(f, N);
  const std::vector<double> times = estimateSegmentTimes(vs, f.vmax, f.amax);
  PolynomialOptimization<N> opt(f.D);
  opt.setupFromVertices(vs, times, f.r);
  EXPECT_TRUE(opt.solveLinear());
  Segment::Vector segs;
  opt.getSegments(&segs);
  checkPath(vs, segs, N);
  checkCost(segs, f.r, opt.computeCost());

  const Dense d = toDense(vs, N / 2);
  std::vector<double> coeffs(f.S * f.D * N), df(f.D * (f.S + 1) * N / 2), dp(f.D * (f.S + 1) * N / 2);
  double cost = 0.0;
  int nf = 0, np = 0;
  EXPECT_TRUE(orc_linear_solve(N, f.D, f.r, f.S, N / 2, d.mask.data(), d.vals.data(),
                               times.data(), coeffs.data(), &cost, df.data(), dp.data(), &nf,
                               &np) == 0);
  EXPECT_TRUE(static_cast<size_t>(nf) == opt.getNumberFixedConstraints());
  EXPECT_TRUE(static_cast<size_t>(np) == opt.getNumberFreeConstraints());
  EXPECT_LE(relErr(coeffsOf(segs, N), coeffs), 1e-6);
  EXPECT_LE(relErr(opt.computeCost(), cost), 1e-6);
  std::vector<VectorXd> fixed, free_c;
  opt.getFixedConstraints(&fixed);
  opt.getFreeConstraints(&free_c);
  std::vector<double> gf, gp;
  for (int dd = 0; dd < f.D; ++dd) {
    for (long i = 0; i < fixed[dd].size(); ++i) gf.push_back(fixed[dd][i]);
    for (long i = 0; i < free_c[dd].size(); ++i) gp.push_back(free_c[dd][i]);
  }
  df.resize(f.D * nf);
  dp.resize(f.D * np);
  EXPECT_TRUE(gf == df);
  EXPECT_LE(relErr(gp, dp), 1e-6);
}

TEST(gpu, ReferenceFixturesN10) {
  for (const Fixture& f : kFixtures) runFixture<10>(f);
}

// test_polynomial_optimization.cpp:270-305 (UnconstrainedLinearEstimateSegmentTimes)
// on every OptimizationParams instance: with estimateSegmentTimes' times the
// solution's sampled maximum speed and acceleration stay below 2.5 times the
// limits the times were estimated for, and checkPath / checkCost hold.
TEST(gpu, UnconstrainedLinearEstimateSegmentTimes) {
  for (const Fixture& f : kFixtures) {
    const Vertex::Vector vs = fixtureVertices(f, 10);
    const std::vector<double> times = estimateSegmentTimes(vs, f.vmax, f.amax);
    PolynomialOptimization<10> opt(f.D);
    opt.setupFromVertices(vs, times, f.r);
    EXPECT_TRUE(opt.solveLinear());
    Segment::Vector segs;
    opt.getSegments(&segs);
    Trajectory traj;
    opt.getTrajectory(&traj);
    checkPath(vs, segs, 10);
    const double v_max_traj = getMaximumMagnitude(traj, derivative_order::VELOCITY);
    const double a_max_traj = getMaximumMagnitude(traj, derivative_order::ACCELERATION);
    EXPECT_LE(v_max_traj, f.vmax * 2.5);
    EXPECT_LE(a_max_traj, f.amax * 2.5);
    EXPECT_TRUE(v_max_traj < f.vmax * 2.5 && a_max_traj < f.amax * 2.5);  // EXPECT_LT
    checkCost(segs, f.r, opt.computeCost());
  }
}

TEST(gpu, OtherOrders) {
  for (const Fixture& f : kFixtures) {
    Fixture g = f;
    g.r = std::min(f.r, 2);
    runFixture<6>(g);
    g.r = std::min(f.r, 3);
    runFixture<8>(g);
  }
}

TEST(gpu, ConstraintPacking) {
  // test_polynomial_optimization.cpp:510-570: feeding the solved free
  // constraints back reproduces the segments; moving them off the optimum
  // raises the cost.
  const Fixture f = kSeg10Dim3;
  const Vertex::Vector vs = fixtureVertices(f, 10);
  PolynomialOptimization<10> opt(f.D);
  opt.setupFromVertices(vs, estimateSegmentTimes(vs, f.vmax, f.amax), f.r);
  opt.solveLinear();
  Segment::Vector s0, s1;
  opt.getSegments(&s0);
  const double c0 = opt.computeCost();
  std::vector<VectorXd> fc;
  opt.getFreeConstraints(&fc);
  opt.setFreeConstraints(fc);
  opt.getSegments(&s1);
  EXPECT_LE(relErr(coeffsOf(s1, 10), coeffsOf(s0, 10)), 1e-12);
  // The solve (standard-pattern kernel) and the recovery (generic
  // formulation) sum the cancelling quadratic form in different orders.
  EXPECT_LE(relErr(opt.computeCost(), c0), 1e-9);
  fc[1][3] += 0.5;
  opt.setFreeConstraints(fc);
  EXPECT_TRUE(opt.computeCost() > c0);
  Segment::Vector s2;
  opt.getSegments(&s2);
  checkPath(vs, s2, 10);  // still meets the fixed constraints and continuity
}

TEST(gpu, AccessorsMatchOracle) {
  const Fixture f = kSeg10Dim3;
  const Vertex::Vector vs = fixtureVertices(f, 10);
  const std::vector<double> times = estimateSegmentTimes(vs, f.vmax, f.amax);
  PolynomialOptimization<10> opt(f.D);
  opt.setupFromVertices(vs, times, f.r);
  const Dense d = toDense(vs, 5);
  const size_t n = opt.getNumberFixedConstraints() + opt.getNumberFreeConstraints();
  const size_t na = opt.getNumberAllConstraints(), nc = 10 * f.S;
  std::vector<double> R(n * n), M(na * n), A(nc * nc), Ai(nc * nc), Mp(n * na);
  EXPECT_TRUE(orc_linear_matrices(10, f.D, f.r, f.S, 5, d.mask.data(), d.vals.data(),
                                  times.data(), R.data(), M.data(), A.data(), Ai.data(),
                                  Mp.data()) == 0);
  MatrixXd gR, gM, gA, gAi, gMp;
  opt.getR(&gR);
  opt.getM(&gM);
  opt.getA(&gA);
  opt.getAInverse(&gAi);
  opt.getMpinv(&gMp);
  EXPECT_LE(relErr(rowMajor(gR), R), 1e-9);
  EXPECT_TRUE(rowMajor(gM) == M);
  EXPECT_LE(relErr(rowMajor(gA), A), 1e-15);
  EXPECT_LE(relErr(rowMajor(gAi), Ai), 1e-12);
  EXPECT_TRUE(rowMajor(gMp) == Mp);
  // data() lists the entries column by column, as Eigen's getM().data() does
  bool col_major = true;
  for (size_t i = 0; i < na; ++i)
    for (size_t j = 0; j < n; ++j) col_major = col_major && gM.data()[j * na + i] == M[i * n + j];
  for (size_t i = 0; i < nc; ++i)
    for (size_t j = 0; j < nc; ++j) col_major = col_major && gA.data()[j * nc + i] == gA(i, j);
  EXPECT_TRUE(col_major);
}

TEST(gpu, StaleCostAfterTimeUpdate) {
  // computeCost after updateSegmentTimes without a re-solve uses the new Q
  // with the old coefficients (linear_impl:113-130, 277-304).
  const Fixture f = kSeg10Dim3;
  const Vertex::Vector vs = fixtureVertices(f, 10);
  std::vector<double> times = estimateSegmentTimes(vs, f.vmax, f.amax);
  PolynomialOptimization<10> opt(f.D);
  opt.setupFromVertices(vs, times, f.r);
  opt.solveLinear();
  Segment::Vector segs;
  opt.getSegments(&segs);
  for (double& t : times) t *= 1.3;
  opt.updateSegmentTimes(times);
  double want = 0.0;
  for (int s = 0; s < f.S; ++s) {
    std::vector<double> Q(100);
    orc_segment_matrices(10, f.r, times[s], Q.data(), nullptr, nullptr, nullptr);
    for (int dd = 0; dd < f.D; ++dd) {
      const VectorXd c = segs[s][dd].getCoefficients();
      for (int i = 0; i < 10; ++i)
        for (int j = 0; j < 10; ++j) want += c[i] * Q[i * 10 + j] * c[j];
    }
  }
  EXPECT_LE(relErr(opt.computeCost(), 0.5 * want), 1e-12);
  opt.solveLinear();  // re-solve at the new times lowers the cost
  EXPECT_TRUE(opt.computeCost() <= 0.5 * want * (1 + 1e-12));
}

TEST(gpu, FullyConstrained) {
  Vertex::Vector vs = fixtureVertices(kSeg10Dim3, 10);
  for (Vertex& v : vs)
    for (int k = 1; k <= 4; ++k)
      if (!v.hasConstraint(k)) v.addConstraint(k, 0.25 * k);
  PolynomialOptimization<10> opt(3);
  const std::vector<double> times = estimateSegmentTimes(vs, 3.0, 5.0);
  opt.setupFromVertices(vs, times, 4);
  EXPECT_TRUE(opt.getNumberFreeConstraints() == 0);
  EXPECT_TRUE(opt.solveLinear());
  Segment::Vector segs;
  opt.getSegments(&segs);
  checkPath(vs, segs, 10);
  const Dense d = toDense(vs, 5);
  const int S = kSeg10Dim3.S;
  std::vector<double> coeffs(S * 3 * 10);
  double cost = 0.0;
  orc_linear_solve(10, 3, 4, S, 5, d.mask.data(), d.vals.data(), times.data(), coeffs.data(),
                   &cost, nullptr, nullptr, nullptr, nullptr);
  EXPECT_LE(relErr(coeffsOf(segs, 10), coeffs), 1e-9);
  EXPECT_LE(relErr(opt.computeCost(), cost), 1e-9);
}

// src/main.cpp:26-75 geometry (4 segments, radii 0.15).
Vertex::Vector mainCppVertices() {
  const double pts[5][3] = {{2.7, 9.5, 4.8},
                            {3.50796, 4.34802, 4.56653},
                            {3.95552, 3.23008, 4.75131},
                            {5.06673, 2.31032, 4.79433},
                            {7.0, 2.2, 4.8}};
  Vertex::Vector vs;
  for (int v = 0; v < 5; ++v) {
    Vertex x(3);
    VectorXd p{pts[v][0], pts[v][1], pts[v][2]};
    if (v == 0 || v == 4)
      x.makeStartOrEnd(p, 4);
    else
      x.addConstraint(derivative_order::POSITION, p);
    vs.push_back(x);
  }
  return vs;
}

TEST(gpu, TubeQCQPMainFixture) {
  const Vertex::Vector vs = mainCppVertices();
  const std::vector<double> times = estimateSegmentTimes(vs, 2.0, 2.0);
  const std::vector<std::pair<double, double>> radii(4, {0.15, 0.15});
  PolynomialOptimizationConstrained<10> opt(3);
  opt.setupFromVertices(vs, times, radii, 4);
  EXPECT_TRUE(opt.getNumberFixedConstraints() == 10);
  EXPECT_TRUE(opt.getNumberFreeConstraints() == 15);
  EXPECT_TRUE(opt.solveQCQP() == 0);
  const Dense d = toDense(vs, 5);
  std::vector<double> rad(8, 0.15), x(45), coeffs(4 * 3 * 10);
  double cost = 0.0;
  int iters = 0;
  EXPECT_TRUE(orc_tube_qcqp_solve(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(), times.data(),
                                  times.data(), rad.data(), 1e-10, 100, x.data(),
                                  coeffs.data(), &cost, &iters) == 0);
  Segment::Vector segs;
  opt.getSegments(&segs);
  EXPECT_LE(relErr(coeffsOf(segs, 10), coeffs), 1e-6);
  EXPECT_LE(relErr(opt.computeCost(), cost), 1e-6);
  std::vector<VectorXd> fc;
  opt.getFreeConstraints(&fc);
  std::vector<double> gx;
  for (const VectorXd& v : fc)
    for (long i = 0; i < v.size(); ++i) gx.push_back(v[i]);
  EXPECT_LE(relErr(gx, x), 1e-6);
  const std::vector<double> res = opt.getConstraintResiduals();
  EXPECT_TRUE(static_cast<int>(res.size()) == orc_tube_num_constraints(10, 4));
  double worst = -1e300;
  for (double r : res) worst = std::max(worst, r);
  EXPECT_LE(worst, 1e-8);
  // Start/end constraints and continuity hold; intermediate positions are
  // free (they define the tube only).
  Vertex::Vector ends{vs.front(), vs.back()};
  EXPECT_LE(segs.front().evaluate(0.0, 0)[0] - 2.7, 1e-9);
  // The unconstrained tube-pattern solve is no costlier than the QCQP.
  const double qcqp_cost = opt.computeCost();
  opt.solveLinear();
  EXPECT_LE(opt.computeCost(), qcqp_cost * (1 + 1e-9));
}

TEST(gpu, TimeCostMatchesOracle) {
  const Fixture f = kSeg10Dim3;
  const Vertex::Vector vs = fixtureVertices(f, 10);
  const std::vector<double> times = estimateSegmentTimes(vs, f.vmax, f.amax);
  NonlinearOptimizationParameters p;
  p.objective = NonlinearOptimizationParameters::kOptimizeTime;
  p.solve_time_with_qcqp = false;  // the upstream linear inner solve
  p.weights.w_c = 0.0;
  PolynomialOptimizationNonLinear<10> opt(f.D, p);
  opt.setupFromVertices(vs, times, std::vector<std::pair<double, double>>(f.S, {0.15, 0.15}),
                        f.r);
  const Dense d = toDense(vs, 5);
  for (int mode = 0; mode <= 2; ++mode) {
    std::vector<double> g, og(f.S);
    const double J = opt.evaluateTimeCost(times, mode, mode ? &g : nullptr);
    double oJ = 0.0;
    EXPECT_TRUE(orc_time_cost(10, f.D, f.r, f.S, 5, d.mask.data(), d.vals.data(), times.data(),
                              p.time_penalty, mode, p.increment_time, p.weights.w_d,
                              p.weights.w_t, &oJ, og.data()) == 0);
    EXPECT_LE(relErr(J, oJ), 1e-9);
    if (mode) EXPECT_LE(relErr(g, og), 1e-5);
  }
}

TEST(gpu, OptimizeTimeLowersObjective) {
  const Fixture f = kSeg10Dim3;
  const Vertex::Vector vs = fixtureVertices(f, 10);
  const std::vector<double> t0 = estimateSegmentTimes(vs, f.vmax, f.amax);
  NonlinearOptimizationParameters p;
  p.objective = NonlinearOptimizationParameters::kOptimizeTime;
  p.solve_time_with_qcqp = false;  // the upstream linear inner solve
  p.weights.w_c = 0.0;
  p.max_iterations = 50;
  PolynomialOptimizationNonLinear<10> opt(f.D, p);
  opt.setupFromVertices(vs, t0, std::vector<std::pair<double, double>>(f.S, {0.15, 0.15}), f.r);
  const double J0 = opt.evaluateTimeCost(t0);
  EXPECT_TRUE(opt.optimize() > 0);
  std::vector<double> t1;
  opt.getPolynomialOptimizationRef().getSegmentTimes(&t1);
  const OptimizationInfo info = opt.getOptimizationInfo();
  EXPECT_TRUE(info.n_iterations <= 50 && info.n_iterations >= 1);
  const double J1 = opt.evaluateTimeCost(t1);
  EXPECT_LE(J1, J0);
  EXPECT_LE(relErr(J1, info.cost_trajectory + info.cost_time), 1e-9);
  for (size_t i = 0; i < t1.size(); ++i) {
    EXPECT_TRUE(t1[i] >= 0.1 - 1e-15);
    EXPECT_TRUE(t1[i] <= 2.0 * t0[i] + 1e-12);
  }
  Trajectory traj;
  opt.getTrajectory(&traj);
  Segment::Vector segs;
  traj.getSegments(&segs);
  checkPath(vs, segs, 10);
}

// The fork's callback form (solveQCQP inside objectiveFunctionTime,
// nonlinear_impl:892): J and its central-difference gradient match the
// oracle; the optimiser lowers J and ends with the QCQP trajectory.
TEST(gpu, TimeCostWithQCQPInnerSolve) {
  const Vertex::Vector vs = mainCppVertices();
  const std::vector<double> t0 = estimateSegmentTimes(vs, 2.0, 2.0);
  const std::vector<std::pair<double, double>> radii(4, {0.15, 0.15});
  NonlinearOptimizationParameters p;
  p.objective = NonlinearOptimizationParameters::kOptimizeTime;
  p.weights.w_c = 0.0;
  p.solve_time_with_qcqp = true;
  p.max_iterations = 8;
  PolynomialOptimizationNonLinear<10> opt(3, p);
  opt.setupFromVertices(vs, t0, radii, 4);
  const Dense d = toDense(vs, 5);
  std::vector<double> t = t0, rad(8, 0.15);
  for (double& v : t) v *= 1.05;
  std::vector<double> g, og(4);
  const double J = opt.evaluateTimeCost(t, 2, &g);
  double oJ = 0.0;
  EXPECT_TRUE(orc_tube_time_cost(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(), t0.data(),
                                 t.data(), rad.data(), 1e-10, 100, p.time_penalty, 2,
                                 p.increment_time, 0, nullptr, nullptr, 100.0, 1e12, &oJ,
                                 og.data()) == 0);
  EXPECT_LE(std::fabs(J - oJ), 1e-5 * 30.0);  // 1e-6 of the QCQP cost (~26), penalty exact
  for (int n = 0; n < 4; ++n) EXPECT_LE(std::fabs(g[n] - og[n]), 1e-5 * 30.0 / 0.1);
  // J at the control-point times themselves, against the oracle.
  std::vector<double> g0;
  const double J0 = opt.evaluateTimeCost(t0);
  const double J0g = opt.evaluateTimeCost(t0, 2, &g0);
  double oJ0 = 0.0;
  EXPECT_TRUE(orc_tube_time_cost(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(), t0.data(),
                                 t0.data(), rad.data(), 1e-10, 100, p.time_penalty, 0,
                                 p.increment_time, 0, nullptr, nullptr, 100.0, 1e12, &oJ0,
                                 nullptr) == 0);
  std::fprintf(stderr, "J0 %.17g J0(grad) %.17g oracle %.17g J(1.05 T) %.17g oracle %.17g\n",
               J0, J0g, oJ0, J, oJ);
  EXPECT_LE(std::fabs(J0 - oJ0), 1e-5 * 30.0);
  EXPECT_LE(std::fabs(J0g - oJ0), 1e-5 * 30.0);
  EXPECT_TRUE(opt.optimize() > 0);
  const OptimizationInfo info = opt.getOptimizationInfo();
  std::fprintf(stderr, "after optimize: evals %d cost_trajectory %.17g cost_time %.17g\n",
               static_cast<int>(info.n_iterations), info.cost_trajectory, info.cost_time);
  EXPECT_TRUE(info.n_iterations >= 1 && info.n_iterations <= 8);
  EXPECT_LE(info.cost_trajectory + info.cost_time, J0 * (1 + 1e-9));
  Trajectory traj;
  opt.getTrajectory(&traj);
  Segment::Vector segs;
  traj.getSegments(&segs);
  EXPECT_TRUE(segs.size() == 4);
  EXPECT_LE(std::fabs(segs.front().evaluate(0.0, 0)[0] - 2.7), 1e-9);
}

// The reference's own kOptimizeTime path with its defaults: LN_SBPLX over
// objectiveFunctionTime with solveQCQP() at every evaluation
// (nonlinear_impl:332-397, 877-945).  The shim's result (evaluations,
// nlopt_result, optimised times, cost) follows the oracle's Subplex over its
// own interior-point QCQP (orc_tube_time_optimize_sbplx).
TEST(gpu, OptimizeTimeQCQPSbplxMatchesOracle) {
  const Vertex::Vector vs = mainCppVertices();
  const std::vector<double> t0 = estimateSegmentTimes(vs, 2.0, 2.0);
  const std::vector<std::pair<double, double>> radii(4, {0.15, 0.15});
  NonlinearOptimizationParameters p;
  p.objective = NonlinearOptimizationParameters::kOptimizeTime;
  p.weights.w_c = 0.0;
  p.solve_time_with_qcqp = true;
  p.max_iterations = 40;
  EXPECT_TRUE(p.algorithm == nlopt::LN_SBPLX);
  PolynomialOptimizationNonLinear<10> opt(3, p);
  opt.setupFromVertices(vs, t0, radii, 4);
  const int res = opt.optimize();
  const OptimizationInfo info = opt.getOptimizationInfo();
  Trajectory traj;
  opt.getTrajectory(&traj);
  const std::vector<double> t1 = traj.getSegmentTimes();
  const Dense d = toDense(vs, 5);
  std::vector<double> ot = t0, rad(8, 0.15);
  double oc = 0.0;
  int oev = 0, ores = 0;
  EXPECT_TRUE(orc_tube_time_optimize_sbplx(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(),
                                           rad.data(), ot.data(), 1e-10, 100, p.time_penalty,
                                           40, p.f_rel, p.f_abs, p.initial_stepsize_rel, 0,
                                           nullptr, nullptr, 100.0, 1e12, &oc, &oev, &ores,
                                           nullptr) == 0);
  std::fprintf(stderr, "QCQP LN_SBPLX: result %d (oracle %d), evals %d (oracle %d)\n", res,
               ores, static_cast<int>(info.n_iterations), oev);
  EXPECT_TRUE(res == ores);
  EXPECT_TRUE(info.n_iterations == oev);
  EXPECT_LE(relErr(t1, ot), 1e-6);
  EXPECT_LE(relErr(info.cost_trajectory + info.cost_time, oc), 1e-6);
}

// kOptimizeTime with the default LN_SBPLX on more than 16 segments (the
// machine's state is sized by the segment count): the objective does not
// rise and the bounds hold.
TEST(gpu, OptimizeTimeSbplxManySegments) {
  const Fixture f{3, 4, 24, 111, 3.0, 5.0};
  const Vertex::Vector vs = fixtureVertices(f, 10);
  const std::vector<double> t0 = estimateSegmentTimes(vs, f.vmax, f.amax);
  NonlinearOptimizationParameters p;
  p.objective = NonlinearOptimizationParameters::kOptimizeTime;
  p.solve_time_with_qcqp = false;  // the upstream linear inner solve
  p.weights.w_c = 0.0;
  p.max_iterations = 60;
  PolynomialOptimizationNonLinear<10> opt(f.D, p);
  opt.setupFromVertices(vs, t0, std::vector<std::pair<double, double>>(f.S, {0.15, 0.15}), f.r);
  const double J0 = opt.evaluateTimeCost(t0);
  const int res = opt.optimize();
  EXPECT_TRUE(res == nlopt::MAXEVAL_REACHED || res == nlopt::FTOL_REACHED ||
              res == nlopt::XTOL_REACHED);
  std::vector<double> t1;
  opt.getPolynomialOptimizationRef().getSegmentTimes(&t1);
  const OptimizationInfo info = opt.getOptimizationInfo();
  EXPECT_TRUE(info.n_iterations >= 1 && info.n_iterations <= 60);
  EXPECT_LE(opt.evaluateTimeCost(t1), J0);
  for (size_t i = 0; i < t1.size(); ++i) {
    EXPECT_TRUE(t1[i] >= 0.1 - 1e-15);
    EXPECT_TRUE(t1[i] <= 2.0 * t0[i] + 1e-12);
  }
  const Dense d = toDense(vs, 5);
  std::vector<double> ot = t0;
  double oc = 0.0;
  int oev = 0, ores = 0;
  EXPECT_TRUE(orc_time_optimize_sbplx(10, f.D, f.r, f.S, 5, d.mask.data(), d.vals.data(),
                                      ot.data(), p.time_penalty, 60, p.f_rel, p.f_abs,
                                      p.initial_stepsize_rel, 0, nullptr, nullptr, 100.0, 1e12,
                                      &oc, &oev, &ores, nullptr) == 0);
  EXPECT_TRUE(res == ores && info.n_iterations == oev);
  EXPECT_LE(relErr(t1, ot), 1e-6);
}

// Extrema test of the reference (test_polynomial_optimization.cpp:370-400):
// the analytic maximum of |v| and |a| agrees with dense sampling within 0.01
// (getMaximumMagnitude, test_utils.h) and with the oracle's
// computeMaximumOfMagnitude restatement.
TEST(gpu, MaximumOfMagnitude) {
  for (const Fixture& f : kFixtures) {
    const Vertex::Vector vs = fixtureVertices(f, 10);
    const std::vector<double> times = estimateSegmentTimes(vs, f.vmax, f.amax);
    PolynomialOptimization<10> opt(f.D);
    opt.setupFromVertices(vs, times, f.r);
    EXPECT_TRUE(opt.solveLinear());
    Segment::Vector segs;
    opt.getSegments(&segs);
    const std::vector<double> c = coeffsOf(segs, 10);
    for (int k = derivative_order::VELOCITY; k <= derivative_order::ACCELERATION; ++k) {
      const Extremum e = k == derivative_order::VELOCITY
                             ? opt.computeMaximumOfMagnitude<derivative_order::VELOCITY>(nullptr)
                             : opt.computeMaximumOfMagnitude(k, nullptr);
      double ot = 0.0, ov = 0.0;
      int os = 0;
      EXPECT_TRUE(orc_max_magnitude(10, f.D, f.S, c.data(), times.data(), k, &ot, &ov, &os,
                                    nullptr) == 0);
      EXPECT_LE(relErr(e.value, ov), 1e-10);
      double sampled = 0.0;  // getMaximumMagnitude: dt = 0.01
      for (const Segment& s : segs)
        for (double t = 0.0; t < s.getTime(); t += 0.01) {
          const VectorXd v = s.evaluate(t, k);
          double n2 = 0.0;
          for (int d = 0; d < f.D; ++d) n2 += v[d] * v[d];
          sampled = std::max(sampled, std::sqrt(n2));
        }
      EXPECT_LE(std::fabs(sampled - e.value), 0.01);
      EXPECT_TRUE(e.value >= sampled - 1e-12);
      // The reported time lies in its segment and attains the value.
      EXPECT_TRUE(e.segment_idx >= 0 && e.segment_idx < f.S);
      const VectorXd v = segs[e.segment_idx].evaluate(e.time, k);
      double n2 = 0.0;
      for (int d = 0; d < f.D; ++d) n2 += v[d] * v[d];
      EXPECT_LE(relErr(std::sqrt(n2), e.value), 1e-12);
    }
  }
}

// ExtremaOfMagnitude (test/test_polynomial_optimization.cpp:307-406) through
// the same names: per segment the analytic candidates
// (computeSegmentMaximumMagnitudeCandidates) contain every candidate the
// sampling helper finds (checkExtrema, 0.01), the sampled candidates are
// stationary points (|p^(k+1)| < 0.01), and computeMaximumOfMagnitude /
// Trajectory::computeMinMaxMagnitude agree with getMaximumMagnitude's dense
// sampling within 0.01.  Also: the optional candidate list of
// computeMaximumOfMagnitude (device lists) against the host Segment lists.
TEST(gpu, ExtremaOfMagnitude) {
  constexpr int kDerivative = derivative_order::VELOCITY;
  for (const Fixture& f : kFixtures) {
    if (f.S > 10) continue;  // the 50/75-segment fixtures: same code, 10x the sampling time
    const Vertex::Vector vs = fixtureVertices(f, 10);
    const std::vector<double> times = estimateSegmentTimes(vs, f.vmax, f.amax);
    PolynomialOptimization<10> opt(f.D);
    opt.setupFromVertices(vs, times, f.r);
    EXPECT_TRUE(opt.solveLinear());
    Segment::Vector segments;
    opt.getSegments(&segments);
    Trajectory trajectory;
    opt.getTrajectory(&trajectory);
    std::vector<int> dimensions;
    for (int i = 0; i < f.D; ++i) dimensions.push_back(i);
    for (const Segment& s : segments) {
      std::vector<double> res, res_sampling;
      EXPECT_TRUE(PolynomialOptimization<10>::computeSegmentMaximumMagnitudeCandidates(
          kDerivative, s, 0, s.getTime(), &res));
      std::vector<double> res_t;
      EXPECT_TRUE(PolynomialOptimization<10>::computeSegmentMaximumMagnitudeCandidates<
                  kDerivative>(s, 0, s.getTime(), &res_t));
      EXPECT_TRUE(res_t == res);
      PolynomialOptimization<10>::computeSegmentMaximumMagnitudeCandidatesBySampling<kDerivative>(
          s, 0, s.getTime(), 0.01, &res_sampling);
      for (double c : res_sampling) EXPECT_LE(s.evaluate(c, kDerivative + 1).norm(), 0.01);
      // checkExtrema(res_sampling, res, 0.01) (:225-245).  A sampled
      // "extremum" where |v| itself is rounding noise (a rest vertex, e.g.
      // deriv_jerk's last segment ends at |v| ~ 3e-12) is a flip of the
      // noise's sign, not a stationary point: skipped.
      for (double t : res_sampling) {
        if (s.evaluate(t, kDerivative).norm() < 1e-9) continue;
        bool found = false;
        for (double r : res) found = found || std::fabs(t - r) < 0.01;
        EXPECT_TRUE(found);
      }
    }
    double v_max_ref = -1e9, a_max_ref = -1e9;  // getMaximumMagnitude (test_utils.h:43-54)
    for (double ts = 0; ts < trajectory.getMaxTime(); ts += 0.01) {
      v_max_ref = std::max(v_max_ref, trajectory.evaluate(ts, derivative_order::VELOCITY).norm());
      a_max_ref =
          std::max(a_max_ref, trajectory.evaluate(ts, derivative_order::ACCELERATION).norm());
    }
    const Extremum v_max_opt = opt.computeMaximumOfMagnitude<derivative_order::VELOCITY>(nullptr);
    const Extremum a_max_opt =
        opt.computeMaximumOfMagnitude<derivative_order::ACCELERATION>(nullptr);
    Extremum v_min_traj, v_max_traj, a_min_traj, a_max_traj;
    EXPECT_TRUE(trajectory.computeMinMaxMagnitude(derivative_order::VELOCITY, dimensions,
                                                  &v_min_traj, &v_max_traj));
    EXPECT_TRUE(trajectory.computeMinMaxMagnitude(derivative_order::ACCELERATION, dimensions,
                                                  &a_min_traj, &a_max_traj));
    EXPECT_LE(std::fabs(v_max_ref - v_max_opt.value), 0.01);
    EXPECT_LE(std::fabs(a_max_ref - a_max_opt.value), 0.01);
    EXPECT_LE(std::fabs(v_max_ref - v_max_traj.value), 0.01);
    EXPECT_LE(std::fabs(a_max_ref - a_max_traj.value), 0.01);

    // The candidate list: same maximum, segment order, every entry inside
    // its segment and attaining its value, endpoints first, and each host
    // Segment candidate time of a simple root matched by a device one.
    std::vector<Extremum> cand;
    const Extremum v_list = opt.computeMaximumOfMagnitude(derivative_order::VELOCITY, &cand);
    EXPECT_TRUE(v_list.value == v_max_opt.value || std::fabs(v_list.value - v_max_opt.value) <=
                                                       1e-12 * v_max_opt.value);
    EXPECT_TRUE(!cand.empty() && cand.back().segment_idx == f.S - 1);
    size_t i = 0;
    for (int sidx = 0; sidx < f.S; ++sidx) {
      const Segment& s = segments[sidx];
      EXPECT_TRUE(i + 1 < cand.size() && cand[i].time == 0.0 && cand[i + 1].time == s.getTime());
      std::vector<Extremum> host;
      EXPECT_TRUE(s.computeMinMaxMagnitudeCandidates(derivative_order::VELOCITY, 0.0, s.getTime(),
                                                     dimensions, &host));
      size_t j = i;
      while (j < cand.size() - 1 && cand[j].segment_idx == sidx) {
        const double v = s.evaluate(cand[j].time, derivative_order::VELOCITY).norm();
        EXPECT_LE(std::fabs(v - cand[j].value), 1e-9 * v + 1e-12);
        EXPECT_TRUE(cand[j].time >= 0.0 && cand[j].time <= s.getTime());
        ++j;
      }
      // The searched polynomial in the monomial basis: f = sum_d v_d a_d
      // (segment.cpp:97-114), or a alone for D = 1 (:123-129).  Near a rest
      // vertex it vanishes to high order and its values fall below the
      // rounding of its coefficients (scale = sum |f_i| T^i): both searches
      // then report roots of that noise, not necessarily the same ones.  Only
      // simple roots, |f'| T > 1e-6 scale, are compared.
      VectorXd fc;
      if (f.D > 1) {
        fc = VectorXd(Polynomial::getConvolutionLength(9, 8));
        for (int d = 0; d < f.D; ++d)
          fc += Polynomial::convolve(s[d].getCoefficients(1).head(9),
                                     s[d].getCoefficients(2).head(8));
      } else {
        fc = s[0].getCoefficients(2).head(8);
      }
      const Polynomial fp(fc);
      double fscale = 0.0;
      for (long q = 0; q < fc.size(); ++q) fscale += std::fabs(fc[q]) * std::pow(s.getTime(), q);
      for (size_t h = 2; h < host.size(); ++h) {
        const double t = host[h].time;
        if (t < 1e-6 * s.getTime() || t > s.getTime() * (1 - 1e-6)) continue;
        if (std::fabs(fp.evaluate(t, 1)) * s.getTime() <= 1e-6 * fscale) continue;
        bool found = false;
        for (size_t k = i + 2; k < j; ++k) found = found || std::fabs(cand[k].time - t) <= 1e-7 * s.getTime();
        if (!found) {
          std::fprintf(stderr, "  host root %.17g (T %.17g, D %d, S %d, seg %d, |v| %g |a| %g) device:",
                       t, s.getTime(), f.D, f.S, sidx, s.evaluate(t, 1).norm(), s.evaluate(t, 2).norm());
          for (size_t k = i; k < j; ++k) std::fprintf(stderr, " %.17g", cand[k].time);
          std::fprintf(stderr, "\n");
        }
        EXPECT_TRUE(found);
      }
      // selectMinMaxMagnitudeFromCandidates over the host list: the maximum
      // is the largest candidate of the segment
      Extremum mn, mx;
      EXPECT_TRUE(s.selectMinMaxMagnitudeFromCandidates(derivative_order::VELOCITY, 0.0,
                                                        s.getTime(), dimensions, host, &mn, &mx));
      double hmax = 0.0, hmin = 1e300;
      for (const Extremum& e : host) {
        hmax = std::max(hmax, e.value);
        hmin = std::min(hmin, e.value);
      }
      EXPECT_TRUE(mx.value == hmax && mn.value == hmin);
      i = j;
    }
    EXPECT_TRUE(i == cand.size() - 1);
  }
}

// Soft magnitude constraints on the callback (addMaximumMagnitudeConstraint
// + use_soft_constraints, nonlinear_impl:847-875, 907-913, 2735-2766).
TEST(gpu, SoftConstraintTimeCost) {
  const Fixture f = kSeg10Dim3;
  const Vertex::Vector vs = fixtureVertices(f, 10);
  const std::vector<double> times = estimateSegmentTimes(vs, f.vmax, f.amax);
  NonlinearOptimizationParameters p;
  p.objective = NonlinearOptimizationParameters::kOptimizeTime;
  p.solve_time_with_qcqp = false;  // the upstream linear inner solve
  p.weights.w_c = 0.0;
  p.max_iterations = 30;
  PolynomialOptimizationNonLinear<10> opt(f.D, p);
  opt.setupFromVertices(vs, times, std::vector<std::pair<double, double>>(f.S, {0.15, 0.15}),
                        f.r);
  EXPECT_TRUE(opt.addMaximumMagnitudeConstraint(derivative_order::VELOCITY, 3.2));
  EXPECT_TRUE(opt.addMaximumMagnitudeConstraint(derivative_order::ACCELERATION, 1.4));
  const Dense d = toDense(vs, 5);
  const int ders[2] = {1, 2};
  const double lims[2] = {3.2, 1.4};
  for (int mode = 0; mode <= 2; mode += 2) {
    std::vector<double> g, og(f.S);
    const double J = opt.evaluateTimeCost(times, mode, mode ? &g : nullptr);
    double oJ = 0.0;
    EXPECT_TRUE(orc_time_cost_soft(10, f.D, f.r, f.S, 5, d.mask.data(), d.vals.data(),
                                   times.data(), p.time_penalty, mode, p.increment_time,
                                   p.weights.w_d, p.weights.w_t, 2, ders, lims,
                                   p.soft_constraint_weight, 1.0e12, &oJ, og.data()) == 0);
    EXPECT_LE(relErr(J, oJ), 1e-9);
    if (mode) EXPECT_LE(relErr(g, og), 1e-5);
  }
  // The optimiser sees the soft cost: the result's objective (with soft
  // terms) is no larger than the start's, and the info splits it.
  const double J0 = opt.evaluateTimeCost(times);
  EXPECT_TRUE(opt.optimize() > 0);
  std::vector<double> t1;
  opt.getPolynomialOptimizationRef().getSegmentTimes(&t1);
  const double J1 = opt.evaluateTimeCost(t1);
  EXPECT_LE(J1, J0);
  const OptimizationInfo info = opt.getOptimizationInfo();
  EXPECT_LE(relErr(J1, info.cost_trajectory + info.cost_time + info.cost_soft_constraints),
            1e-9);
  EXPECT_TRUE(info.maxima.count(derivative_order::VELOCITY) == 1);
  // Hard constraints (use_soft_constraints = false, nonlinear_impl:861-872):
  // the objective has no soft term, a feasible start stays feasible.
  NonlinearOptimizationParameters hard = p;
  hard.use_soft_constraints = false;
  {
    // With the default LN_SBPLX the inequality is refused, as NLopt's
    // add_inequality_constraint throws (nonlinear_impl:862-872).
    PolynomialOptimizationNonLinear<10> sbplx(f.D, hard);
    sbplx.setupFromVertices(vs, times,
                            std::vector<std::pair<double, double>>(f.S, {0.15, 0.15}), 4);
    EXPECT_TRUE(!sbplx.addMaximumMagnitudeConstraint(derivative_order::VELOCITY, 1.0));
  }
  hard.algorithm = nlopt::LN_COBYLA;  // takes inequality constraints
  PolynomialOptimizationNonLinear<10> opt2(f.D, hard);
  opt2.setupFromVertices(vs, times, std::vector<std::pair<double, double>>(f.S, {0.15, 0.15}),
                         4);
  opt2.solveLinear();
  const double vmax0 =
      opt2.getPolynomialOptimizationRef().computeMaximumOfMagnitude(1, nullptr).value;
  EXPECT_TRUE(opt2.addMaximumMagnitudeConstraint(derivative_order::VELOCITY, 1.01 * vmax0));
  double Jplain = 0.0;
  EXPECT_TRUE(orc_time_cost(10, f.D, f.r, f.S, 5, d.mask.data(), d.vals.data(), times.data(),
                            p.time_penalty, 0, p.increment_time, p.weights.w_d, p.weights.w_t,
                            &Jplain, nullptr) == 0);
  EXPECT_LE(relErr(opt2.evaluateTimeCost(times), Jplain), 1e-9);
  EXPECT_TRUE(opt2.optimize() > 0);
  const double vmax1 =
      opt2.getPolynomialOptimizationRef().computeMaximumOfMagnitude(1, nullptr).value;
  EXPECT_LE(vmax1, 1.01 * vmax0 + hard.inequality_constraint_tolerance + 1e-9);
  EXPECT_TRUE(opt2.getOptimizationInfo().cost_soft_constraints == 0.0);
}

}  // namespace

// Free-derivative objectives of the nonlinear class on the tube-pattern
// problem (objectiveFunctionFreeConstraints, objectiveFunctionTimeAndConstraints,
// nonlinear_impl:947-1113) against the oracle, and optimizeFreeConstraints
// (:399-493) on the device.
TEST(gpu, FreeConstraintsObjective) {
  const Vertex::Vector vs = mainCppVertices();
  const std::vector<double> times = estimateSegmentTimes(vs, 2.0, 2.0);
  NonlinearOptimizationParameters p;
  p.objective = NonlinearOptimizationParameters::kOptimizeFreeConstraints;
  p.weights.w_c = 0.0;
  p.max_iterations = 20;
  p.min_bound = VectorXd::Constant(3, -100.0);
  p.max_bound = VectorXd::Constant(3, 100.0);
  PolynomialOptimizationNonLinear<10> opt(3, p);
  opt.setupFromVertices(vs, times, std::vector<std::pair<double, double>>(4, {0.15, 0.15}), 4);
  EXPECT_TRUE(opt.solveQCQP() == 0);
  std::vector<VectorXd> fc;
  opt.getConstrainedOptimizationRef().getFreeConstraints(&fc);
  // Tube pattern in dense form: start/end fully fixed, intermediates free.
  Dense d = toDense(vs, 5);
  for (int v = 1; v < d.S; ++v)
    for (int k = 0; k < 5; ++k) d.mask[v * 5 + k] = 0;
  std::vector<double> x;
  for (const VectorXd& v : fc)
    for (long i = 0; i < v.size(); ++i) x.push_back(v[i]);
  std::vector<VectorXd> g;
  const double J = opt.evaluateFreeConstraintsCost(fc, &g);
  double oJ = 0.0;
  std::vector<double> og(x.size());
  EXPECT_TRUE(orc_free_cost(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(), times.data(),
                            x.data(), 0, p.time_penalty, 0, nullptr, nullptr, 100.0, 1e12, &oJ,
                            og.data()) == 0);
  EXPECT_LE(relErr(J, oJ), 1e-9);
  std::vector<double> gx;
  for (const VectorXd& v : g)
    for (long i = 0; i < v.size(); ++i) gx.push_back(v[i]);
  EXPECT_LE(relErr(gx, og), 1e-8);
  const double J1 = opt.evaluateTimeAndFreeConstraintsCost(times, fc);
  double oJ1 = 0.0;
  EXPECT_TRUE(orc_free_cost(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(), times.data(),
                            x.data(), 1, p.time_penalty, 0, nullptr, nullptr, 100.0, 1e12, &oJ1,
                            nullptr) == 0);
  EXPECT_LE(relErr(J1, oJ1), 1e-9);
  // Without soft constraints J_d is minimised by the tube-pattern linear
  // solve, which the optimiser reaches from the QCQP solution.
  EXPECT_TRUE(opt.optimize() > 0);
  const OptimizationInfo info = opt.getOptimizationInfo();
  EXPECT_LE(info.cost_trajectory, J * (1 + 1e-12));
  PolynomialOptimizationConstrained<10> lin(3);
  lin.setupFromVertices(vs, times, std::vector<std::pair<double, double>>(4, {0.15, 0.15}), 4);
  lin.solveLinear();
  EXPECT_LE(relErr(info.cost_trajectory, 2.0 * lin.computeCost()), 1e-7);
  Trajectory traj;
  opt.getTrajectory(&traj);
  EXPECT_TRUE(traj.K() == 4);
}

// FindMinMax (test/test_polynomial.cpp:81-137): roots-based extrema of a
// random polynomial and its derivatives vs dense sampling (1e-2 there; the
// candidate search is exact, so 1e-6 of the range here).
TEST(host, PolynomialMinMax) {
  std::mt19937 gen(7);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  for (int trial = 0; trial < 20; ++trial) {
    VectorXd c(10);
    for (int k = 0; k < 10; ++k) c[k] = u(gen);
    const Polynomial p(c);
    const double t0 = -1.5 + 0.1 * trial, t1 = t0 + 3.0;
    for (int der = 0; der < 4; ++der) {
      std::pair<double, double> mn, mx;
      EXPECT_TRUE(p.computeMinMax(t0, t1, der, &mn, &mx));
      double smin = 1e300, smax = -1e300;
      for (double t = t0; t <= t1; t += 1e-4) {
        const double v = p.evaluate(t, der);
        smin = std::min(smin, v);
        smax = std::max(smax, v);
      }
      const double tol = 1e-6 * std::max(1.0, smax - smin);
      EXPECT_LE(mn.second, smin + tol);
      EXPECT_LE(smax, mx.second + tol);
      EXPECT_LE(smin - 1e-3 * std::max(1.0, smax - smin), mn.second);  // a real value
      EXPECT_LE(std::fabs(p.evaluate(mn.first, der) - mn.second), 1e-12 * (1.0 + smax - smin));
      EXPECT_TRUE(mn.first >= t0 && mn.first <= t1 && mx.first >= t0 && mx.first <= t1);
    }
  }
  // constant derivative: only the end points are candidates
  VectorXd lc(2);
  lc[0] = 1.0;
  lc[1] = 2.0;
  const Polynomial lin(lc);
  std::vector<double> cand;
  EXPECT_TRUE(lin.computeMinMaxCandidates(0.0, 1.0, 0, &cand));
  EXPECT_TRUE(cand.size() == 2);
}

// findRootsJenkinsTraub / Polynomial::getRoots (rpoly_ak1.cpp:70-117,
// polynomial.cpp:28-30): polynomials built from known roots (real, complex
// pairs, zeros at the origin) up to the 22nd degree of the magnitude
// convolution; the contract's edge cases (trailing zeros dropped, constant
// and zero polynomials have no roots).
TEST(host, FindRoots) {
  std::mt19937 gen(11);
  std::uniform_real_distribution<double> u(-2.0, 2.0);
  for (int trial = 0; trial < 60; ++trial) {
    const int n_real = trial % 7, n_pair = (trial / 7) % 4, n_zero = trial % 3 == 0 ? 1 : 0;
    std::vector<std::complex<double>> want;
    for (int k = 0; k < n_real; ++k) want.emplace_back(u(gen) * (1 + k), 0.0);
    for (int k = 0; k < n_pair; ++k) {
      const std::complex<double> z(u(gen), 0.1 + std::fabs(u(gen)));
      want.push_back(z);
      want.push_back(std::conj(z));
    }
    for (int k = 0; k < n_zero; ++k) want.emplace_back(0.0, 0.0);
    if (want.empty()) continue;
    // coefficients (increasing) of 3.5 * prod (t - r)
    std::vector<std::complex<double>> c(1, std::complex<double>(3.5, 0.0));
    for (const auto& r : want) {
      std::vector<std::complex<double>> nc(c.size() + 1);
      for (size_t i = 0; i < c.size(); ++i) {
        nc[i + 1] += c[i];
        nc[i] -= r * c[i];
      }
      c = nc;
    }
    VectorXd inc(static_cast<long>(c.size()) + 2);  // two trailing zeros, dropped
    for (size_t i = 0; i < c.size(); ++i) inc[static_cast<long>(i)] = c[i].real();
    VectorXcd roots;
    EXPECT_TRUE(findRootsJenkinsTraub(inc, &roots));
    EXPECT_TRUE(roots.size() == static_cast<long>(want.size()));
    for (const auto& r : want) {
      double best = 1e300;
      for (long i = 0; i < roots.size(); ++i) best = std::min(best, std::abs(roots[i] - r));
      EXPECT_LE(best, 1e-8 * (1.0 + std::abs(r)));
      if (r.imag() == 0.0) {  // a simple real root is reported exactly real
        bool real = false;
        for (long i = 0; i < roots.size(); ++i)
          real = real || (std::abs(roots[i] - r) <= 1e-8 * (1.0 + std::abs(r)) &&
                          roots[i].imag() == 0.0);
        EXPECT_TRUE(real);
      }
    }
  }
  VectorXcd roots;
  EXPECT_TRUE(findRootsJenkinsTraub(VectorXd{0.0, 0.0}, &roots) && roots.size() == 0);
  EXPECT_TRUE(findRootsJenkinsTraub(VectorXd{4.0, 0.0, 0.0}, &roots) && roots.size() == 0);
  EXPECT_TRUE(findRootsJenkinsTraub(VectorXd{0.0, 0.0, 2.0}, &roots) && roots.size() == 2 &&
              roots[0] == std::complex<double>(0.0, 0.0));
  // getRoots(derivative) finds the roots of that derivative: p = (t-1)(t-2)(t-3)
  const Polynomial p(VectorXd{-6.0, 11.0, -6.0, 1.0});
  EXPECT_TRUE(p.getRoots(0, &roots) && roots.size() == 3);
  EXPECT_LE(std::fabs(roots[0].real() - 1.0) + std::fabs(roots[1].real() - 2.0) +
                std::fabs(roots[2].real() - 3.0), 1e-12);
  EXPECT_TRUE(p.getRoots(1, &roots) && roots.size() == 2);  // 3t^2 - 12t + 11
  EXPECT_LE(std::fabs(roots[0].real() - (2.0 - 1.0 / std::sqrt(3.0))), 1e-12);
  // selectMinMaxFromRoots with getRoots(derivative + 1) = computeMinMax
  std::pair<double, double> mn, mx, mn2, mx2;
  EXPECT_TRUE(p.selectMinMaxFromRoots(0.5, 3.2, 0, roots, &mn, &mx));
  EXPECT_TRUE(p.computeMinMax(0.5, 3.2, 0, &mn2, &mx2));
  EXPECT_LE(std::fabs(mn.first - mn2.first) + std::fabs(mx.first - mx2.first), 1e-12);
  std::vector<double> cand;
  EXPECT_TRUE(!Polynomial::selectMinMaxCandidatesFromRoots(2.0, 1.0, roots, &cand));
}

// Segment::computeMinMaxMagnitudeCandidate(Time)s (segment.cpp:82-161) on
// random segments: the candidates attain the dense-sampled maximum of the
// magnitude, the start / end times come first, one-dimension lists are the
// derivative's candidates, and bad arguments return false.
TEST(host, SegmentMagnitudeCandidates) {
  std::mt19937 gen(5);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  for (int trial = 0; trial < 20; ++trial) {
    const int D = 1 + trial % 3;
    Segment s(10, D);
    s.setTime(2.0);
    for (int d = 0; d < D; ++d) {
      VectorXd c(10);
      for (int k = 0; k < 10; ++k) c[k] = u(gen) / (1 + k);
      s[d] = Polynomial(c);
    }
    std::vector<int> dims;
    for (int d = 0; d < D; ++d) dims.push_back(d);
    for (int der = 0; der < 3; ++der) {
      std::vector<Extremum> cand;
      EXPECT_TRUE(s.computeMinMaxMagnitudeCandidates(der, 0.0, 2.0, dims, &cand));
      EXPECT_TRUE(cand.size() >= 2 && cand[0].time == 0.0 && cand[1].time == 2.0);
      Extremum mn, mx;
      EXPECT_TRUE(s.selectMinMaxMagnitudeFromCandidates(der, 0.0, 2.0, dims, cand, &mn, &mx));
      double smax = 0.0;
      for (double t = 0.0; t <= 2.0; t += 1e-4) smax = std::max(smax, s.evaluate(t, der).norm());
      EXPECT_LE(smax, mx.value * (1 + 1e-9));
      EXPECT_LE(mx.value, smax + 1e-3 * std::max(1.0, smax));
      if (D == 1) {
        std::vector<double> pc, st;
        EXPECT_TRUE(s[0].computeMinMaxCandidates(0.0, 2.0, der, &pc));
        EXPECT_TRUE(s.computeMinMaxMagnitudeCandidateTimes(der, 0.0, 2.0, dims, &st));
        EXPECT_TRUE(pc == st);
      }
    }
  }
  Segment s(10, 2);
  s.setTime(1.0);
  std::vector<double> t;
  EXPECT_TRUE(!s.computeMinMaxMagnitudeCandidateTimes(1, 0.0, 1.0, {}, &t));
  EXPECT_TRUE(!s.computeMinMaxMagnitudeCandidateTimes(1, 0.0, 1.0, {0, 2}, &t));
  EXPECT_TRUE(!s.computeMinMaxMagnitudeCandidateTimes(1, 1.0, 0.0, {0, 1}, &t));
  Extremum mn, mx;
  EXPECT_TRUE(!s.selectMinMaxMagnitudeFromCandidates(1, 1.0, 0.0, {0, 1}, {}, &mn, &mx));
}

// test_polynomial.cpp:68-79 (PolynomialTest.Convolution): the product of
// 1 + 2t and -1 + 3t, coefficient by coefficient.
TEST(host, PolynomialConvolution) {
  VectorXd c1(2), c2(2);
  c1[0] = 1.0;
  c1[1] = 2.0;
  c2[0] = -1.0;
  c2[1] = 3.0;
  const Polynomial p(c1), q(c2);
  const Polynomial conv = p * q;
  const VectorXd got = conv.getCoefficients();
  const double want[3] = {c1[0] * c2[0], c1[0] * c2[1] + c1[1] * c2[0], c1[1] * c2[1]};
  EXPECT_TRUE(got.size() == 3);
  for (int k = 0; k < 3 && k < got.size(); ++k) EXPECT_TRUE(got[k] == want[k]);
}

// Trajectory container operations (trajectory.cpp:136-251).
TEST(host, TrajectoryContainers) {
  Segment::Vector segs;
  for (int s = 0; s < 3; ++s) {
    Segment seg(10, 3);
    seg.setTime(1.0 + s);
    for (int d = 0; d < 3; ++d) {
      VectorXd c(10);
      for (int k = 0; k < 10; ++k) c[k] = (d + s) + k * (2.0 * d - s - d - s) / 9.0;
      seg[d] = Polynomial(c);
    }
    segs.push_back(seg);
  }
  Trajectory traj;
  traj.setSegments(segs);
  const Trajectory y = traj.getTrajectoryWithSingleDimension(1);
  EXPECT_TRUE(y.D() == 1 && y.K() == 3);
  for (int s = 0; s < 3; ++s) EXPECT_TRUE(y.segments()[s][0] == segs[s][1]);
  Trajectory x = traj.getTrajectoryWithSingleDimension(0), xy;
  EXPECT_TRUE(x.getTrajectoryWithAppendedDimension(y, &xy));
  EXPECT_TRUE(xy.D() == 2 && xy.K() == 3);
  for (int s = 0; s < 3; ++s) {
    EXPECT_TRUE(xy.segments()[s][0] == segs[s][0]);
    EXPECT_TRUE(xy.segments()[s][1] == segs[s][1]);
  }
  Trajectory empty, same;
  EXPECT_TRUE(empty.getTrajectoryWithAppendedDimension(traj, &same));
  EXPECT_TRUE(same == traj);
  Trajectory merged;
  EXPECT_TRUE(traj.addTrajectories({traj, traj}, &merged));
  EXPECT_TRUE(merged.K() == 9);
  EXPECT_LE(std::fabs(merged.getMaxTime() - 18.0), 1e-12);
  EXPECT_TRUE(!traj.addTrajectories({y}, &merged));  // D differs
}

// ExtremaOfMagnitude (test_polynomial_optimization.cpp:307-406): the device
// min / max of |p^(k)| over all dimensions or a subset vs dense sampling, and
// the maximum vs computeMaximumOfMagnitude.
TEST(gpu, TrajectoryMinMaxMagnitude) {
  const Fixture& f = kSeg10Dim3;
  const Vertex::Vector vs = fixtureVertices(f, 10);
  const std::vector<double> times = estimateSegmentTimes(vs, f.vmax, f.amax);
  PolynomialOptimization<10> opt(3);
  opt.setupFromVertices(vs, times, 4);
  opt.solveLinear();
  Trajectory traj;
  opt.getTrajectory(&traj);
  for (int der = 0; der < 4; ++der)
    for (const std::vector<int>& dims : {std::vector<int>{0, 1, 2}, std::vector<int>{0, 2}}) {
      Extremum mn, mx;
      EXPECT_TRUE(traj.computeMinMaxMagnitude(der, dims, &mn, &mx));
      double smin = 1e300, smax = -1.0;
      for (int s = 0; s < traj.K(); ++s)
        for (double t = 0.0; t <= traj.segments()[s].getTime(); t += 1e-3) {
          const VectorXd v = traj.segments()[s].evaluate(t, der);
          double m2 = 0.0;
          for (int d : dims) m2 += v[d] * v[d];
          smin = std::min(smin, std::sqrt(m2));
          smax = std::max(smax, std::sqrt(m2));
        }
      EXPECT_LE(std::fabs(mx.value - smax), 1e-2 * std::max(1.0, smax));
      EXPECT_LE(smax, mx.value * (1 + 1e-12) + 1e-12);
      EXPECT_LE(mn.value, smin + 1e-12);
      EXPECT_LE(std::fabs(mn.value - smin), 1e-2 * std::max(1.0, smax));
      const VectorXd at = traj.segments()[mx.segment_idx].evaluate(mx.time, der);
      double m2 = 0.0;
      for (int d : dims) m2 += at[d] * at[d];
      EXPECT_LE(std::fabs(std::sqrt(m2) - mx.value), 1e-9 * std::max(1.0, mx.value));
      if (dims.size() == 3)
        EXPECT_LE(relErr(mx.value, opt.computeMaximumOfMagnitude(der, nullptr).value), 1e-12);
    }
}

// printMatlabSampledTrajectory (nonlinear_impl:2907-3003): row count, column
// layout and values against host evaluation at the 6 printed digits.
TEST(gpu, PrintMatlabSampledTrajectory) {
  const Fixture& f = kSeg10Dim3;
  const Vertex::Vector all = fixtureVertices(f, 10);
  Vertex::Vector vs(all.begin(), all.begin() + 4);
  vs.back().makeStartOrEnd(VectorXd::Constant(3, 1.0), 4);
  const std::vector<double> times = estimateSegmentTimes(vs, f.vmax, f.amax);
  NonlinearOptimizationParameters p;
  p.objective = NonlinearOptimizationParameters::kOptimizeTime;
  p.solve_time_with_qcqp = false;  // the upstream linear inner solve
  p.weights.w_c = 0.0;
  p.max_iterations = 5;
  PolynomialOptimizationNonLinear<10> opt(3, p);
  opt.setupFromVertices(vs, times, std::vector<std::pair<double, double>>(3, {0.15, 0.15}), 4);
  opt.optimize();
  const std::string path = "/tmp/mtg_matlab_test.txt";
  opt.printMatlabSampledTrajectory(path);
  Trajectory traj;
  opt.getTrajectory(&traj);
  const std::vector<double> T = traj.getSegmentTimes();
  int rows = 0;
  for (double t : T) rows += static_cast<int>(std::ceil(t / 0.01)) + 1;
  std::ifstream in(path);
  std::vector<std::vector<double>> m;
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream is(line);
    std::vector<double> r;
    double v;
    while (is >> v) r.push_back(v);
    m.push_back(r);
  }
  EXPECT_TRUE(static_cast<int>(m.size()) == rows);
  EXPECT_TRUE(m.front().size() == 17u);
  double acc = 0.0;
  for (size_t s = 0; s < T.size(); ++s) {
    acc += T[s];
    EXPECT_LE(std::fabs(m[s][16] - acc), 1e-5 * acc);
  }
  // row 150 lies in the first segment (T_0 > 1.5 s at these limits)
  const int r = std::min(150, static_cast<int>(std::ceil(T[0] / 0.01)) - 1);
  EXPECT_LE(std::fabs(m[r][0] - r * 0.01), 1e-9 + 1e-5 * r * 0.01);
  for (int k = 0; k <= 4; ++k) {
    const VectorXd v = traj.segments()[0].evaluate(r * 0.01, k);
    for (int d = 0; d < 3; ++d)
      EXPECT_LE(std::fabs(m[r][1 + 3 * k + d] - v[d]), 1e-5 * std::max(1e-3, std::fabs(v[d])));
  }
}

// getCostAndGradientCollision (nonlinear_impl:1609-1780) through the shim on
// a dense occupancy grid (setOccupancyGrid) vs the oracle restatement.
TEST(gpu, CollisionCostMatchesOracle) {
  const Vertex::Vector vs = mainCppVertices();
  const std::vector<double> times = estimateSegmentTimes(vs, 2.0, 2.0);
  NonlinearOptimizationParameters p;
  p.map_resolution = 0.05;
  p.min_bound = VectorXd::Constant(3, 0.0);
  p.max_bound = VectorXd::Constant(3, 16.0);
  p.robot_radius = 0.1;
  PolynomialOptimizationNonLinear<10> opt(3, p);
  opt.setupFromVertices(vs, times, std::vector<std::pair<double, double>>(4, {0.15, 0.15}), 4);
  EXPECT_TRUE(opt.solveQCQP() == 0);
  const int n = 320;
  std::vector<float> occ(static_cast<size_t>(n) * n * n, -1.0f);
  std::mt19937 gen(11);
  std::uniform_int_distribution<int> u(0, n - 1);
  for (int i = 0; i < 200000; ++i) occ[(static_cast<size_t>(u(gen)) * n + u(gen)) * n + u(gen)] = 0.5f;
  opt.setOccupancyGrid(occ, n, n, n);
  std::vector<VectorXd> g;
  bool coll = true;
  const double J = opt.getCostAndGradientCollision(&g, &coll);
  std::vector<VectorXd> fc;
  opt.getConstrainedOptimizationRef().getFreeConstraints(&fc);
  std::vector<double> x;
  for (const VectorXd& v : fc)
    for (long i = 0; i < v.size(); ++i) x.push_back(v[i]);
  Dense d = toDense(vs, 5);
  for (int v = 1; v < d.S; ++v)
    for (int k = 0; k < 5; ++k) d.mask[v * 5 + k] = 0;
  const double prm[11] = {0.05, 0, 0, 0, 16, 16, 16, p.epsilon, 0.1, p.coll_pot_multiplier,
                          p.coll_check_time_increment};
  double oJ = 0.0;
  int oc = 0;
  std::vector<double> og(x.size());
  EXPECT_TRUE(orc_collision_cost(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(), times.data(),
                                 x.data(), occ.data(), n, n, n, prm, 20, &oJ, &oc, nullptr,
                                 og.data()) == 0);
  EXPECT_TRUE((coll ? 1 : 0) == oc);
  EXPECT_LE(std::fabs(J - oJ), 1e-9 * std::max(1.0, std::fabs(oJ)));
  std::vector<double> gx;
  for (const VectorXd& v : g)
    for (long i = 0; i < v.size(); ++i) gx.push_back(v[i]);
  if (!oc && oJ > 0) EXPECT_LE(relErr(gx, og), 1e-7);
  std::printf("  collision cost %.6g (oracle %.6g), collision %d\n", J, oJ, oc);
}

// kOptimizeFreeConstraintsAndTime (optimizeTimeAndFreeConstraints,
// nonlinear_impl:610-706) from the tube QCQP start: with the default
// LN_SBPLX the shim runs the device Subplex over all S + 3 n_p variables
// (mtg_time_free_optimize_ex, optimizer 1) and follows the oracle's Subplex
// (orc_time_free_optimize_sbplx); with another algorithm the
// block-alternating descent and the oracle port of it.  The objective does
// not rise and the bounds hold.
void runTimeAndFreeConstraints(nlopt::algorithm algo) {
  const Vertex::Vector vs = mainCppVertices();
  const std::vector<double> times = estimateSegmentTimes(vs, 2.0, 2.0);
  NonlinearOptimizationParameters p;
  p.objective = NonlinearOptimizationParameters::kOptimizeFreeConstraintsAndTime;
  p.weights.w_c = 0.0;
  p.algorithm = algo;
  p.max_iterations = algo == nlopt::LN_SBPLX ? 120 : 30;
  PolynomialOptimizationNonLinear<10> opt(3, p);
  opt.setupFromVertices(vs, times, std::vector<std::pair<double, double>>(4, {0.15, 0.15}), 4);
  EXPECT_TRUE(opt.solveQCQP() == 0);
  std::vector<VectorXd> fc;
  opt.getConstrainedOptimizationRef().getFreeConstraints(&fc);
  const double J0 = opt.evaluateTimeAndFreeConstraintsCost(times, fc);
  const int res = opt.optimize();
  EXPECT_TRUE(res > 0);
  const OptimizationInfo info = opt.getOptimizationInfo();
  EXPECT_TRUE(info.n_iterations >= 2 && info.n_iterations <= p.max_iterations);
  std::vector<double> t1;
  opt.getConstrainedOptimizationRef().getSegmentTimes(&t1);
  std::vector<VectorXd> f1;
  opt.getConstrainedOptimizationRef().getFreeConstraints(&f1);
  const double J1 = opt.evaluateTimeAndFreeConstraintsCost(t1, f1);
  EXPECT_LE(J1, J0);
  EXPECT_LE(relErr(J1, info.cost_trajectory + info.cost_time), 1e-9);
  for (size_t i = 0; i < t1.size(); ++i) EXPECT_TRUE(t1[i] >= 0.1 && t1[i] <= 2.0 * times[i]);
  // Oracle from the same start.
  Dense d = toDense(vs, 5);
  for (int v = 1; v < d.S; ++v)
    for (int k = 0; k < 5; ++k) d.mask[v * 5 + k] = 0;
  std::vector<double> x, ot = times;
  for (const VectorXd& v : fc)
    for (long i = 0; i < v.size(); ++i) x.push_back(v[i]);
  double oJ = 0.0;
  int oev = 0, ores = 0;
  if (algo == nlopt::LN_SBPLX) {
    EXPECT_TRUE(orc_time_free_optimize_sbplx(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(),
                                             x.data(), ot.data(), p.time_penalty, 0, nullptr,
                                             nullptr, 100.0, 1e12, p.max_iterations, p.f_rel,
                                             p.f_abs, p.initial_stepsize_rel, &oJ, &oev, &ores,
                                             nullptr) == 0);
    EXPECT_TRUE(ores == res);
  } else {
    EXPECT_TRUE(orc_time_free_optimize(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(), x.data(),
                                       ot.data(), p.time_penalty, p.increment_time, 0, nullptr,
                                       nullptr, 100.0, 1e12, 30, &oJ, &oev) == 0);
  }
  std::fprintf(stderr, "  free+time (%s): evals %d (oracle %d), J %.12g (oracle %.12g)\n",
               algo == nlopt::LN_SBPLX ? "LN_SBPLX" : "descent",
               static_cast<int>(info.n_iterations), oev, J1, oJ);
  EXPECT_TRUE(oev == info.n_iterations);
  EXPECT_LE(relErr(J1, oJ), 1e-6);
  EXPECT_LE(relErr(t1, ot), 1e-6);
}

TEST(gpu, OptimizeTimeAndFreeConstraints) { runTimeAndFreeConstraints(nlopt::LN_SBPLX); }
TEST(gpu, OptimizeTimeAndFreeConstraintsDescent) {
  runTimeAndFreeConstraints(nlopt::LN_BOBYQA);
}

// The reference demo (src/main.cpp:15-126): kOptimizeFreeConstraintsAndCollision
// with LD_LBFGS and main.cpp's parameters, here over a synthetic forest (the
// demo's supereight map is a private file, main.cpp:17-19).  optimize() runs
// mtg_coll_optimize (device L-BFGS in place of NLopt): it lowers the objective
// from the QCQP start and takes the same steps as the oracle port; likewise
// the time variant kOptimizeFreeConstraintsAndCollisionAndTime.
std::vector<float> demoForest(int* nx, int* ny, int* nz) {
  *nx = 120;
  *ny = 120;
  *nz = 90;
  const double res = 0.1, r = 0.25;
  const double trees[][2] = {{3.73, 6.57}, {4.28, 3.60}, {6.74, 2.78}, {8.5, 8.5},
                             {9.5, 4.0},   {6.0, 9.0},   {2.0, 2.5}};
  std::vector<float> occ(static_cast<size_t>(*nx) * *ny * *nz, -1.0f);
  for (int z = 0; z < *nz; ++z)
    for (int y = 0; y < *ny; ++y)
      for (int x = 0; x < *nx; ++x)
        for (const auto& c : trees) {
          const double dx = (x + 0.5) * res - c[0], dy = (y + 0.5) * res - c[1];
          if (dx * dx + dy * dy <= r * r) occ[(static_cast<size_t>(z) * *ny + y) * *nx + x] = 1.0f;
        }
  return occ;
}

NonlinearOptimizationParameters demoParameters() {  // main.cpp:75-110
  NonlinearOptimizationParameters p;
  p.solve_with_position_constraint = true;
  p.objective = NonlinearOptimizationParameters::kOptimizeFreeConstraintsAndCollision;
  p.print_debug_info = false;
  p.max_iterations = 25;
  p.max_time = -1;
  p.f_rel = 0.000001;
  p.x_rel = 0.01;
  p.use_soft_constraints = false;
  p.soft_constraint_weight = 100.0;
  p.time_penalty = 500.0;
  p.initial_stepsize_rel = 0.1;
  p.inequality_constraint_tolerance = 0.1;
  p.weights.w_d = 50;
  p.weights.w_c = 50;
  p.weights.w_t = 0.1;
  p.weights.w_sc = 1.0;
  p.use_numeric_grad = false;
  p.use_continous_distance = false;
  p.increment_time = 0.000001;
  p.epsilon = 0.3;
  p.coll_pot_multiplier = 20.0;
  p.is_collision_safe = true;
  p.is_simple_numgrad_time = true;
  p.is_simple_numgrad_constraints = true;
  p.coll_check_time_increment = 0.1;
  p.is_coll_raise_first_iter = true;
  p.robot_radius = 0.15;
  p.add_coll_raise = 0.0000001;
  p.algorithm = static_cast<nlopt::algorithm>(11);
  p.random_seed = 12345678;
  p.map_resolution = 0.1;
  VectorXd lo(3), hi(3);
  lo[0] = 1.4; lo[1] = 1.4; lo[2] = 3.9;
  hi[0] = 11.3; hi[1] = 11.3; hi[2] = 8.8;
  p.min_bound = lo;
  p.max_bound = hi;
  p.side = 5;
  return p;
}

TEST(gpu, DemoCollisionObjective) {
  const Vertex::Vector vs = mainCppVertices();
  const std::vector<double> times = estimateSegmentTimesNfabian(vs, 2.0, 2.0, 6.5);
  const std::vector<std::pair<double, double>> radii(4, {0.15, 0.15});
  int nx, ny, nz;
  const std::vector<float> occ = demoForest(&nx, &ny, &nz);
  Dense d = toDense(vs, 5);
  for (int v = 1; v < d.S; ++v)
    for (int k = 0; k < 5; ++k) d.mask[v * 5 + k] = 0;
  for (int with_time = 0; with_time < 2; ++with_time) {
    NonlinearOptimizationParameters p = demoParameters();
    if (with_time)
      p.objective = NonlinearOptimizationParameters::kOptimizeFreeConstraintsAndCollisionAndTime;
    PolynomialOptimizationNonLinear<10> opt(3, p);
    opt.setOctree(nullptr);  // source compatibility: the map comes from setOccupancyGrid
    EXPECT_TRUE(opt.setupFromVertices(vs, times, radii, 4));
    opt.setOccupancyGrid(occ, nx, ny, nz);
    // The start the optimiser uses: the tube QCQP (main.cpp sets
    // solve_with_position_constraint).
    PolynomialOptimizationConstrained<10> qp(3);
    qp.setupFromVertices(vs, times, radii, 4);
    EXPECT_TRUE(qp.solveQCQP() == 0);
    std::vector<VectorXd> fc;
    qp.getFreeConstraints(&fc);
    std::vector<double> x0;
    if (with_time) x0 = times;
    for (const VectorXd& v : fc)
      for (long i = 0; i < v.size(); ++i) x0.push_back(v[i]);
    const double prm[23] = {0.1, 1.4, 1.4, 3.9, 11.3, 11.3, 8.8, 0.3, 0.15, 20.0, 0.1,
                            50.0, 50.0, 0.1, 1.0, 1e-7, 1e-6, 100.0, 1e12, 1e-6, -1.0, 0.01,
                            -1.0};
    const int ip[7] = {20, 1, 1, 1, 1, 0, 10};
    double J0 = 0.0;
    int c0 = 1;
    EXPECT_TRUE(orc_coll_cost(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(), times.data(),
                              with_time, x0.data(), occ.data(), nx, ny, nz, prm, ip, nullptr,
                              nullptr, 0.0, &J0, nullptr, nullptr, &c0) == 0);
    EXPECT_TRUE(c0 == 0);
    const int res = opt.optimize();
    EXPECT_TRUE(res == nlopt::FTOL_REACHED || res == nlopt::XTOL_REACHED ||
                res == nlopt::MAXEVAL_REACHED || res == nlopt::SUCCESS);
    const OptimizationInfo info = opt.getOptimizationInfo();
    const double J1 = info.cost_trajectory + info.cost_collision + info.cost_time +
                      info.cost_soft_constraints;
    EXPECT_TRUE(J1 < J0);
    EXPECT_TRUE(info.n_iterations >= 2 && info.n_iterations <= 25);
    if (with_time) {
      // main.cpp's increment_time = 1e-6: the reference's forward difference
      // of J_d over it is rounding noise (~1e-4 relative), so the port's path
      // parts from the device's; descent and the T >= 0.1 bounds only.
      std::vector<double> t1;
      opt.getConstrainedOptimizationRef().getSegmentTimes(&t1);
      for (double ti : t1) EXPECT_TRUE(ti >= 0.1);
      std::printf("  collision+time: J %.6g -> %.6g in %d evaluations (result %d)\n", J0, J1,
                  info.n_iterations, res);
      continue;
    }
    // Oracle port from the same start with the reference's bounds and steps.
    const size_t nv = x0.size();
    std::vector<double> lo(nv, -HUGE_VAL), hi(nv, HUGE_VAL), step(nv), ox = x0;
    for (size_t i = 0; i < nv; ++i) {
      const double a = std::fabs(x0[i]);
      step[i] = (!with_time && a > 5) ? p.initial_stepsize_position : 0.1 * a;
      if (with_time && i < 4) lo[i] = 0.1;
    }
    double oJ = 0.0, oterms[4];
    int oev = 0, ores = 0;
    EXPECT_TRUE(orc_coll_optimize(10, 3, 4, 4, 5, d.mask.data(), d.vals.data(), times.data(),
                                  with_time, occ.data(), nx, ny, nz, prm, ip, nullptr, nullptr,
                                  lo.data(), hi.data(), step.data(), 25, ox.data(), &oJ, &oev,
                                  &ores, oterms) == 0);
    EXPECT_TRUE(oev == info.n_iterations);
    EXPECT_TRUE(ores == res);
    EXPECT_LE(relErr(J1, oJ), 1e-6);
    std::vector<VectorXd> f1;
    opt.getConstrainedOptimizationRef().getFreeConstraints(&f1);
    std::vector<double> x1;
    if (with_time) opt.getConstrainedOptimizationRef().getSegmentTimes(&x1);
    for (const VectorXd& v : f1)
      for (long i = 0; i < v.size(); ++i) x1.push_back(v[i]);
    EXPECT_LE(relErr(x1, ox), 1e-6);
    // The trajectory keeps the start / end constraints (makeStartOrEnd).
    Trajectory traj;
    opt.getTrajectory(&traj);
    EXPECT_LE(std::fabs(traj.evaluate(0.0, 0)[0] - 2.7), 1e-8);
    EXPECT_LE(std::fabs(traj.evaluate(traj.getMaxTime(), 0)[1] - 2.2), 1e-8);
    std::printf("  %s: J %.6g -> %.6g in %d evaluations (result %d; oracle %.6g, %d)\n",
                with_time ? "collision+time" : "collision", J0, J1, info.n_iterations, res, oJ,
                oev);
  }
}

// getAllTrajectories (polynomial_optimization_nonlinear.h:316-331): one
// trajectory per evaluation of the collision objective (nonlinear_impl:1244),
// in order, accumulating over optimize() calls as the reference's
// all_trajectories_ does.  The first is the start (the tube QCQP solution),
// the result is one of them (the device optimiser keeps the best evaluated
// point), and the initial trajectories match the start.
TEST(gpu, AllTrajectoriesHistory) {
  const Vertex::Vector vs = mainCppVertices();
  const std::vector<double> times = estimateSegmentTimesNfabian(vs, 2.0, 2.0, 6.5);
  const std::vector<std::pair<double, double>> radii(4, {0.15, 0.15});
  int nx, ny, nz;
  const std::vector<float> occ = demoForest(&nx, &ny, &nz);
  PolynomialOptimizationNonLinear<10> opt(3, demoParameters());
  EXPECT_TRUE(opt.setupFromVertices(vs, times, radii, 4));
  opt.setOccupancyGrid(occ, nx, ny, nz);
  std::vector<Trajectory> none;
  opt.getAllTrajectories(&none);
  EXPECT_TRUE(none.empty());
  opt.optimize();
  const int n1 = opt.getOptimizationInfo().n_iterations;
  std::vector<Trajectory> hist;
  opt.getAllTrajectories(&hist);
  EXPECT_TRUE(static_cast<int>(hist.size()) == n1 && n1 >= 2);
  Trajectory init, init_rp, result;
  opt.getInitialSolutionTrajectory(&init);
  opt.getInitialTrajectoryAfterRemovingPos(&init_rp);
  opt.getTrajectory(&result);
  auto coeffDiff = [](const Trajectory& a, const Trajectory& b) {
    Segment::Vector sa, sb;
    a.getSegments(&sa);
    b.getSegments(&sb);
    if (sa.size() != sb.size()) return 1e300;
    const std::vector<double> ca = coeffsOf(sa, 10), cb = coeffsOf(sb, 10);
    double tdiff = 0.0;
    for (size_t s = 0; s < sa.size(); ++s) tdiff += std::fabs(sa[s].getTime() - sb[s].getTime());
    return relErr(ca, cb) + tdiff;
  };
  EXPECT_LE(coeffDiff(init_rp, init), 0.0);
  if (!hist.empty()) EXPECT_LE(coeffDiff(hist.front(), init), 1e-9);
  double best = 1e300;
  for (const Trajectory& t : hist) best = std::min(best, coeffDiff(t, result));
  EXPECT_LE(best, 1e-9);
  // Free derivatives as x, y, z triples: the tube problem's d_p, per index.
  std::vector<Vector3d> f3;
  opt.getFreeConstraints(&f3);
  std::vector<VectorXd> fx;
  opt.getConstrainedOptimizationRef().getFreeConstraints(&fx);
  EXPECT_TRUE(fx.size() == 3 && f3.size() == static_cast<size_t>(fx[0].size()));
  for (size_t i = 0; i < f3.size() && fx.size() == 3; ++i)
    EXPECT_TRUE(f3[i].x() == fx[0][static_cast<long>(i)] &&
                f3[i].y() == fx[1][static_cast<long>(i)] &&
                f3[i].z() == fx[2][static_cast<long>(i)]);
  // A second run appends its evaluations.
  opt.optimize();
  const int n2 = opt.getOptimizationInfo().n_iterations;
  std::vector<Trajectory> hist2;
  opt.getAllTrajectories(&hist2);
  EXPECT_TRUE(static_cast<int>(hist2.size()) == n1 + n2);
  std::printf("  history: %d + %d evaluations\n", n1, n2);
}

// computeInitialSolutionWithPositionConstraints (nonlinear_impl:199-272) and
// the declared WithoutPositionConstraints: the QCQP solution becomes the
// initial trajectory and its d_p (intermediate positions free) the problem's
// free constraints.
TEST(gpu, ComputeInitialSolution) {
  const Vertex::Vector vs = mainCppVertices();
  const std::vector<double> times = estimateSegmentTimesNfabian(vs, 2.0, 2.0, 6.5);
  const std::vector<std::pair<double, double>> radii(4, {0.15, 0.15});
  PolynomialOptimizationConstrained<10> qp(3);
  qp.setupFromVertices(vs, times, radii, 4);
  EXPECT_TRUE(qp.solveQCQP() == 0);
  std::vector<VectorXd> want;
  qp.getFreeConstraints(&want);
  for (int variant = 0; variant < 2; ++variant) {
    PolynomialOptimizationNonLinear<10> opt(3, demoParameters());
    EXPECT_TRUE(opt.setupFromVertices(vs, times, radii, 4));
    EXPECT_TRUE(variant ? opt.computeInitialSolutionWithoutPositionConstraints()
                        : opt.computeInitialSolutionWithPositionConstraints());
    std::vector<VectorXd> got;
    opt.getConstrainedOptimizationRef().getFreeConstraints(&got);
    EXPECT_TRUE(got.size() == want.size());
    for (size_t d = 0; d < got.size() && d < want.size(); ++d)
      EXPECT_LE(relErr(std::vector<double>(got[d].data(), got[d].data() + got[d].size()),
                       std::vector<double>(want[d].data(), want[d].data() + want[d].size())),
                1e-12);
    Trajectory init;
    opt.getInitialSolutionTrajectory(&init);
    Segment::Vector segs;
    qp.getSegments(&segs);
    Segment::Vector isegs;
    init.getSegments(&isegs);
    EXPECT_LE(relErr(coeffsOf(isegs, 10), coeffsOf(segs, 10)), 1e-12);
  }
}

// setFreeEndpointDerivativeHardConstraints (nonlinear_impl:2858-2905) writes
// through .at(): a position-magnitude constraint with
// solve_with_position_constraint wraps (derivative - 1) and throws
// std::out_of_range instead of writing out of bounds.
TEST(gpu, EndpointBoundsRejectPositionMagnitude) {
  const Vertex::Vector vs = mainCppVertices();
  const std::vector<double> times = estimateSegmentTimesNfabian(vs, 2.0, 2.0, 6.5);
  const std::vector<std::pair<double, double>> radii(4, {0.15, 0.15});
  int nx, ny, nz;
  const std::vector<float> occ = demoForest(&nx, &ny, &nz);
  PolynomialOptimizationNonLinear<10> opt(3, demoParameters());
  EXPECT_TRUE(opt.setupFromVertices(vs, times, radii, 4));
  opt.setOccupancyGrid(occ, nx, ny, nz);
  opt.addMaximumMagnitudeConstraint(derivative_order::POSITION, 20.0);
  EXPECT_THROW(opt.optimize());
}

// Latency of the drop-in single-trajectory call (run on demand: the
// "latency" group).  PolynomialOptimization<10>::solveLinear() at S = 3 (C1,
// BASELINE.json configs[0]) and S = 10 goes through mtg_linear_solve_host:
// one H2D copy, one launch and one D2H copy on the plan's own stream.  Each
// call is timed alone (steady_clock) after a warm-up; the oracle's
// setupFromVertices + solveLinear + computeCost on one host core
// (orc_bench_linear, the reference's timed region) is timed beside it.
// Prints one JSON line per size.
TEST(latency, SolveLinearSingle) {
  for (int S : {3, 10}) {
    const Fixture f{3, 4, S, 105, 3.0, 5.0};
    const Vertex::Vector vs = fixtureVertices(f, 10);
    const std::vector<double> t = estimateSegmentTimes(vs, f.vmax, f.amax);
    PolynomialOptimization<10> opt(f.D);
    opt.setupFromVertices(vs, t, f.r);
    for (int i = 0; i < 200; ++i) EXPECT_TRUE(opt.solveLinear());
    const int reps = 5000;
    std::vector<double> us(reps);
    const auto t_all = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) {
      const auto a = std::chrono::steady_clock::now();
      opt.solveLinear();
      us[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a)
                  .count();
    }
    const double mean =
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_all)
            .count() / reps;
    std::sort(us.begin(), us.end());
    const Dense d = toDense(vs, 5);
    int64_t n = 0;
    double sec = 0.0;
    EXPECT_TRUE(orc_bench_linear(10, f.D, f.r, S, 5, 1, d.mask.data(), d.vals.data(), t.data(),
                                 1, 2.0, &n, &sec) == 0);
    const double cpu_us = sec / static_cast<double>(n) * 1e6;
    std::printf("LATENCY {\"call\": \"PolynomialOptimization<10>::solveLinear\", \"S\": %d, "
                "\"D\": 3, \"reps\": %d, \"median_us\": %.3f, \"p10_us\": %.3f, "
                "\"p90_us\": %.3f, \"mean_us\": %.3f, \"cpu_port_us\": %.3f, "
                "\"cpu_cores\": 1}\n",
                S, reps, us[reps / 2], us[reps / 10], us[reps * 9 / 10], mean, cpu_us);
    // the solution is the oracle's (the staging path returns the same data)
    Segment::Vector segs;
    opt.getSegments(&segs);
    checkPath(vs, segs, 10);
  }
}

int main(int argc, char** argv) {
  const std::string group = argc > 1 ? argv[1] : "host";
  int run = 0, failed_tests = 0;
  for (const TestCase& t : registry()) {
    if (group != "all" && group != t.group) continue;
    const int before = g_failures;
    std::printf("[ RUN      ] %s.%s\n", t.group, t.name);
    try {
      t.fn();
    } catch (const std::exception& e) {
      ++g_failures;
      std::fprintf(stderr, "  EXCEPTION: %s\n", e.what());
    }
    const bool ok = g_failures == before;
    failed_tests += ok ? 0 : 1;
    std::printf("[ %s ] %s.%s\n", ok ? "      OK" : " FAILED ", t.group, t.name);
    ++run;
  }
  std::printf("%d tests, %d checks, %d failed tests\n", run, g_checks, failed_tests);
  return failed_tests == 0 && run > 0 ? 0 : 1;
}
