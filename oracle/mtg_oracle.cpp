// ORACLE — TEST INFRASTRUCTURE ONLY (see mtg_oracle.h for the contract).
//
// Reference-faithful FP64 CPU restatement of the reference's hot path.  The
// data structures follow the reference step by step (per-segment Q, A, A^-1
// via the Schur complement, the 0/1 reordering matrix M built from std::set
// ordered constraints, R = M^T blkdiag(H) M, a Householder QR solve of R_pp
// standing in for Eigen::SparseQR<COLAMD>, per-segment coefficient recovery),
// without the reference's unconditional stdout prints.
#include "mtg_oracle.h"
#include "orc_sbplx.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <random>
#include <set>
#include <vector>

namespace {

// ----------------------------------------------------------------------------
// Small dense matrix (row-major).
struct Mat {
  int r = 0, c = 0;
  std::vector<double> a;
  Mat() {}
  Mat(int r_, int c_) : r(r_), c(c_), a(static_cast<size_t>(r_) * c_, 0.0) {}
  double& operator()(int i, int j) { return a[static_cast<size_t>(i) * c + j]; }
  double operator()(int i, int j) const {
    return a[static_cast<size_t>(i) * c + j];
  }
};

Mat matmul(const Mat& A, const Mat& B) {
  Mat C(A.r, B.c);
  for (int i = 0; i < A.r; ++i)
    for (int k = 0; k < A.c; ++k) {
      const double aik = A(i, k);
      if (aik == 0.0) continue;
      for (int j = 0; j < B.c; ++j) C(i, j) += aik * B(k, j);
    }
  return C;
}

Mat transpose(const Mat& A) {
  Mat T(A.c, A.r);
  for (int i = 0; i < A.r; ++i)
    for (int j = 0; j < A.c; ++j) T(j, i) = A(i, j);
  return T;
}

// Inverse by partial-pivot LU (what Eigen's fixed-size inverse() uses for
// sizes > 4, linear_impl:160-161 / qcqp_impl:299).
bool lu_inverse(const Mat& A, Mat* out) {
  const int n = A.r;
  Mat LU = A;
  std::vector<int> piv(n);
  for (int i = 0; i < n; ++i) piv[i] = i;
  for (int k = 0; k < n; ++k) {
    int p = k;
    double best = std::fabs(LU(k, k));
    for (int i = k + 1; i < n; ++i)
      if (std::fabs(LU(i, k)) > best) best = std::fabs(LU(i, k)), p = i;
    if (best == 0.0) return false;
    if (p != k) {
      for (int j = 0; j < n; ++j) std::swap(LU(k, j), LU(p, j));
      std::swap(piv[k], piv[p]);
    }
    for (int i = k + 1; i < n; ++i) {
      LU(i, k) /= LU(k, k);
      const double l = LU(i, k);
      for (int j = k + 1; j < n; ++j) LU(i, j) -= l * LU(k, j);
    }
  }
  *out = Mat(n, n);
  for (int col = 0; col < n; ++col) {
    std::vector<double> y(n);
    for (int i = 0; i < n; ++i) {
      double s = (piv[i] == col) ? 1.0 : 0.0;
      for (int j = 0; j < i; ++j) s -= LU(i, j) * y[j];
      y[i] = s;
    }
    for (int i = n - 1; i >= 0; --i) {
      double s = y[i];
      for (int j = i + 1; j < n; ++j) s -= LU(i, j) * y[j];
      y[i] = s / LU(i, i);
    }
    for (int i = 0; i < n; ++i) (*out)(i, col) = y[i];
  }
  return true;
}

// Householder QR of a square matrix and solve; stands in for
// Eigen::SparseQR<SparseMatrix, COLAMDOrdering> (linear_impl:364-375).
struct HouseholderQR {
  Mat qr;
  std::vector<double> beta;
  bool ok = true;
  explicit HouseholderQR(const Mat& A) : qr(A), beta(A.c, 0.0) {
    const int m = qr.r, n = qr.c;
    for (int k = 0; k < n && k < m; ++k) {
      double norm = 0.0;
      for (int i = k; i < m; ++i) norm += qr(i, k) * qr(i, k);
      norm = std::sqrt(norm);
      if (norm == 0.0) {
        ok = false;
        beta[k] = 0.0;
        continue;
      }
      const double alpha = qr(k, k) > 0 ? -norm : norm;
      const double v0 = qr(k, k) - alpha;
      // v = [1, qr(k+1:,k)/v0]
      for (int i = k + 1; i < m; ++i) qr(i, k) /= v0;
      beta[k] = -v0 / alpha;
      qr(k, k) = alpha;
      for (int j = k + 1; j < n; ++j) {
        double s = qr(k, j);
        for (int i = k + 1; i < m; ++i) s += qr(i, k) * qr(i, j);
        s *= beta[k];
        qr(k, j) -= s;
        for (int i = k + 1; i < m; ++i) qr(i, j) -= s * qr(i, k);
      }
    }
  }
  std::vector<double> solve(std::vector<double> b) const {
    const int m = qr.r, n = qr.c;
    for (int k = 0; k < n && k < m; ++k) {
      double s = b[k];
      for (int i = k + 1; i < m; ++i) s += qr(i, k) * b[i];
      s *= beta[k];
      b[k] -= s;
      for (int i = k + 1; i < m; ++i) b[i] -= s * qr(i, k);
    }
    std::vector<double> x(n);
    for (int i = n - 1; i >= 0; --i) {
      double s = b[i];
      for (int j = i + 1; j < n; ++j) s -= qr(i, j) * x[j];
      x[i] = s / qr(i, i);
    }
    return x;
  }
};

// Dense Cholesky (lower) in place; false if not positive definite.
bool cholesky(Mat* A) {
  const int n = A->r;
  for (int j = 0; j < n; ++j) {
    double d = (*A)(j, j);
    for (int k = 0; k < j; ++k) d -= (*A)(j, k) * (*A)(j, k);
    if (!(d > 0.0)) return false;
    d = std::sqrt(d);
    (*A)(j, j) = d;
    for (int i = j + 1; i < n; ++i) {
      double s = (*A)(i, j);
      for (int k = 0; k < j; ++k) s -= (*A)(i, k) * (*A)(j, k);
      (*A)(i, j) = s / d;
    }
    for (int k = j + 1; k < n; ++k) (*A)(j, k) = 0.0;
  }
  return true;
}

void cholesky_solve(const Mat& L, std::vector<double>* b) {
  const int n = L.r;
  std::vector<double>& x = *b;
  for (int i = 0; i < n; ++i) {
    double s = x[i];
    for (int k = 0; k < i; ++k) s -= L(i, k) * x[k];
    x[i] = s / L(i, i);
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = x[i];
    for (int k = i + 1; k < n; ++k) s -= L(k, i) * x[k];
    x[i] = s / L(i, i);
  }
}

// ----------------------------------------------------------------------------
// Polynomial base coefficients (polynomial.cpp:145-161, 200-201;
// polynomial.h:45-51: kMaxConvolutionSize = 2*12-2 = 22).
constexpr int kMaxConvolutionSize = 22;

Mat computeBaseCoefficients(int N) {
  Mat base(N, N);
  for (int i = 0; i < N; ++i) base(0, i) = 1.0;
  const int DEG = N - 1;
  int order = DEG;
  for (int n = 1; n < N; ++n) {
    for (int i = DEG - order; i < N; ++i)
      base(n, i) = (order - DEG + i) * base(n - 1, i);
    --order;
  }
  return base;
}

const Mat& baseTable() {
  static const Mat table = computeBaseCoefficients(kMaxConvolutionSize);
  return table;
}

// polynomial.h:201-219.
void baseCoeffsWithTime(int N, int derivative, double t, double* coeffs) {
  const Mat& base = baseTable();
  for (int j = 0; j < N; ++j) coeffs[j] = 0.0;
  coeffs[derivative] = base(derivative, derivative);
  if (std::abs(t) < std::numeric_limits<double>::epsilon()) return;
  double t_power = t;
  for (int j = derivative + 1; j < N; ++j) {
    coeffs[j] = base(derivative, j) * t_power;
    t_power = t_power * t;
  }
}

// linear_impl:557-573.
Mat computeQuadraticCostJacobian(int N, int derivative, double t) {
  const Mat& base = baseTable();
  Mat Q(N, N);
  for (int col = 0; col < N - derivative; ++col) {
    for (int row = 0; row < N - derivative; ++row) {
      const double exponent = (N - 1 - derivative) * 2 + 1 - row - col;
      Q(N - 1 - row, N - 1 - col) = base(derivative, N - 1 - row) *
                                    base(derivative, N - 1 - col) *
                                    std::pow(t, exponent) * 2.0 / exponent;
    }
  }
  return Q;
}

// linear_impl:101-111.
Mat setupMappingMatrix(int N, double T) {
  Mat A(N, N);
  std::vector<double> row(N);
  for (int i = 0; i < N / 2; ++i) {
    baseCoeffsWithTime(N, i, 0.0, row.data());
    for (int j = 0; j < N; ++j) A(i, j) = row[j];
    baseCoeffsWithTime(N, i, T, row.data());
    for (int j = 0; j < N; ++j) A(i + N / 2, j) = row[j];
  }
  return A;
}

// linear_impl:132-169 (Schur complement inverse).
Mat invertMappingMatrix(int N, const Mat& A) {
  const int h = N / 2;
  Mat Ainv(N, N);
  Mat Dblk(h, h), C(h, h);
  std::vector<double> diag_inv(h);
  for (int i = 0; i < h; ++i) diag_inv[i] = 1.0 / A(i, i);
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < h; ++j) {
      C(i, j) = A(h + i, j);
      Dblk(i, j) = A(h + i, h + j);
    }
  Mat Dinv;
  lu_inverse(Dblk, &Dinv);
  for (int i = 0; i < h; ++i) Ainv(i, i) = diag_inv[i];
  // -D^-1 * C * A_inv
  Mat DC = matmul(Dinv, C);
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < h; ++j) {
      Ainv(h + i, j) = -DC(i, j) * diag_inv[j];
      Ainv(h + i, h + j) = Dinv(i, j);
    }
  return Ainv;
}

// ----------------------------------------------------------------------------
// Vertex (vertex.h:42-112) in map form.
struct Vertex {
  int D;
  std::map<int, std::vector<double>> constraints;
  explicit Vertex(int d) : D(d) {}
  bool get(int k, std::vector<double>* v) const {
    auto it = constraints.find(k);
    if (it == constraints.end()) return false;
    *v = it->second;
    return true;
  }
};

std::vector<Vertex> verticesFromDense(int S, int D, int K, const uint8_t* mask,
                                      const double* vals) {
  std::vector<Vertex> vs;
  for (int v = 0; v <= S; ++v) {
    Vertex vx(D);
    for (int k = 0; k < K; ++k) {
      if (!mask[v * K + k]) continue;
      std::vector<double> val(D);
      for (int d = 0; d < D; ++d) val[d] = vals[(static_cast<size_t>(v) * K + k) * D + d];
      vx.constraints[k] = val;
    }
    vs.push_back(vx);
  }
  return vs;
}

// Constraint record (polynomial_optimization_linear.h:288-305).
struct Constraint {
  size_t vertex_idx;
  size_t constraint_idx;
  std::vector<double> value;
  bool operator<(const Constraint& rhs) const {
    if (vertex_idx < rhs.vertex_idx) return true;
    if (rhs.vertex_idx < vertex_idx) return false;
    return constraint_idx < rhs.constraint_idx;
  }
  bool operator==(const Constraint& rhs) const {
    return vertex_idx == rhs.vertex_idx && constraint_idx == rhs.constraint_idx;
  }
};

// ----------------------------------------------------------------------------
// PolynomialOptimization<N> restated with a runtime N
// (polynomial_optimization_linear.h:45-285, linear_impl).
struct LinearProblem {
  int N = 10, D = 3, r = 4;
  int S = 0;
  std::vector<Vertex> vertices;
  std::vector<double> times;
  std::vector<Mat> Q, Ainv;
  Mat M;                                  // constraint_reordering_
  std::vector<std::vector<double>> df, dp;  // per dimension
  int n_all = 0, nf = 0, np = 0;
  std::vector<double> coeffs;  // S x D x N

  // linear_impl:46-99.
  int setupFromVertices(const std::vector<Vertex>& vs,
                        const std::vector<double>& t, int deriv) {
    if (N % 2 != 0 || N < 2 || N > kMaxConvolutionSize) return -1;
    if (deriv < 0 || deriv > N / 2 - 1) return -2;
    r = deriv;
    vertices = vs;
    times = t;
    S = static_cast<int>(vs.size()) - 1;
    if (S < 1 || static_cast<int>(t.size()) != S) return -3;
    for (Vertex& v : vertices) {
      Vertex tmp(D);
      bool valid = true;
      for (auto& kv : v.constraints) {
        if (kv.first > N / 2 - 1)
          valid = false;
        else
          tmp.constraints[kv.first] = kv.second;
      }
      if (!valid) v = tmp;
    }
    int rc = updateSegmentTimes(t);
    if (rc) return rc;
    setupConstraintReorderingMatrix();
    return 0;
  }

  // linear_impl:277-304 (without the unconditional prints of :287-292).
  int updateSegmentTimes(const std::vector<double>& t) {
    if (static_cast<int>(t.size()) != S) return -3;
    times = t;
    Q.assign(S, Mat());
    Ainv.assign(S, Mat());
    for (int i = 0; i < S; ++i) {
      if (!(t[i] > 0)) return -4;
      Q[i] = computeQuadraticCostJacobian(N, r, t[i]);
      Mat A = setupMappingMatrix(N, t[i]);
      Ainv[i] = invertMappingMatrix(N, A);
    }
    return 0;
  }

  // linear_impl:171-252.
  void setupConstraintReorderingMatrix() {
    std::vector<Constraint> all;
    std::set<Constraint> fixed, free_;
    for (int v = 0; v <= S; ++v) {
      const Vertex& vx = vertices[v];
      const int occurrences = (v == 0 || v == S) ? 1 : 2;
      for (int co = 0; co < occurrences; ++co) {
        for (int k = 0; k < N / 2; ++k) {
          Constraint c;
          c.vertex_idx = v;
          c.constraint_idx = k;
          if (vx.get(k, &c.value)) {
            all.push_back(c);
            fixed.insert(c);
          } else {
            c.value.assign(D, 0.0);
            all.push_back(c);
            free_.insert(c);
          }
        }
      }
    }
    n_all = static_cast<int>(all.size());
    nf = static_cast<int>(fixed.size());
    np = static_cast<int>(free_.size());
    M = Mat(n_all, nf + np);
    df.assign(D, std::vector<double>(nf, 0.0));
    dp.assign(D, std::vector<double>(np, 0.0));
    int row = 0;
    for (const Constraint& ca : all) {
      int col = 0;
      for (const Constraint& cf : fixed) {
        if (ca == cf) {
          M(row, col) = 1.0;
          for (int d = 0; d < D; ++d) df[d][col] = cf.value[d];
        }
        ++col;
      }
      for (const Constraint& cp : free_) {
        if (ca == cp) M(row, col) = 1.0;
        ++col;
      }
      ++row;
    }
  }

  // linear_impl:306-335: R = M^T blkdiag(H_i) M, with H_i = A_i^-T Q_i A_i^-1.
  // M has exactly one 1 per row, so the sparse product is the scatter below.
  Mat constructR() const {
    std::vector<int> col_of(n_all, -1);
    for (int i = 0; i < n_all; ++i)
      for (int j = 0; j < nf + np; ++j)
        if (M(i, j) != 0.0) col_of[i] = j;
    Mat R(nf + np, nf + np);
    for (int s = 0; s < S; ++s) {
      Mat H = matmul(matmul(transpose(Ainv[s]), Q[s]), Ainv[s]);
      for (int a = 0; a < N; ++a)
        for (int b = 0; b < N; ++b)
          R(col_of[s * N + a], col_of[s * N + b]) += H(a, b);
    }
    return R;
  }

  // linear_impl:254-275.
  void updateSegmentsFromCompactConstraints() {
    coeffs.assign(static_cast<size_t>(S) * D * N, 0.0);
    const int nall = nf + np;
    for (int d = 0; d < D; ++d) {
      std::vector<double> d_all(nall);
      for (int i = 0; i < nf; ++i) d_all[i] = df[d][i];
      for (int i = 0; i < np; ++i) d_all[nf + i] = dp[d][i];
      for (int s = 0; s < S; ++s) {
        std::vector<double> new_d(N, 0.0);
        for (int a = 0; a < N; ++a)
          for (int j = 0; j < nall; ++j) new_d[a] += M(s * N + a, j) * d_all[j];
        for (int a = 0; a < N; ++a) {
          double c = 0.0;
          for (int b = 0; b < N; ++b) c += Ainv[s](a, b) * new_d[b];
          coeffs[(static_cast<size_t>(s) * D + d) * N + a] = c;
        }
      }
    }
  }

  // linear_impl:337-379 (without the print of :370).
  int solveLinear() {
    if (np == 0) {
      updateSegmentsFromCompactConstraints();
      return 0;
    }
    Mat R = constructR();
    Mat Rpp(np, np), Rpf(np, nf);
    for (int i = 0; i < np; ++i) {
      for (int j = 0; j < nf; ++j) Rpf(i, j) = R(nf + i, j);
      for (int j = 0; j < np; ++j) Rpp(i, j) = R(nf + i, nf + j);
    }
    HouseholderQR qr(Rpp);
    for (int d = 0; d < D; ++d) {
      std::vector<double> rhs(np, 0.0);
      for (int i = 0; i < np; ++i) {
        double s = 0.0;
        for (int j = 0; j < nf; ++j) s += Rpf(i, j) * df[d][j];
        rhs[i] = -s;
      }
      dp[d] = qr.solve(rhs);
    }
    updateSegmentsFromCompactConstraints();
    return qr.ok ? 0 : -5;
  }

  // linear_impl:113-130.
  double computeCost() const {
    double cost = 0.0;
    for (int s = 0; s < S; ++s)
      for (int d = 0; d < D; ++d) {
        const double* c = &coeffs[(static_cast<size_t>(s) * D + d) * N];
        double part = 0.0;
        for (int a = 0; a < N; ++a) {
          double qc = 0.0;
          for (int b = 0; b < N; ++b) qc += Q[s](a, b) * c[b];
          part += c[a] * qc;
        }
        cost += part;
      }
    return 0.5 * cost;
  }

  // getCostAndGradientDerivative's J_d (nonlinear_impl:1537-1606): the full
  // d^T R d over all dimensions with the current (not re-solved) d_p.
  double costDerivativeJd() const {
    Mat R = constructR();
    double J = 0.0;
    for (int d = 0; d < D; ++d) {
      std::vector<double> all(nf + np);
      for (int i = 0; i < nf; ++i) all[i] = df[d][i];
      for (int i = 0; i < np; ++i) all[nf + i] = dp[d][i];
      for (int i = 0; i < nf + np; ++i)
        for (int j = 0; j < nf + np; ++j) J += all[i] * R(i, j) * all[j];
    }
    return J;
  }
};

int setupLinear(int N, int D, int r, int S, int K, const uint8_t* mask,
                const double* vals, const double* times, LinearProblem* lp) {
  if (!mask || !vals || !times || S < 1 || D < 1 || K < 1) return -1;
  lp->N = N;
  lp->D = D;
  std::vector<Vertex> vs = verticesFromDense(S, D, K, mask, vals);
  std::vector<double> t(times, times + S);
  return lp->setupFromVertices(vs, t, r);
}

// ----------------------------------------------------------------------------
// Tube QCQP (PolynomialOptimizationConstrained<N>, qcqp_impl).
int factorial(int n) { return n > 1 ? n * factorial(n - 1) : 1; }  // :791-797
int binomialCoeff(int n, int k) {  // :799-814
  int res = 1;
  if (k > n - k) k = n - k;
  for (int i = 0; i < k; ++i) {
    res *= (n - i);
    res /= (i + 1);
  }
  return res;
}

// qcqp_impl:267-319.
Mat setupInverseControlPointMappingMatrix(int N, double T) {
  const int h = N / 2;
  Mat Bul(h, h);
  Bul(0, 0) = 1;
  const int n = N - 1;
  for (int l = 1; l < h; ++l)
    for (int j = 0; j < h; ++j)
      if (j <= l)
        Bul(l, j) = factorial(n) / factorial(n - l) * std::pow(-1, l + j) /
                    std::pow(T, l) * binomialCoeff(l, j);
  Mat Bul_inv;
  lu_inverse(Bul, &Bul_inv);
  for (int k = 0; k < h; ++k)
    for (int i = 0; i < h; ++i)
      if (Bul_inv(k, i) > -0.00001 && Bul_inv(k, i) < 0.00001) Bul_inv(k, i) = 0;
  Mat Binv(N, N);
  for (int k = 0; k < h; ++k)
    for (int i = 0; i < h; ++i) {
      Binv(k, i) = Bul_inv(k, i);
      // B_lr_inv = rowreverse(B_ul_inv) * diag((-1)^i)
      Binv(h + k, h + i) = Bul_inv(h - 1 - k, i) * std::pow(-1, i);
    }
  return Binv;
}

// One inequality constraint 0.5 x^T quad x + lin x + cst <= 0, stored on its
// support (the free variables it touches).
struct QConstraint {
  std::vector<int> supp;
  std::vector<double> quad;  // |supp|^2
  std::vector<double> lin;   // |supp|
  double cst = 0.0;
};

// Warm-start state of the interior-point method (the device's
// Tube::warm_start): x, s, lam of a trajectory's last usable solve.
struct TubeWarm {
  std::vector<double> x, s, lam;
  bool valid = false;
};

struct TubeProblem {
  LinearProblem lp;  // Q, A^-1, 1-D reordering (qcqp_impl:95-117)
  int N = 10, D = 3, S = 0;
  std::vector<std::pair<double, double>> radii;
  std::vector<Mat> Binv;     // per segment, at setup times (qcqp_impl:152-157)
  int nfk = 0, npk = 0, nak = 0;
  std::vector<int> colk;     // kDim reordering: row -> column
  std::vector<double> dfk;   // fixed_constraints_compact_kDim_
  std::vector<int> col1;     // 1-D reordering rows -> columns
  std::vector<QConstraint> cons;

  // qcqp_impl:121-186 + :18-118.
  int setup(const std::vector<Vertex>& vs, const std::vector<double>& times_cp,
            const std::vector<double>& times, int deriv) {
    N = lp.N;
    D = lp.D;
    if (D != 3) return -10;  // hard-coded D=3 (qcqp_impl:377-384, 777-781)
    S = static_cast<int>(vs.size()) - 1;
    if (static_cast<int>(radii.size()) != S) return -11;
    Binv.clear();
    for (int i = 0; i < S; ++i) {
      if (!(times_cp[i] > 0)) return -4;
      Binv.push_back(setupInverseControlPointMappingMatrix(N, times_cp[i]));
    }
    int rc = lp.setupFromVertices(vs, times, deriv);
    if (rc) return rc;
    // setupConstraintReorderingMatrixkDim (qcqp_impl:18-118).
    const int h = N / 2;
    lp.nf = N;
    nfk = N * D;
    lp.np = (S - 1) * h;
    npk = lp.np * D;
    lp.n_all = N * S;
    nak = D * N * S;
    dfk.assign(nfk, 0.0);
    lp.df.assign(D, std::vector<double>(N, 0.0));
    lp.dp.assign(D, std::vector<double>(lp.np, 0.0));
    for (int ending = 0; ending < 2; ++ending) {
      const int v = ending * S;
      for (int k = 0; k < h; ++k) {
        std::vector<double> val;
        if (!lp.vertices[v].get(k, &val)) return -12;  // reference: UB
        for (int d = 0; d < D; ++d) {
          dfk[ending * h + d * N + k] = val[d];
          lp.df[d][ending * h + k] = val[d];
        }
      }
    }
    colk.assign(nak, -1);
    for (int d = 0; d < D; ++d)
      for (int k = 0; k < 2; ++k) {
        int row = d * (2 * h + (S - 1) * N) + k * (h + (S - 1) * N);
        int col = d * 2 * h + k * h;
        for (int i = 0; i < h; ++i) colk[row++] = col++;
      }
    for (int d = 0; d < D; ++d)
      for (int k = 0; k < S - 1; ++k) {
        int row = d * (2 * h + (S - 1) * N) + k * N + h;
        int col = D * 2 * h + d * (S - 1) * h + k * h;
        for (int i = 0; i < h; ++i) {
          colk[row] = col;
          colk[row + h] = col;
          ++row;
          ++col;
        }
      }
    col1.assign(N * S, -1);
    for (int k = 0; k < 2; ++k) {
      int row = k * (h + (S - 1) * N);
      int col = k * h;
      for (int i = 0; i < h; ++i) col1[row++] = col++;
    }
    for (int k = 0; k < S - 1; ++k) {
      int row = k * N + h;
      int col = 2 * h + k * h;
      for (int i = 0; i < h; ++i) {
        col1[row] = col;
        col1[row + h] = col;
        ++row;
        ++col;
      }
    }
    lp.M = Mat(N * S, N + lp.np);
    for (int i = 0; i < N * S; ++i) lp.M(i, col1[i]) = 1.0;
    return 0;
  }

  // constructRkDim (qcqp_impl:188-221) restricted to the blocks used:
  // P = 2 R_pp, q = (2 d_f^T R_fp)^T (qcqp_impl:497-502).
  void objective(Mat* P, std::vector<double>* q) const {
    Mat R(nfk + npk, nfk + npk);
    for (int s = 0; s < S; ++s) {
      Mat H = matmul(matmul(transpose(lp.Ainv[s]), lp.Q[s]), lp.Ainv[s]);
      for (int d = 0; d < D; ++d) {
        const int start = s * N + d * N * S;
        for (int a = 0; a < N; ++a)
          for (int b = 0; b < N; ++b)
            R(colk[start + a], colk[start + b]) += H(a, b);
      }
    }
    *P = Mat(npk, npk);
    q->assign(npk, 0.0);
    for (int i = 0; i < npk; ++i)
      for (int j = 0; j < npk; ++j) (*P)(i, j) = 2.0 * R(nfk + i, nfk + j);
    for (int j = 0; j < npk; ++j) {
      double s = 0.0;
      for (int i = 0; i < nfk; ++i) s += dfk[i] * R(i, nfk + j);
      (*q)[j] = 2.0 * s;
    }
  }

  // Control point j of segment i as an extraction E (D x (nfk+npk)),
  // E = F_j * B_inv * M_kDim (qcqp_impl:337-349), kept sparse per row.
  void extraction(int i, int j, std::vector<std::vector<double>>* E) const {
    E->assign(D, std::vector<double>(nfk + npk, 0.0));
    for (int k = 0; k < D; ++k)
      for (int m = 0; m < N; ++m) {
        const double b = Binv[i](j, m);
        if (b == 0.0) continue;
        (*E)[k][colk[k * N * S + i * N + m]] += b;
      }
  }

  static QConstraint fromDense(int npk, const std::vector<double>& lin_full,
                               const std::vector<std::vector<double>>* Ep,
                               const double* LL, double quad_scale, double cst,
                               int D) {
    // quad = quad_scale * Ep^T LL Ep (Ep: D x npk), lin = lin_full.
    QConstraint c;
    std::vector<char> touch(npk, 0);
    for (int j = 0; j < npk; ++j) {
      if (lin_full[j] != 0.0) touch[j] = 1;
      if (Ep)
        for (int k = 0; k < D; ++k)
          if ((*Ep)[k][j] != 0.0) touch[j] = 1;
    }
    for (int j = 0; j < npk; ++j)
      if (touch[j]) c.supp.push_back(j);
    const int m = static_cast<int>(c.supp.size());
    c.lin.resize(m);
    for (int a = 0; a < m; ++a) c.lin[a] = lin_full[c.supp[a]];
    c.quad.assign(static_cast<size_t>(m) * m, 0.0);
    if (Ep && quad_scale != 0.0) {
      for (int a = 0; a < m; ++a)
        for (int b = 0; b < m; ++b) {
          double s = 0.0;
          for (int k = 0; k < D; ++k)
            for (int l = 0; l < D; ++l)
              s += (*Ep)[k][c.supp[a]] * LL[k * D + l] * (*Ep)[l][c.supp[b]];
          c.quad[static_cast<size_t>(a) * m + b] = quad_scale * s;
        }
    }
    c.cst = cst;
    return c;
  }

  // setupControlPointConstraints (qcqp_impl:321-474).
  void buildConstraints() {
    cons.clear();
    const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    std::vector<std::vector<double>> E;
    for (int i = 0; i < S; ++i) {
      std::vector<double> p0, p1;
      lp.vertices[i].get(0, &p0);
      lp.vertices[i + 1].get(0, &p1);
      // Fixed part c_f = E_f d_f and free part E_p of a control point.
      auto split = [&](int j, std::vector<double>* cf,
                       std::vector<std::vector<double>>* Ep) {
        extraction(i, j, &E);
        cf->assign(D, 0.0);
        Ep->assign(D, std::vector<double>(npk, 0.0));
        for (int k = 0; k < D; ++k) {
          for (int c = 0; c < nfk; ++c) (*cf)[k] += E[k][c] * dfk[c];
          for (int c = 0; c < npk; ++c) (*Ep)[k][c] = E[k][nfk + c];
        }
      };
      std::vector<double> cf;
      std::vector<std::vector<double>> Ep;
      // compute_sphere_constraints (qcqp_impl:357-365): only the free columns.
      if (i < S - 1) {
        split(N - 1, &cf, &Ep);
        const double r2 = radii[i].second;
        double pp = 0.0;
        for (int k = 0; k < D; ++k) pp += p1[k] * p1[k];
        std::vector<double> lin(npk, 0.0);
        for (int c = 0; c < npk; ++c)
          for (int k = 0; k < D; ++k) lin[c] += -2.0 * p1[k] * Ep[k][c];
        cons.push_back(fromDense(npk, lin, &Ep, I3, 2.0, pp - r2 * r2, D));
      }
      // compute_tube_constraints (qcqp_impl:369-429).
      double n[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
      const double nn = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
      for (int k = 0; k < 3; ++k) n[k] /= nn;
      const double nx = n[0], ny = n[1], nz = n[2];
      const double px = p0[0], py = p0[1], pz = p0[2];
      double A[9] = {1 - std::pow(nx, 2), -nx * ny,          -nx * nz,
                     -nx * ny,            1 - std::pow(ny, 2), -ny * nz,
                     -nx * nz,            -ny * nz,          1 - std::pow(nz, 2)};
      for (int k = 0; k < 9; ++k)
        if (A[k] > -0.000001 && A[k] < 0.000001) A[k] = 0;
      double b[3] = {(std::pow(nx, 2) - 1) * px + nx * ny * py + nx * nz * pz,
                     nx * ny * px + (std::pow(ny, 2) - 1) * py + ny * nz * pz,
                     nx * nz * px + ny * nz * py + (std::pow(nz, 2) - 1) * pz};
      for (int k = 0; k < 3; ++k)
        if (b[k] > -0.000001 && b[k] < 0.000001) b[k] = 0;
      double LL[9], L[3];
      for (int a = 0; a < 3; ++a)
        for (int c = 0; c < 3; ++c) {
          double s = 0.0;
          for (int k = 0; k < 3; ++k) s += A[k * 3 + a] * A[k * 3 + c];
          LL[a * 3 + c] = s;
        }
      for (int c = 0; c < 3; ++c) {
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += b[k] * A[k * 3 + c];
        L[c] = 2.0 * s;
      }
      const double r1 = radii[i].first;
      const double mu = b[0] * b[0] + b[1] * b[1] + b[2] * b[2] - std::pow(r1, 2);
      for (int j = 1; j < N - 1; ++j) {
        split(j, &cf, &Ep);
        // const = cf^T LL cf + L cf + mu; lin = 2 cf^T LL Ep + L Ep;
        // quad = 2 Ep^T LL Ep.
        double cst = mu;
        double LLcf[3];
        for (int a = 0; a < 3; ++a) {
          LLcf[a] = 0.0;
          for (int c = 0; c < 3; ++c) LLcf[a] += LL[a * 3 + c] * cf[c];
        }
        for (int a = 0; a < 3; ++a) cst += cf[a] * LLcf[a] + L[a] * cf[a];
        std::vector<double> lin(npk, 0.0);
        for (int c = 0; c < npk; ++c)
          for (int a = 0; a < 3; ++a)
            lin[c] += (2.0 * LLcf[a] + L[a]) * Ep[a][c];
        cons.push_back(fromDense(npk, lin, &Ep, LL, 2.0, cst, D));
      }
      // compute_tube_end_constraints (qcqp_impl:431-474).
      const double rs = (i == 0) ? radii[0].first : radii[i - 1].second;
      const double re = radii[i].second;
      double ps[3], pe[3];
      for (int k = 0; k < 3; ++k) {
        ps[k] = p0[k] - n[k] * rs;
        pe[k] = p1[k] + n[k] * re;
      }
      for (int k = 0; k < N - 2; ++k) {
        split(k + 1, &cf, &Ep);
        for (int side = 0; side < 2; ++side) {
          const double sgn = side == 0 ? -1.0 : 1.0;  // n_start = -n, n_end = n
          const double* p = side == 0 ? ps : pe;
          double cst = 0.0;
          for (int a = 0; a < 3; ++a) cst += -sgn * n[a] * p[a] + sgn * n[a] * cf[a];
          std::vector<double> lin(npk, 0.0);
          for (int c = 0; c < npk; ++c)
            for (int a = 0; a < 3; ++a) lin[c] += sgn * n[a] * Ep[a][c];
          cons.push_back(fromDense(npk, lin, nullptr, I3, 0.0, cst, D));
        }
      }
    }
  }

  double residual(const QConstraint& c, const std::vector<double>& x) const {
    const int m = static_cast<int>(c.supp.size());
    double g = c.cst;
    for (int a = 0; a < m; ++a) {
      const double xa = x[c.supp[a]];
      g += c.lin[a] * xa;
      double qx = 0.0;
      for (int b = 0; b < m; ++b) qx += c.quad[static_cast<size_t>(a) * m + b] * x[c.supp[b]];
      g += 0.5 * xa * qx;
    }
    return g;
  }

  // qcqp_impl:777-785 -> linear_impl:254-275 with the 1-D reordering.
  void recover(const std::vector<double>& x) {
    for (int d = 0; d < D; ++d)
      for (int i = 0; i < lp.np; ++i) lp.dp[d][i] = x[d * lp.np + i];
    lp.updateSegmentsFromCompactConstraints();
  }

  // Primal-dual interior point (Mehrotra predictor-corrector) for
  //   min 0.5 x^T P x + q^T x  s.t.  g_k(x) <= 0  (convex QCQP),
  // replacing MSK_optimizetrm (qcqp_impl:700-712).  Status 0 converged,
  // 1 iteration cap / stalled, 2 breakdown, 3 near-optimal at a breakdown.
  static constexpr double kComplFloor = 2e-2;
  static constexpr double kKktReg = 1e-10;
  // ws (nullable): with a valid state, start from it (x as it was, s and
  // lam floored at kWarmFloor) instead of the cold start; every usable solve
  // (status 0, 1, 3) stores its final state there.
  static constexpr double kWarmFloor = 1e-2;
  static constexpr double kLamStart = 30.0;
  int solveIPM(double tol, int max_iter, std::vector<double>* xout, int* iters,
               TubeWarm* ws = nullptr) {
    Mat P;
    std::vector<double> q;
    objective(&P, &q);
    const int n = npk;
    const int m = static_cast<int>(cons.size());
    // Start from the unconstrained minimiser P x = -q.
    // Where P is numerically singular (long segments: with T = 20 s a
    // vertex's position barely changes the snap cost, T^-7) the start is the
    // tube axis: every intermediate vertex at its position, its higher
    // derivatives zero (control points on the vertex, strictly inside every
    // tube and sphere).  The device kernel uses the same rule.
    std::vector<double> x(n, 0.0);
    const bool warm = ws && ws->valid && static_cast<int>(ws->x.size()) == n &&
                      static_cast<int>(ws->s.size()) == static_cast<int>(cons.size());
    if (!warm) {
      Mat L = P;
      if (cholesky(&L)) {
        for (int i = 0; i < n; ++i) x[i] = -q[i];
        cholesky_solve(L, &x);
      } else {
        const int h = N / 2;
        for (int d = 0; d < D; ++d)
          for (int v = 1; v < S; ++v) {
            std::vector<double> pv;
            lp.vertices[v].get(0, &pv);
            x[d * (S - 1) * h + (v - 1) * h] = pv[d];
          }
      }
    }
    // Cold start scaled to the problem (round 6): slacks at least the square
    // of the largest vertex coordinate (the constraints' units are squared
    // lengths), multipliers at least 30 |q|_inf (the objective's gradient
    // scale).  Unit slacks and multipliers started the iteration far below
    // both scales: 30.6 -> 21.6 IPM iterations on 400 C3 problems, the same
    // status for every problem of a 432-case sweep over N, S, radii and
    // coordinate scales, converged costs within tolerance.  The device kernel
    // uses the same rule.
    double qnorm = 0.0;
    for (int i = 0; i < n; ++i) qnorm = std::max(qnorm, std::fabs(q[i]));
    double pmax = 1.0;
    for (int v = 0; v <= S; ++v) {
      std::vector<double> pv;
      lp.vertices[v].get(0, &pv);
      for (double c : pv) pmax = std::max(pmax, std::fabs(c));
    }
    const double s_start = pmax * pmax, lam_start = std::max(1.0, kLamStart * qnorm);
    std::vector<double> s(m), lam(m, lam_start), g(m);
    if (warm) {
      x = ws->x;
      for (int k = 0; k < m; ++k) {
        s[k] = std::max(ws->s[k], kWarmFloor);
        lam[k] = std::max(ws->lam[k], kWarmFloor);
      }
    } else {
      for (int k = 0; k < m; ++k) {
        g[k] = residual(cons[k], x);
        s[k] = std::max(-g[k], s_start);
      }
    }
    int it = 0;
    int status = 1;
    std::vector<std::vector<double>> a(m);
    for (it = 0; it < max_iter; ++it) {
      // Gradients a_k = Q_k x + l_k on the support; residuals.
      std::vector<double> rd(n, 0.0);
      for (int i = 0; i < n; ++i) {
        double s2 = q[i];
        for (int j = 0; j < n; ++j) s2 += P(i, j) * x[j];
        rd[i] = s2;
      }
      std::vector<double> rp(m);
      double mu = 0.0;
      for (int k = 0; k < m; ++k) {
        const QConstraint& c = cons[k];
        const int ms = static_cast<int>(c.supp.size());
        a[k].assign(ms, 0.0);
        for (int u = 0; u < ms; ++u) {
          double v = c.lin[u];
          for (int w = 0; w < ms; ++w) v += c.quad[static_cast<size_t>(u) * ms + w] * x[c.supp[w]];
          a[k][u] = v;
          rd[c.supp[u]] += lam[k] * v;
        }
        g[k] = residual(c, x);
        rp[k] = g[k] + s[k];
        mu += s[k] * lam[k];
      }
      mu /= std::max(m, 1);
      double rdn = 0.0, rpn = 0.0;
      for (int i = 0; i < n; ++i) rdn = std::max(rdn, std::fabs(rd[i]));
      for (int k = 0; k < m; ++k) rpn = std::max(rpn, std::fabs(rp[k]));
      if (rdn <= tol * (1.0 + qnorm) && rpn <= tol && mu <= tol) {
        status = 0;
        break;
      }
      // Safeguard: on a breakdown of the KKT factorisation or step, stop at
      // the current iterate and accept it if within 1e3 * tol (status 3,
      // near-optimal), or
      // report it as not converged (status 1, value usable) when it is
      // primal feasible and complementary to 1e3 * tol with the dual
      // residual within 1e5 * tol: with lam_k / s_k ~ 1e12 on the active
      // constraints the dual residual stalls at the KKT solve's accuracy.
      const bool near = rdn <= 1e3 * tol * (1.0 + qnorm) && rpn <= 1e3 * tol && mu <= 1e3 * tol;
      const bool stalled = rdn <= 1e5 * tol * (1.0 + qnorm) && rpn <= 1e3 * tol && mu <= 1e3 * tol;
      const int brk = near ? 3 : (stalled ? 1 : 2);
      // K = P + sum lam_k Q_k + sum (lam_k/s_k) a_k a_k^T.
      Mat Kmat = P;
      for (int k = 0; k < m; ++k) {
        const QConstraint& c = cons[k];
        const int ms = static_cast<int>(c.supp.size());
        const double w = lam[k] / s[k];
        for (int u = 0; u < ms; ++u)
          for (int v = 0; v < ms; ++v)
            Kmat(c.supp[u], c.supp[v]) +=
                lam[k] * c.quad[static_cast<size_t>(u) * ms + v] + w * a[k][u] * a[k][v];
      }
      // A non-positive pivot (lam / s ~ 1e12 on active constraints swamps
      // the rest of K in rounding) away from the optimum (brk == 2) is
      // retried once on K + kKktReg diag(K); the regularised Newton step
      // still converges (to the same optimum), where stopping left 16 % of
      // the points of the time optimiser's box [0.1, 2 T0] without a value.
      // Near the optimum (brk 1 or 3) the iterate is kept, as before: going
      // on regularised only stalls the dual residual to the iteration cap.
      // The device kernel uses the same rule.
      {
        Mat K0 = Kmat;
        if (!cholesky(&Kmat)) {
          if (brk != 2) {
            status = brk;
            break;
          }
          for (int i = 0; i < n; ++i) K0(i, i) += kKktReg * K0(i, i);
          Kmat = K0;
          if (!cholesky(&Kmat)) {
            status = brk;
            break;
          }
        }
      }
      auto direction = [&](const std::vector<double>& rc, std::vector<double>* dx,
                           std::vector<double>* dl, std::vector<double>* ds) {
        std::vector<double> rhs(n);
        for (int i = 0; i < n; ++i) rhs[i] = -rd[i];
        for (int k = 0; k < m; ++k) {
          const QConstraint& c = cons[k];
          const double coef = (lam[k] * rp[k] - rc[k]) / s[k];
          for (size_t u = 0; u < c.supp.size(); ++u) rhs[c.supp[u]] -= a[k][u] * coef;
        }
        cholesky_solve(Kmat, &rhs);
        *dx = rhs;
        dl->resize(m);
        ds->resize(m);
        for (int k = 0; k < m; ++k) {
          const QConstraint& c = cons[k];
          double adx = 0.0;
          for (size_t u = 0; u < c.supp.size(); ++u) adx += a[k][u] * (*dx)[c.supp[u]];
          (*dl)[k] = (lam[k] / s[k]) * (adx + rp[k]) - rc[k] / s[k];
          (*ds)[k] = (-rc[k] - s[k] * (*dl)[k]) / lam[k];
        }
      };
      auto max_step = [&](const std::vector<double>& dl, const std::vector<double>& ds) {
        double alpha = 1.0;
        for (int k = 0; k < m; ++k) {
          if (ds[k] < 0) alpha = std::min(alpha, -s[k] / ds[k]);
          if (dl[k] < 0) alpha = std::min(alpha, -lam[k] / dl[k]);
        }
        return alpha;
      };
      std::vector<double> rc(m), dx, dl, ds;
      for (int k = 0; k < m; ++k) rc[k] = s[k] * lam[k];
      direction(rc, &dx, &dl, &ds);
      const double a_aff = max_step(dl, ds);
      double mu_aff = 0.0;
      for (int k = 0; k < m; ++k)
        mu_aff += (s[k] + a_aff * ds[k]) * (lam[k] + a_aff * dl[k]);
      mu_aff /= std::max(m, 1);
      // Mehrotra's sigma, with the complementarity target kept at or above
      // kComplFloor x the (relative) infeasibility: letting mu run ahead of
      // the dual residual sends lam_k / s_k on the active constraints past
      // 1e12, where the condensed KKT matrix loses its null-space part to
      // rounding and the dual residual stalls (and the factorisation breaks
      // down: 87 of 400 problems stopped that way before).  kComplFloor 1e-2
      // with unit starts (round 5); 2e-2 with the scaled start (round 6):
      // 30.8 -> 22.9 iterations on 4096 C3 problems, every one converged
      // (round 5: two near-optimal stops).  Lower floors save up to two more
      // iterations but stop more problems near-optimal on the device, whose
      // block LDL^T meets the breakdown where this dense Cholesky does not
      // (config 3, device / oracle near-optimal: 1e-2 3 / 3 on different
      // problems, 5e-3 7 / 2, 2e-3 11 / 5; profiles/r06_tube_floor_ab.txt).
      double sigma = std::pow(mu_aff / mu, 3);
      {
        const double infeas = std::max(rdn / (1.0 + qnorm), rpn);
        const double floor_mu = std::min(mu, kComplFloor * infeas);
        if (sigma * mu < floor_mu) sigma = floor_mu / mu;
      }
      for (int k = 0; k < m; ++k) rc[k] = s[k] * lam[k] + ds[k] * dl[k] - sigma * mu;
      direction(rc, &dx, &dl, &ds);
      const double alpha = std::min(1.0, 0.99 * max_step(dl, ds));
      double dxn = 0.0;
      for (int i = 0; i < n; ++i) dxn = std::max(dxn, std::fabs(dx[i]));
      if (!(alpha > 0.0) || !(dxn < 1e300) || !(sigma < 1e300)) {
        status = brk;
        break;
      }
      for (int i = 0; i < n; ++i) x[i] += alpha * dx[i];
      for (int k = 0; k < m; ++k) {
        s[k] += alpha * ds[k];
        lam[k] += alpha * dl[k];
      }
    }
    *xout = x;
    *iters = it;
    if (ws && (status == 0 || status == 1 || status == 3)) {
      ws->x = x;
      ws->s = s;
      ws->lam = lam;
      ws->valid = true;
    }
    return status;
  }
};

int setupTube(int N, int D, int r, int S, int K, const uint8_t* mask,
              const double* vals, const double* times_cp, const double* times,
              const double* radii, TubeProblem* tp) {
  if (!mask || !vals || !times || !times_cp || !radii || S < 1) return -1;
  tp->lp.N = N;
  tp->lp.D = D;
  tp->radii.clear();
  for (int i = 0; i < S; ++i) tp->radii.push_back({radii[2 * i], radii[2 * i + 1]});
  std::vector<Vertex> vs = verticesFromDense(S, D, K, mask, vals);
  for (int v = 0; v <= S; ++v)
    if (!vs[v].constraints.count(0)) return -13;  // tube geometry needs positions
  std::vector<double> tcp(times_cp, times_cp + S), t(times, times + S);
  int rc = tp->setup(vs, tcp, t, r);
  if (rc) return rc;
  tp->buildConstraints();
  return 0;
}

}  // namespace

// ============================================================================
// C ABI
extern "C" {

int orc_base_coefficients(int n, double* out) {
  if (n < 1 || n > kMaxConvolutionSize || !out) return -1;
  const Mat& b = baseTable();
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) out[i * n + j] = b(i, j);
  return 0;
}

int orc_base_coeffs_with_time(int N, int deriv, double t, double* out) {
  if (N < 1 || N > kMaxConvolutionSize || deriv < 0 || deriv >= N || !out) return -1;
  baseCoeffsWithTime(N, deriv, t, out);
  return 0;
}

int orc_segment_matrices(int N, int r, double T, double* Q, double* A,
                         double* Ainv, double* H) {
  if (N < 2 || N % 2 || N > kMaxConvolutionSize || r < 0 || r >= N) return -1;
  Mat q = computeQuadraticCostJacobian(N, r, T);
  Mat a = setupMappingMatrix(N, T);
  Mat ai = invertMappingMatrix(N, a);
  Mat h = matmul(matmul(transpose(ai), q), ai);
  if (Q) std::memcpy(Q, q.a.data(), sizeof(double) * N * N);
  if (A) std::memcpy(A, a.a.data(), sizeof(double) * N * N);
  if (Ainv) std::memcpy(Ainv, ai.a.data(), sizeof(double) * N * N);
  if (H) std::memcpy(H, h.a.data(), sizeof(double) * N * N);
  return 0;
}

// vertex.cpp:27-82.
int orc_random_vertices(int max_deriv, int S, int D, const double* pos_min,
                        const double* pos_max, uint64_t seed, int K,
                        uint8_t* mask, double* vals) {
  if (S < 1 || D < 1 || max_deriv < 1 || K < max_deriv + 1) return -1;
  double span = 0.0;
  for (int d = 0; d < D; ++d) span += (pos_max[d] - pos_min[d]) * (pos_max[d] - pos_min[d]);
  if (std::sqrt(span) < 0.2) return -2;
  std::mt19937 generator(static_cast<std::mt19937::result_type>(seed));
  std::vector<std::uniform_real_distribution<double>> dist(D);
  for (int d = 0; d < D; ++d)
    dist[d] = std::uniform_real_distribution<double>(pos_min[d], pos_max[d]);
  const double min_distance = 0.2;
  std::memset(mask, 0, static_cast<size_t>(S + 1) * K);
  std::memset(vals, 0, sizeof(double) * static_cast<size_t>(S + 1) * K * D);
  std::vector<double> last(D), pos(D);
  for (int d = 0; d < D; ++d) last[d] = dist[d](generator);
  auto setc = [&](int v, int k, const std::vector<double>& val) {
    mask[v * K + k] = 1;
    for (int d = 0; d < D; ++d) vals[(static_cast<size_t>(v) * K + k) * D + d] = val[d];
  };
  // makeStartOrEnd (vertex.cpp:147-153).
  auto start_or_end = [&](int v, const std::vector<double>& p) {
    setc(v, 0, p);
    std::vector<double> zero(D, 0.0);
    for (int i = 1; i <= max_deriv; ++i) setc(v, i, zero);
  };
  start_or_end(0, last);
  for (int v = 1; v <= S; ++v) {
    while (true) {
      for (int d = 0; d < D; ++d) pos[d] = dist[d](generator);
      double dist2 = 0.0;
      for (int d = 0; d < D; ++d) dist2 += (pos[d] - last[d]) * (pos[d] - last[d]);
      if (std::sqrt(dist2) > min_distance) break;
    }
    setc(v, 0, pos);
    last = pos;
  }
  start_or_end(S, last);
  return 0;
}

int orc_estimate_segment_times(int S, int D, const double* positions,
                               double v_max, double a_max, int method,
                               double magic_or_factor, double* times) {
  if (S < 1 || D < 1 || !positions || !times) return -1;
  for (int i = 0; i < S; ++i) {
    double dist2 = 0.0;
    for (int d = 0; d < D; ++d) {
      const double e = positions[(i + 1) * D + d] - positions[i * D + d];
      dist2 += e * e;
    }
    const double distance = std::sqrt(dist2);
    if (method == 0) {  // vertex.cpp:252-269
      times[i] = distance / v_max * 2 *
                 (1.0 + magic_or_factor * v_max / a_max * std::exp(-distance / v_max * 2));
    } else {  // vertex.cpp:271-287 (+ time_factor, :233-250)
      const double acc_time = v_max / a_max;
      const double acc_distance = 0.5 * v_max * acc_time;
      double t;
      if (distance < 2.0 * acc_distance)
        t = 2.0 * std::sqrt(distance / a_max);
      else
        t = 2.0 * acc_time + (distance - 2.0 * acc_distance) / v_max;
      times[i] = t * magic_or_factor;
    }
  }
  return 0;
}

int orc_linear_solve(int N, int D, int r, int S, int K, const uint8_t* mask,
                     const double* vals, const double* times, double* coeffs,
                     double* cost, double* df, double* dp, int* nf, int* np) {
  LinearProblem lp;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times, &lp);
  if (rc) return rc;
  rc = lp.solveLinear();
  if (coeffs) std::memcpy(coeffs, lp.coeffs.data(), sizeof(double) * lp.coeffs.size());
  if (cost) *cost = lp.computeCost();
  if (nf) *nf = lp.nf;
  if (np) *np = lp.np;
  for (int d = 0; d < D; ++d) {
    if (df) std::memcpy(df + static_cast<size_t>(d) * lp.nf, lp.df[d].data(), sizeof(double) * lp.nf);
    if (dp) std::memcpy(dp + static_cast<size_t>(d) * lp.np, lp.dp[d].data(), sizeof(double) * lp.np);
  }
  return rc;
}

int orc_linear_matrices(int N, int D, int r, int S, int K, const uint8_t* mask,
                        const double* vals, const double* times, double* R,
                        double* M, double* A, double* Ainv, double* Mpinv) {
  LinearProblem lp;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times, &lp);
  if (rc) return rc;
  const int nc = lp.nf + lp.np;
  if (R) {
    Mat Rm = lp.constructR();
    std::memcpy(R, Rm.a.data(), sizeof(double) * nc * nc);
  }
  if (M) std::memcpy(M, lp.M.a.data(), sizeof(double) * lp.n_all * nc);
  const int NS = N * S;
  if (A || Ainv) {
    if (A) std::memset(A, 0, sizeof(double) * NS * NS);
    if (Ainv) std::memset(Ainv, 0, sizeof(double) * NS * NS);
    for (int s = 0; s < S; ++s) {
      Mat a = setupMappingMatrix(N, lp.times[s]);
      for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
          if (A) A[(s * N + i) * NS + s * N + j] = a(i, j);
          if (Ainv) Ainv[(s * N + i) * NS + s * N + j] = lp.Ainv[s](i, j);
        }
    }
  }
  if (Mpinv) {  // linear_impl:546-555
    Mat Mt = transpose(lp.M);
    for (int i = 0; i < Mt.r; ++i) {
      double sum = 0.0;
      for (int j = 0; j < Mt.c; ++j) sum += Mt(i, j);
      for (int j = 0; j < Mt.c; ++j) Mt(i, j) /= sum;
    }
    std::memcpy(Mpinv, Mt.a.data(), sizeof(double) * nc * lp.n_all);
  }
  return 0;
}

// Soft-constraint part of objectiveFunctionTime (nonlinear_impl:907-913).
struct SoftSpec {
  int n;
  const int* derivatives;
  const double* limits;
  double weight, maximum_cost;
  bool hard = false;       // use_soft_constraints = false: inequality constraints
  double tolerance = 0.0;  // inequality_constraint_tolerance
};

static int timeCostImpl(int N, int D, int r, int S, int K, const uint8_t* mask,
                        const double* vals, const double* times, double time_penalty,
                        int grad_mode, double increment, double w_d, double w_t,
                        const SoftSpec* soft, double* cost, double* grad) {
  LinearProblem lp;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times, &lp);
  if (rc) return rc;
  auto objective = [&](LinearProblem& p, const std::vector<double>& t) {
    p.updateSegmentTimes(t);
    p.solveLinear();
    double total = 0.0;
    for (double v : t) total += v;  // nonlinear_impl:2768-2774
    double J = p.computeCost() + total * total * time_penalty;
    if (soft && soft->n > 0) {
      double c = 0.0;
      orc_soft_constraint_cost(N, D, S, p.coeffs.data(), t.data(), soft->n, soft->derivatives,
                               soft->limits, soft->weight, soft->maximum_cost, nullptr, &c);
      J += c;
    }
    return J;
  };

  std::vector<double> t(times, times + S);
  const double J = objective(lp, t);
  if (cost) *cost = J;
  if (grad_mode == 0 || !grad) return 0;
  if (grad_mode == 1) {
    // nonlinear_impl:2515-2574: d_p held at the solution for t.
    for (int n = 0; n < S; ++n) {
      std::vector<double> ts = t, tb = t;
      ts[n] = ts[n] <= 0.1 ? 0.1 : ts[n] - increment;
      tb[n] = tb[n] <= 0.1 ? 0.1 : tb[n] + increment;
      lp.updateSegmentTimes(ts);
      const double Js = lp.costDerivativeJd();
      lp.updateSegmentTimes(tb);
      const double Jb = lp.costDerivativeJd();
      grad[n] = w_d * (Jb - Js) / (2.0 * increment) + w_t * 1.0;
    }
    lp.updateSegmentTimes(t);
    return 0;
  }
  // grad_mode 2: central differences of the re-solved objective.
  for (int n = 0; n < S; ++n) {
    std::vector<double> ts = t, tb = t;
    ts[n] = ts[n] <= 0.1 ? 0.1 : ts[n] - increment;
    tb[n] = tb[n] <= 0.1 ? 0.1 : tb[n] + increment;
    LinearProblem p2 = lp;
    const double Js = objective(p2, ts);
    const double Jb = objective(p2, tb);
    grad[n] = (Jb - Js) / (2.0 * increment);
  }
  return 0;
}

int orc_time_cost(int N, int D, int r, int S, int K, const uint8_t* mask,
                  const double* vals, const double* times, double time_penalty,
                  int grad_mode, double increment, double w_d, double w_t,
                  double* cost, double* grad) {
  return timeCostImpl(N, D, r, S, K, mask, vals, times, time_penalty, grad_mode, increment,
                      w_d, w_t, nullptr, cost, grad);
}

int orc_time_cost_soft(int N, int D, int r, int S, int K, const uint8_t* mask,
                       const double* vals, const double* times, double time_penalty,
                       int grad_mode, double increment, double w_d, double w_t, int n_soft,
                       const int* soft_derivatives, const double* soft_limits,
                       double soft_weight, double soft_maximum_cost, double* cost,
                       double* grad) {
  const SoftSpec soft{n_soft, soft_derivatives, soft_limits, soft_weight, soft_maximum_cost};
  return timeCostImpl(N, D, r, S, K, mask, vals, times, time_penalty, grad_mode, increment,
                      w_d, w_t, &soft, cost, grad);
}

// Polynomial::evaluate (polynomial.h:135-149): Horner with the derivative
// row of the base table.
static double polyEvaluate(int N, const double* c, double t, int derivative) {
  if (derivative >= N) return 0.0;
  const Mat& base = baseTable();
  const int tmp = N - 1;
  double result = base(derivative, tmp) * c[tmp];
  for (int i = tmp - 1; i >= derivative; --i) {
    result *= t;
    result += base(derivative, i) * c[i];
  }
  return result;
}

// Trajectory::evaluateRange (trajectory.cpp:74-134), statement by statement.
int orc_evaluate_range(int N, int D, int S, const double* coeffs, const double* times,
                       double t_start, double t_end, double dt, int derivative,
                       int max_out, double* out, double* times_out, int* count) {
  if (N < 1 || D < 1 || S < 1 || !coeffs || !times || !count) return -2;
  *count = 0;
  double accumulated_time = 0.0;
  int i = 0;
  for (i = 0; i < S; ++i) {
    accumulated_time += times[i];
    if (accumulated_time > t_start) break;
  }
  if (t_start > accumulated_time) return -1;
  if (i >= S) i = S - 1;  // (the reference indexes past the end here)
  accumulated_time -= times[i];
  double time_in_segment = t_start - accumulated_time;
  int n = 0;
  while (accumulated_time < t_end) {
    if (time_in_segment > times[i]) {
      time_in_segment = time_in_segment - times[i];
      i++;
      if (i >= S) break;
      continue;
    }
    if (n < max_out) {
      for (int d = 0; d < D; ++d)
        out[static_cast<size_t>(n) * D + d] =
            polyEvaluate(N, coeffs + (static_cast<size_t>(i) * D + d) * N, time_in_segment,
                         derivative);
      if (times_out) times_out[n] = accumulated_time;
    }
    ++n;
    time_in_segment += dt;
    accumulated_time += dt;
  }
  *count = n;
  return 0;
}

// ----------------------------------------------------------------------------
// Magnitude extrema.
//
// The reference finds all complex roots with Jenkins-Traub
// (findRootsJenkinsTraub, src/rpoly/rpoly_ak1.cpp:70-117; the TOMS-493
// translation needs Eigen and cannot be built here).  The
// oracle computes the same roots as the eigenvalues of the companion matrix
// (balancing + Francis double-shift QR on the Hessenberg form, as
// numpy.roots / LAPACK dgeev do); real roots come out with an imaginary part
// of exactly 0 in both, which is what selectMinMaxCandidatesFromRoots
// (polynomial.cpp:32-63) filters on.

// Balancing of a general matrix (radix 2; Parlett-Reinsch), in place.
static void balanceMatrix(std::vector<double>& a, int n) {
  const double radix = 2.0, sqrdx = radix * radix;
  bool done = false;
  while (!done) {
    done = true;
    for (int i = 0; i < n; ++i) {
      double r = 0.0, c = 0.0;
      for (int j = 0; j < n; ++j)
        if (j != i) {
          c += std::fabs(a[j * n + i]);
          r += std::fabs(a[i * n + j]);
        }
      if (c != 0.0 && r != 0.0) {
        double g = r / radix, f = 1.0;
        const double s0 = c + r;
        while (c < g) {
          f *= radix;
          c *= sqrdx;
        }
        g = r * radix;
        while (c > g) {
          f /= radix;
          c /= sqrdx;
        }
        if ((c + r) / f < 0.95 * s0) {
          done = false;
          g = 1.0 / f;
          for (int j = 0; j < n; ++j) a[i * n + j] *= g;
          for (int j = 0; j < n; ++j) a[j * n + i] *= f;
        }
      }
    }
  }
}

// Eigenvalues of an upper Hessenberg matrix by the Francis double-shift QR
// iteration (EISPACK hqr).  Returns false if an eigenvalue did not converge
// in 60 iterations.
static bool hessenbergEigenvalues(std::vector<double>& A, int n, std::vector<double>* wr,
                                  std::vector<double>* wi) {
  auto a = [&](int i, int j) -> double& { return A[i * n + j]; };
  wr->assign(n, 0.0);
  wi->assign(n, 0.0);
  double anorm = 0.0;
  for (int i = 0; i < n; ++i)
    for (int j = std::max(i - 1, 0); j < n; ++j) anorm += std::fabs(a(i, j));
  int nn = n - 1;
  double t = 0.0;
  double p = 0.0, q = 0.0, r = 0.0, s = 0.0, w = 0.0, x = 0.0, y = 0.0, z = 0.0;
  while (nn >= 0) {
    int its = 0, l = 0;
    do {
      for (l = nn; l >= 1; --l) {
        s = std::fabs(a(l - 1, l - 1)) + std::fabs(a(l, l));
        if (s == 0.0) s = anorm;
        if (std::fabs(a(l, l - 1)) + s == s) {
          a(l, l - 1) = 0.0;
          break;
        }
      }
      x = a(nn, nn);
      if (l == nn) {  // one root
        (*wr)[nn] = x + t;
        (*wi)[nn] = 0.0;
        --nn;
      } else {
        y = a(nn - 1, nn - 1);
        w = a(nn, nn - 1) * a(nn - 1, nn);
        if (l == nn - 1) {  // two roots
          p = 0.5 * (y - x);
          q = p * p + w;
          z = std::sqrt(std::fabs(q));
          x += t;
          if (q >= 0.0) {
            z = p + (p >= 0.0 ? std::fabs(z) : -std::fabs(z));
            (*wr)[nn - 1] = (*wr)[nn] = x + z;
            if (z != 0.0) (*wr)[nn] = x - w / z;
            (*wi)[nn - 1] = (*wi)[nn] = 0.0;
          } else {
            (*wr)[nn - 1] = (*wr)[nn] = x + p;
            (*wi)[nn - 1] = -z;
            (*wi)[nn] = z;
          }
          nn -= 2;
        } else {
          if (its == 60) return false;
          if (its == 10 || its == 20) {  // exceptional shift
            t += x;
            for (int i = 0; i <= nn; ++i) a(i, i) -= x;
            s = std::fabs(a(nn, nn - 1)) + std::fabs(a(nn - 1, nn - 2));
            y = x = 0.75 * s;
            w = -0.4375 * s * s;
          }
          ++its;
          int m = nn - 2;
          for (; m >= l; --m) {
            z = a(m, m);
            r = x - z;
            s = y - z;
            p = (r * s - w) / a(m + 1, m) + a(m, m + 1);
            q = a(m + 1, m + 1) - z - r - s;
            r = a(m + 2, m + 1);
            s = std::fabs(p) + std::fabs(q) + std::fabs(r);
            p /= s;
            q /= s;
            r /= s;
            if (m == l) break;
            const double u = std::fabs(a(m, m - 1)) * (std::fabs(q) + std::fabs(r));
            const double v =
                std::fabs(p) * (std::fabs(a(m - 1, m - 1)) + std::fabs(z) + std::fabs(a(m + 1, m + 1)));
            if (u + v == v) break;
          }
          for (int i = m + 2; i <= nn; ++i) {
            a(i, i - 2) = 0.0;
            if (i != m + 2) a(i, i - 3) = 0.0;
          }
          for (int k = m; k <= nn - 1; ++k) {
            if (k != m) {
              p = a(k, k - 1);
              q = a(k + 1, k - 1);
              r = 0.0;
              if (k != nn - 1) r = a(k + 2, k - 1);
              if ((x = std::fabs(p) + std::fabs(q) + std::fabs(r)) != 0.0) {
                p /= x;
                q /= x;
                r /= x;
              }
            }
            const double nrm = std::sqrt(p * p + q * q + r * r);
            if ((s = (p >= 0.0 ? nrm : -nrm)) != 0.0) {
              if (k == m) {
                if (l != m) a(k, k - 1) = -a(k, k - 1);
              } else {
                a(k, k - 1) = -s * x;
              }
              p += s;
              x = p / s;
              y = q / s;
              z = r / s;
              q /= p;
              r /= p;
              for (int j = k; j <= nn; ++j) {
                p = a(k, j) + q * a(k + 1, j);
                if (k != nn - 1) {
                  p += r * a(k + 2, j);
                  a(k + 2, j) -= p * z;
                }
                a(k + 1, j) -= p * y;
                a(k, j) -= p * x;
              }
              const int mmin = nn < k + 3 ? nn : k + 3;
              for (int i = l; i <= mmin; ++i) {
                p = x * a(i, k) + y * a(i, k + 1);
                if (k != nn - 1) {
                  p += z * a(i, k + 2);
                  a(i, k + 2) -= p * r;
                }
                a(i, k + 1) -= p * q;
                a(i, k) -= p;
              }
            }
          }
        }
      }
    } while (nn >= 0 && l < nn - 1);
  }
  return true;
}

// findRootsJenkinsTraub's contract (rpoly_ak1.cpp:70-117): coefficients in
// increasing order; trailing (highest-order) coefficients below DBL_MIN are
// dropped; constant or zero polynomials have no roots.  Roots at the origin
// are split off exactly, as rpoly does.
static bool findRoots(const std::vector<double>& inc, std::vector<double>* re,
                      std::vector<double>* im) {
  re->clear();
  im->clear();
  int last = -1;
  for (int i = static_cast<int>(inc.size()) - 1; i >= 0; --i)
    if (std::fabs(inc[i]) >= std::numeric_limits<double>::min()) {
      last = i;
      break;
    }
  if (last < 1) return last == 0 ? false : true;
  int lo = 0;
  while (inc[lo] == 0.0) {  // zero roots
    re->push_back(0.0);
    im->push_back(0.0);
    ++lo;
  }
  const int n = last - lo;
  if (n == 0) return true;
  std::vector<double> C(static_cast<size_t>(n) * n, 0.0);
  for (int j = 0; j < n; ++j) C[j] = -inc[last - 1 - j] / inc[last];  // first row
  for (int i = 1; i < n; ++i) C[i * n + i - 1] = 1.0;
  balanceMatrix(C, n);
  std::vector<double> wr, wi;
  if (!hessenbergEigenvalues(C, n, &wr, &wi)) return false;
  for (int i = 0; i < n; ++i) {
    re->push_back(wr[i]);
    im->push_back(wi[i]);
  }
  return true;
}

// Polynomial::getCoefficients(derivative) (polynomial.h:113-127): the
// derivative's coefficients, index 0 = t^0, zero-padded to N.
static std::vector<double> derivCoefficients(int N, const double* c, int derivative) {
  const Mat& base = baseTable();
  std::vector<double> out(N, 0.0);
  for (int i = derivative; i < N; ++i) out[i - derivative] = base(derivative, i) * c[i];
  return out;
}

// Polynomial::convolve (polynomial.cpp:163-181).
static std::vector<double> convolveCoefficients(const std::vector<double>& data,
                                                const std::vector<double>& kernel) {
  const int nd = static_cast<int>(data.size()), nk = static_cast<int>(kernel.size());
  std::vector<double> out(nd + nk - 1, 0.0);
  for (int i = 0; i < nd + nk - 1; ++i) {
    const int data_idx = i - nk + 1;
    const int lower = std::max(0, -data_idx), upper = std::min(nk, nd - data_idx);
    for (int k = lower; k < upper; ++k) out[i] += kernel[nk - 1 - k] * data[data_idx + k];
  }
  return out;
}

// Segment::computeMinMaxMagnitudeCandidateTimes (segment.cpp:82-133) +
// Polynomial::computeMinMaxCandidates (polynomial.cpp:65-81) for all D
// dimensions (linear_impl:395-409).  Appends to *cand.
static void magnitudeCandidateTimes(int N, int D, const double* seg, int derivative,
                                    double t_start, double t_end, std::vector<double>* cand) {
  std::vector<double> f;
  if (D > 1) {
    const int n_d = N - derivative, n_dd = n_d - 1;
    f.assign(n_d + n_dd - 1, 0.0);
    for (int d = 0; d < D; ++d) {
      std::vector<double> dv = derivCoefficients(N, seg + d * N, derivative);
      std::vector<double> ddv = derivCoefficients(N, seg + d * N, derivative + 1);
      dv.resize(n_d);
      ddv.resize(n_dd);
      const std::vector<double> c = convolveCoefficients(dv, ddv);
      for (size_t i = 0; i < f.size(); ++i) f[i] += c[i];
    }
  } else {
    f = derivCoefficients(N, seg, derivative + 1);
  }
  std::vector<double> re, im;
  findRoots(f, &re, &im);
  cand->push_back(t_start);  // selectMinMaxCandidatesFromRoots :44-45
  cand->push_back(t_end);
  for (size_t i = 0; i < re.size(); ++i) {
    if (std::fabs(im[i]) > std::numeric_limits<double>::epsilon()) continue;
    if (re[i] < t_start || re[i] > t_end) continue;
    cand->push_back(re[i]);
  }
}

static double magnitudeAt(int N, int D, const double* seg, double t, int derivative) {
  double sq = 0.0;
  for (int d = 0; d < D; ++d) {
    const double v = polyEvaluate(N, seg + d * N, t, derivative);
    sq += v * v;
  }
  return std::sqrt(sq);
}

// PolynomialOptimization::computeMaximumOfMagnitude (linear_impl:455-487) on
// a trajectory's coefficients (S x D x N).  n_candidates (optional) receives
// the number of candidates the reference would list.
int orc_max_magnitude(int N, int D, int S, const double* coeffs, const double* times,
                      int derivative, double* time, double* value, int* segment,
                      int* n_candidates) {
  if (N < 2 || D < 1 || S < 1 || !coeffs || !times) return -2;
  if (N - derivative - 1 <= 0 || derivative < 0) return -3;  // linear_impl:400
  double best_t = 0.0, best_v = 0.0;  // Extremum() = {0, 0, 0}
  int best_s = 0, count = 0;
  for (int s = 0; s < S; ++s) {
    const double* seg = coeffs + static_cast<size_t>(s) * D * N;
    std::vector<double> ts;
    ts.push_back(0.0);
    magnitudeCandidateTimes(N, D, seg, derivative, 0.0, times[s], &ts);
    for (double t : ts) {
      const double v = magnitudeAt(N, D, seg, t, derivative);
      if (best_v < v) {
        best_t = t;
        best_v = v;
        best_s = s;
      }
      ++count;
    }
  }
  const double* last = coeffs + static_cast<size_t>(S - 1) * D * N;
  const double v = magnitudeAt(N, D, last, times[S - 1], derivative);
  if (best_v < v) {
    best_t = times[S - 1];
    best_v = v;
    best_s = S - 1;
  }
  ++count;
  if (time) *time = best_t;
  if (value) *value = best_v;
  if (segment) *segment = best_s;
  if (n_candidates) *n_candidates = count;
  return 0;
}

// The candidate lists of computeMaximumOfMagnitude (linear_impl:455-487),
// per segment: Segment::computeMinMaxMagnitudeCandidates (segment.cpp:
// 136-161) = t_start 0, t_end T_s, then the real roots (|Im| <= DBL_EPSILON)
// of the magnitude derivative in [0, T_s] in the root finder's order.
// cand_time / cand_value [S][cap]; n_cand[S] = the list length (entries past
// cap dropped).  Returns 0.
int orc_magnitude_candidates(int N, int D, int S, const double* coeffs, const double* times,
                             int derivative, int cap, double* cand_time, double* cand_value,
                             int* n_cand) {
  if (N < 2 || D < 1 || S < 1 || !coeffs || !times || cap < 0) return -2;
  if (N - derivative - 1 <= 0 || derivative < 0) return -3;
  for (int s = 0; s < S; ++s) {
    const double* seg = coeffs + static_cast<size_t>(s) * D * N;
    std::vector<double> ts;
    if (times[s] >= 0.0) magnitudeCandidateTimes(N, D, seg, derivative, 0.0, times[s], &ts);
    n_cand[s] = static_cast<int>(ts.size());
    for (int k = 0; k < static_cast<int>(ts.size()) && k < cap; ++k) {
      cand_time[s * cap + k] = ts[k];
      cand_value[s * cap + k] = magnitudeAt(N, D, seg, ts[k], derivative);
    }
  }
  return 0;
}

// Real roots of a polynomial (increasing coefficients) by the oracle's root
// finder; re/im hold up to n-1 entries.  Returns the number of roots.
int orc_poly_roots(int n, const double* inc, double* re, double* im) {
  std::vector<double> c(inc, inc + n), r, i;
  if (!findRoots(c, &r, &i)) return -1;
  for (size_t k = 0; k < r.size(); ++k) {
    re[k] = r[k];
    im[k] = i[k];
  }
  return static_cast<int>(r.size());
}

// evaluateMaximumMagnitudeAsSoftConstraint (nonlinear_impl:2735-2766):
// sum over constraints of min(maximum_cost, exp((max - limit) / limit * w)).
int orc_soft_constraint_cost(int N, int D, int S, const double* coeffs, const double* times,
                             int n_constraints, const int* derivatives, const double* limits,
                             double weight, double maximum_cost, double* maxima,
                             double* cost) {
  double total = 0.0;
  for (int c = 0; c < n_constraints; ++c) {
    double value = 0.0;
    int rc = orc_max_magnitude(N, D, S, coeffs, times, derivatives[c], nullptr, &value, nullptr,
                               nullptr);
    if (rc) return rc;
    if (maxima) maxima[c] = value;
    const double abs_violation = value - limits[c];
    const double relative_violation = abs_violation / limits[c];
    total += std::min(maximum_cost, std::exp(relative_violation * weight));
  }
  if (cost) *cost = total;
  return 0;
}

int orc_control_point_map(int N, double T, double* Binv) {
  if (N < 2 || N % 2 || N > 12 || !(T > 0) || !Binv) return -1;
  Mat b = setupInverseControlPointMappingMatrix(N, T);
  std::memcpy(Binv, b.a.data(), sizeof(double) * N * N);
  return 0;
}

int orc_tube_num_constraints(int N, int S) {
  return (S - 1) + S * (N - 2) + 2 * S * (N - 2);
}

int orc_tube_qcqp_assemble(int N, int D, int r, int S, int K,
                           const uint8_t* mask, const double* vals,
                           const double* times_cp, const double* times,
                           const double* radii, double* P, double* q,
                           double* quad, double* lin, double* cst, int* n_free) {
  TubeProblem tp;
  int rc = setupTube(N, D, r, S, K, mask, vals, times_cp, times, radii, &tp);
  if (rc) return rc;
  const int n = tp.npk;
  if (n_free) *n_free = n;
  Mat Pm;
  std::vector<double> qv;
  tp.objective(&Pm, &qv);
  if (P) std::memcpy(P, Pm.a.data(), sizeof(double) * n * n);
  if (q) std::memcpy(q, qv.data(), sizeof(double) * n);
  const int m = static_cast<int>(tp.cons.size());
  for (int k = 0; k < m; ++k) {
    const QConstraint& c = tp.cons[k];
    const int ms = static_cast<int>(c.supp.size());
    if (quad) {
      double* Qk = quad + static_cast<size_t>(k) * n * n;
      std::memset(Qk, 0, sizeof(double) * n * n);
      for (int a = 0; a < ms; ++a)
        for (int b = 0; b < ms; ++b)
          Qk[c.supp[a] * n + c.supp[b]] = c.quad[static_cast<size_t>(a) * ms + b];
    }
    if (lin) {
      double* lk = lin + static_cast<size_t>(k) * n;
      std::memset(lk, 0, sizeof(double) * n);
      for (int a = 0; a < ms; ++a) lk[c.supp[a]] = c.lin[a];
    }
    if (cst) cst[k] = c.cst;
  }
  return 0;
}

int orc_tube_residuals(int N, int D, int r, int S, int K, const uint8_t* mask,
                       const double* vals, const double* times_cp,
                       const double* times, const double* radii,
                       const double* x, double* resid) {
  TubeProblem tp;
  int rc = setupTube(N, D, r, S, K, mask, vals, times_cp, times, radii, &tp);
  if (rc) return rc;
  std::vector<double> xv(x, x + tp.npk);
  for (size_t k = 0; k < tp.cons.size(); ++k) resid[k] = tp.residual(tp.cons[k], xv);
  return 0;
}

static int tubeQcqpSolve(int N, int D, int r, int S, int K, const uint8_t* mask,
                         const double* vals, const double* times_cp, const double* times,
                         const double* radii, double tol, int max_iter, double* x_out,
                         double* coeffs, double* cost, int* iters, TubeWarm* ws);

int orc_tube_qcqp_solve(int N, int D, int r, int S, int K, const uint8_t* mask,
                        const double* vals, const double* times_cp,
                        const double* times, const double* radii, double tol,
                        int max_iter, double* x_out, double* coeffs,
                        double* cost, int* iters) {
  return tubeQcqpSolve(N, D, r, S, K, mask, vals, times_cp, times, radii, tol, max_iter, x_out,
                       coeffs, cost, iters, nullptr);
}

static int tubeQcqpSolve(int N, int D, int r, int S, int K, const uint8_t* mask,
                         const double* vals, const double* times_cp, const double* times,
                         const double* radii, double tol, int max_iter, double* x_out,
                         double* coeffs, double* cost, int* iters, TubeWarm* ws) {
  TubeProblem tp;
  int rc = setupTube(N, D, r, S, K, mask, vals, times_cp, times, radii, &tp);
  if (rc) return rc;
  std::vector<double> x;
  int it = 0;
  int status = tp.solveIPM(tol, max_iter, &x, &it, ws);
  if (status < 0) return status;
  if (status == 2) status = -22;  // numerical breakdown away from the optimum
  tp.recover(x);
  if (x_out) std::memcpy(x_out, x.data(), sizeof(double) * x.size());
  if (coeffs) std::memcpy(coeffs, tp.lp.coeffs.data(), sizeof(double) * tp.lp.coeffs.size());
  if (cost) *cost = tp.lp.computeCost();
  if (iters) *iters = it;
  return status;
}

static int timeOptimizeImpl(int N, int D, int r, int S, int K, const uint8_t* mask,
                            const double* vals, double* times_io, double time_penalty,
                            double increment, int max_evals, const SoftSpec* soft,
                            double* cost, int* evals) {
  LinearProblem lp;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times_io, &lp);
  if (rc) return rc;
  // Violation of the hard constraints at the last objective point:
  // max(0, max_c (computeMaximumOfMagnitude - value - tolerance))
  // (evaluateMaximumMagnitudeConstraint, nonlinear_impl:2687-2733).
  double viol = 0.0;
  auto objective = [&](const std::vector<double>& t) {
    lp.updateSegmentTimes(t);
    lp.solveLinear();
    double total = 0.0;
    for (double v : t) total += v;
    double J = lp.computeCost() + total * total * time_penalty;
    viol = 0.0;
    if (soft && soft->n > 0 && soft->hard) {
      std::vector<double> mx(soft->n);
      orc_soft_constraint_cost(N, D, S, lp.coeffs.data(), t.data(), soft->n, soft->derivatives,
                               soft->limits, soft->weight, soft->maximum_cost, mx.data(),
                               nullptr);
      for (int c = 0; c < soft->n; ++c)
        viol = std::max(viol, mx[c] - soft->limits[c] - soft->tolerance);
    } else if (soft && soft->n > 0) {
      double c = 0.0;
      orc_soft_constraint_cost(N, D, S, lp.coeffs.data(), t.data(), soft->n, soft->derivatives,
                               soft->limits, soft->weight, soft->maximum_cost, nullptr, &c);
      J += c;
    }
    return J;
  };

  // Central differences of J (grad_mode 2 of orc_time_cost) and, for the
  // hard constraints, of the violation at the same points.
  auto gradient = [&](const std::vector<double>& t, std::vector<double>* g,
                      std::vector<double>* gv) {
    for (int n = 0; n < S; ++n) {
      std::vector<double> ts = t, tb = t;
      ts[n] = ts[n] <= 0.1 ? 0.1 : ts[n] - increment;
      tb[n] = tb[n] <= 0.1 ? 0.1 : tb[n] + increment;
      const double Js = objective(ts);
      const double vs = viol;
      const double Jb = objective(tb);
      (*g)[n] = (Jb - Js) / (2.0 * increment);
      (*gv)[n] = (viol - vs) / (2.0 * increment);
    }
  };
  const std::vector<double> T0(times_io, times_io + S);
  std::vector<double> T = T0, g(S), gv(S), trial(S);
  double f = objective(T);
  double fv = viol;
  gradient(T, &g, &gv);
  int n_eval = 1;
  double alpha = 0.1;
  while (n_eval < max_evals && alpha > 1e-9) {
    // From an infeasible incumbent the step descends the violation.
    const std::vector<double>& dir = fv > 0.0 ? gv : g;
    double gmax = 0.0;
    for (int n = 0; n < S; ++n) gmax = std::max(gmax, std::fabs(dir[n] * T0[n]));
    if (!(gmax > 0.0)) break;
    bool same = true;
    for (int n = 0; n < S; ++n) {
      const double x = T[n] - alpha * T0[n] * (dir[n] * T0[n]) / gmax;
      trial[n] = std::min(std::max(x, 0.1), 2.0 * T0[n]);
      same = same && trial[n] == T[n];
    }
    if (same) break;
    const double ft = objective(trial);
    const double vt = viol;
    ++n_eval;
    // Feasibility first (hard constraints; the violation is 0 otherwise).
    if (vt == 0.0 ? (fv > 0.0 || ft < f) : vt < fv) {
      T = trial;
      f = ft;
      fv = vt;
      alpha = std::min(alpha * 1.5, 1.0);
      gradient(T, &g, &gv);
    } else {
      alpha *= 0.5;
    }
  }
  std::memcpy(times_io, T.data(), sizeof(double) * S);
  if (cost) *cost = f;
  if (evals) *evals = n_eval;
  return 0;
}

// optimizeTime (nonlinear_impl:332-397) with the reference's default
// algorithm: LN_SBPLX (orc_sbplx.cpp) on objectiveFunctionTime with the
// linear inner solve, bounds [0.1, 2 T0] (:350-358, 375-378), initial step
// initial_stepsize_rel T0 (:343-346), maxeval = max_iterations (:101),
// ftol_rel = f_rel, ftol_abs = f_abs (:97-98).  times_io: in T0, out the
// best point (NLopt's x); *cost its objective; history (nullable, max_evals
// x S) the evaluated points in order.
int orc_time_optimize_sbplx(int N, int D, int r, int S, int K, const uint8_t* mask,
                            const double* vals, double* times_io, double time_penalty,
                            int max_evals, double f_rel, double f_abs, double step_rel,
                            int n_soft, const int* soft_derivatives, const double* soft_limits,
                            double soft_weight, double soft_maximum_cost, double* cost,
                            int* evals, int* result, double* history) {
  LinearProblem lp;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times_io, &lp);
  if (rc) return rc;
  const SoftSpec soft{n_soft, soft_derivatives, soft_limits, soft_weight, soft_maximum_cost};
  int k = 0;
  auto objective = [&](const double* tp) {
    std::vector<double> t(tp, tp + S);
    if (history && k < max_evals) std::memcpy(history + static_cast<size_t>(k) * S, tp, sizeof(double) * S);
    ++k;
    lp.updateSegmentTimes(t);
    lp.solveLinear();
    double total = 0.0;
    for (double v : t) total += v;  // nonlinear_impl:2768-2774
    double J = lp.computeCost() + total * total * time_penalty;
    if (n_soft > 0) {
      double c = 0.0;
      orc_soft_constraint_cost(N, D, S, lp.coeffs.data(), t.data(), soft.n, soft.derivatives,
                               soft.limits, soft.weight, soft.maximum_cost, nullptr, &c);
      J += c;
    }
    return J;
  };
  std::vector<double> lb(S, 0.1), ub(S), step(S);
  for (int i = 0; i < S; ++i) {
    ub[i] = 2.0 * times_io[i];
    step[i] = step_rel * times_io[i];
  }
  double minf = 0.0;
  int nev = 0;
  const int res = orc_sbplx_run(S, objective, lb.data(), ub.data(), times_io, &minf, step.data(),
                                max_evals, f_rel, f_abs, &nev);
  if (cost) *cost = minf;
  if (evals) *evals = nev;
  if (result) *result = res;
  return 0;
}

int orc_time_optimize(int N, int D, int r, int S, int K, const uint8_t* mask,
                      const double* vals, double* times_io, double time_penalty,
                      double increment, int max_evals, double* cost, int* evals) {
  return timeOptimizeImpl(N, D, r, S, K, mask, vals, times_io, time_penalty, increment,
                          max_evals, nullptr, cost, evals);
}

int orc_time_optimize_hard(int N, int D, int r, int S, int K, const uint8_t* mask,
                           const double* vals, double* times_io, double time_penalty,
                           double increment, int max_evals, int n_con, const int* derivatives,
                           const double* limits, double tolerance, double* cost, int* evals) {
  SoftSpec hard{n_con, derivatives, limits, 100.0, 1.0e12};
  hard.hard = true;
  hard.tolerance = tolerance;
  return timeOptimizeImpl(N, D, r, S, K, mask, vals, times_io, time_penalty, increment,
                          max_evals, &hard, cost, evals);
}

int orc_time_optimize_soft(int N, int D, int r, int S, int K, const uint8_t* mask,
                           const double* vals, double* times_io, double time_penalty,
                           double increment, int max_evals, int n_soft,
                           const int* soft_derivatives, const double* soft_limits,
                           double soft_weight, double soft_maximum_cost, double* cost,
                           int* evals) {
  const SoftSpec soft{n_soft, soft_derivatives, soft_limits, soft_weight, soft_maximum_cost};
  return timeOptimizeImpl(N, D, r, S, K, mask, vals, times_io, time_penalty, increment,
                          max_evals, &soft, cost, evals);
}

// objectiveFunctionTime in the fork's form (nonlinear_impl:877-945):
// updateSegmentTimes + solveQCQP (:891-892) + computeCost + time penalty
// [+ soft]; NaN where the QCQP setup or solve fails (mtg_tube_time_cost).
static double tubeTimeObjective(int N, int D, int r, int S, int K, const uint8_t* mask,
                                const double* vals, const double* times_cp,
                                const double* radii, double tol, int max_iter,
                                double time_penalty, const SoftSpec* soft,
                                const std::vector<double>& t, TubeWarm* ws = nullptr) {
  std::vector<double> coeffs(static_cast<size_t>(S) * D * N);
  double c = 0.0;
  int it = 0;
  const int rc = tubeQcqpSolve(N, D, r, S, K, mask, vals, times_cp, t.data(), radii, tol,
                               max_iter, nullptr, coeffs.data(), &c, &it, ws);
  if (rc < 0) return std::numeric_limits<double>::quiet_NaN();
  double total = 0.0;
  for (double v : t) total += v;  // nonlinear_impl:2768-2774
  double J = c + total * total * time_penalty;
  if (soft && soft->n > 0) {
    double sc = 0.0;
    orc_soft_constraint_cost(N, D, S, coeffs.data(), t.data(), soft->n, soft->derivatives,
                             soft->limits, soft->weight, soft->maximum_cost, nullptr, &sc);
    J += sc;
  }
  return J;
}

// Central differences of the re-solved objective (grad_mode 2 and the
// clamp rule of getCostAndGradientTime, nonlinear_impl:2525-2530).
static void fdTimeGradient(int S, double increment, const std::vector<double>& t,
                           const std::function<double(const std::vector<double>&)>& objective,
                           double* g) {
  for (int n = 0; n < S; ++n) {
    std::vector<double> ts = t, tb = t;
    ts[n] = ts[n] <= 0.1 ? 0.1 : ts[n] - increment;
    tb[n] = tb[n] <= 0.1 ? 0.1 : tb[n] + increment;
    const double Js = objective(ts);
    const double Jb = objective(tb);
    g[n] = (Jb - Js) / (2.0 * increment);
  }
}

int orc_tube_time_cost(int N, int D, int r, int S, int K, const uint8_t* mask,
                       const double* vals, const double* times_cp, const double* times,
                       const double* radii, double tol, int max_iter, double time_penalty,
                       int grad_mode, double increment, int n_soft,
                       const int* soft_derivatives, const double* soft_limits,
                       double soft_weight, double soft_maximum_cost, double* cost,
                       double* grad) {
  if (grad_mode != 0 && grad_mode != 2) return -1;
  const SoftSpec soft{n_soft, soft_derivatives, soft_limits, soft_weight, soft_maximum_cost};
  auto objective = [&](const std::vector<double>& t) {
    return tubeTimeObjective(N, D, r, S, K, mask, vals, times_cp, radii, tol, max_iter,
                             time_penalty, &soft, t);
  };
  const std::vector<double> t(times, times + S);
  if (cost) *cost = objective(t);
  if (grad_mode == 2 && grad) fdTimeGradient(S, increment, t, objective, grad);
  return 0;
}

// optimizeTime in the fork's form with the reference's default LN_SBPLX
// (nonlinear_impl:332-397): NLopt's Subplex (orc_sbplx.cpp) on
// objectiveFunctionTime with solveQCQP() at every evaluation (:891-892),
// control-point maps at the initial times (built once at setup,
// qcqp_impl:152-157), bounds [0.1, 2 T0], initial steps step_rel T0,
// maxeval max_evals, ftol f_rel / f_abs (:95-101).  The initial solveQCQP
// (:342) only stores trajectory_initial_; NLopt's first evaluation solves
// at T0 again, so it is not repeated here.  times_io: in T0, out NLopt's x;
// *cost opt_f; result the nlopt_result code; status the QCQP return at T0
// (0, or the orc_tube_qcqp_solve failure code); history (nullable,
// max_evals x S) the evaluated points in order.
int orc_tube_time_optimize_sbplx(int N, int D, int r, int S, int K, const uint8_t* mask,
                                 const double* vals, const double* radii, double* times_io,
                                 double tol, int max_iter, double time_penalty, int max_evals,
                                 double f_rel, double f_abs, double step_rel, int n_soft,
                                 const int* soft_derivatives, const double* soft_limits,
                                 double soft_weight, double soft_maximum_cost, double* cost,
                                 int* evals, int* result, double* history) {
  const SoftSpec soft{n_soft, soft_derivatives, soft_limits, soft_weight, soft_maximum_cost};
  const std::vector<double> T0(times_io, times_io + S);
  int k = 0;
  // Consecutive evaluations share the constraints (maps at T0): each solve
  // warm-starts from the previous usable one (the device's rule).
  TubeWarm warm;
  auto objective = [&](const double* tp) {
    if (history && k < max_evals)
      std::memcpy(history + static_cast<size_t>(k) * S, tp, sizeof(double) * S);
    ++k;
    const std::vector<double> t(tp, tp + S);
    return tubeTimeObjective(N, D, r, S, K, mask, vals, T0.data(), radii, tol, max_iter,
                             time_penalty, &soft, t, &warm);
  };
  std::vector<double> lb(S, 0.1), ub(S), step(S);
  for (int i = 0; i < S; ++i) {
    ub[i] = 2.0 * T0[i];
    step[i] = step_rel * T0[i];
  }
  double minf = 0.0;
  int nev = 0;
  const int res = orc_sbplx_run(S, objective, lb.data(), ub.data(), times_io, &minf, step.data(),
                                max_evals, f_rel, f_abs, &nev);
  if (cost) *cost = minf;
  if (evals) *evals = nev;
  if (result) *result = res;
  return 0;
}

// mtg_tube_time_optimize's algorithm: timeOptimizeImpl's steps on the QCQP
// objective, control-point maps at the initial times, stopping also at a
// non-finite objective or gradient.
int orc_tube_time_optimize(int N, int D, int r, int S, int K, const uint8_t* mask,
                           const double* vals, const double* radii, double* times_io,
                           double tol, int max_iter, double time_penalty, double increment,
                           int max_evals, int n_soft, const int* soft_derivatives,
                           const double* soft_limits, double soft_weight,
                           double soft_maximum_cost, double* cost, int* evals) {
  const SoftSpec soft{n_soft, soft_derivatives, soft_limits, soft_weight, soft_maximum_cost};
  const std::vector<double> T0(times_io, times_io + S);
  auto objective = [&](const std::vector<double>& t) {
    return tubeTimeObjective(N, D, r, S, K, mask, vals, T0.data(), radii, tol, max_iter,
                             time_penalty, &soft, t);
  };
  std::vector<double> T = T0, g(S), trial(S);
  double f = objective(T);
  int n_eval = 1;
  if (std::isfinite(f)) {
    fdTimeGradient(S, increment, T, objective, g.data());
    double alpha = 0.1;
    while (n_eval < max_evals && alpha > 1e-9) {
      double gmax = 0.0;
      bool finite = true;
      for (int n = 0; n < S; ++n) {
        finite = finite && std::isfinite(g[n]);
        gmax = std::max(gmax, std::fabs(g[n] * T0[n]));
      }
      if (!finite || !(gmax > 0.0)) break;
      bool same = true;
      for (int n = 0; n < S; ++n) {
        const double x = T[n] - alpha * T0[n] * (g[n] * T0[n]) / gmax;
        trial[n] = std::min(std::max(x, 0.1), 2.0 * T0[n]);
        same = same && trial[n] == T[n];
      }
      if (same) break;
      const double ft = objective(trial);
      ++n_eval;
      if (ft < f) {
        T = trial;
        f = ft;
        alpha = std::min(alpha * 1.5, 1.0);
        fdTimeGradient(S, increment, T, objective, g.data());
      } else {
        alpha *= 0.5;
      }
    }
  }
  std::memcpy(times_io, T.data(), sizeof(double) * S);
  if (cost) *cost = f;
  if (evals) *evals = n_eval;
  return 0;
}

int orc_bench_workload(int kind, int N, int D, int r, int S, int K, int B,
                       const uint8_t* masks, const double* vals, const double* times,
                       const double* radii, int param_i, double param_d, int threads,
                       double min_seconds, int64_t* units, double* seconds) {
  if (B < 1 || threads < 1 || !masks || !vals || !times || kind < 1 || kind > 7) return -1;
  if ((kind == 2 || kind == 5 || kind == 7) && !radii) return -1;
  if (kind == 3 && !(param_d > 0.0)) return -1;
  const size_t mstride = static_cast<size_t>(S + 1) * K;
  // kinds 3, 4: coefficients solved before the clock starts.
  std::vector<std::vector<double>> coeffs;
  if (kind >= 3) {
    coeffs.resize(B);
    for (int b = 0; b < B; ++b) {
      LinearProblem lp;
      int rc = setupLinear(N, D, r, S, K, masks + b * mstride, vals + b * mstride * D,
                           times + static_cast<size_t>(b) * S, &lp);
      if (!rc) rc = lp.solveLinear();
      if (rc) return -2;
      coeffs[b] = lp.coeffs;
    }
  }
  std::atomic<int64_t> total(0);
  std::atomic<int> failed(0);
  volatile double sink = 0.0;
  auto t0 = std::chrono::steady_clock::now();
  auto worker = [&](int tid) {
    int64_t n = 0, iters = 0;
    double acc = 0.0;
    std::vector<double> out, tout;
    for (int64_t it = tid;; it += threads) {
      const int b = static_cast<int>(it % B);
      const uint8_t* mk = masks + b * mstride;
      const double* vl = vals + b * mstride * D;
      const double* tb = times + static_cast<size_t>(b) * S;
      if (kind == 1) {
        std::vector<double> t(tb, tb + S);
        double c = 0.0;
        int ev = 0;
        if (orc_time_optimize(N, D, r, S, K, mk, vl, t.data(), 500.0, 0.1, param_i, &c, &ev))
          failed = 1;
        acc += c;
        ++n;
      } else if (kind == 6) {
        // optimizeTime with LN_SBPLX (orc_time_optimize_sbplx), maxeval param_i
        std::vector<double> t(tb, tb + S);
        double c = 0.0;
        int ev = 0, res = 0;
        if (orc_time_optimize_sbplx(N, D, r, S, K, mk, vl, t.data(), 500.0, param_i, 0.05, -1.0,
                                    0.1, 0, nullptr, nullptr, 100.0, 1.0e12, &c, &ev, &res,
                                    nullptr))
          failed = 1;
        acc += c;
        ++n;
      } else if (kind == 7) {
        // optimizeTime in the fork's QCQP form with LN_SBPLX, maxeval param_i
        std::vector<double> t(tb, tb + S);
        double c = 0.0;
        int ev = 0, res = 0;
        if (orc_tube_time_optimize_sbplx(N, D, r, S, K, mk, vl,
                                         radii + static_cast<size_t>(b) * S * 2, t.data(), 1e-10,
                                         100, 500.0, param_i, 0.05, -1.0, 0.1, 0, nullptr,
                                         nullptr, 100.0, 1.0e12, &c, &ev, &res, nullptr))
          failed = 1;
        acc += std::isfinite(c) ? c : 0.0;
        ++n;
      } else if (kind == 2) {
        double c = 0.0;
        int itn = 0;
        const int rc = orc_tube_qcqp_solve(N, D, r, S, K, mk, vl, tb, tb,
                                           radii + static_cast<size_t>(b) * S * 2, 1e-10, 100,
                                           nullptr, nullptr, &c, &itn);
        if (rc < 0 && rc != -22) failed = 1;
        acc += c;
        ++n;
      } else if (kind == 5) {
        // objectiveFunctionTime with the QCQP inner solve and its
        // central-difference gradient (2S + 1 QCQP solves).
        double c = 0.0;
        std::vector<double> g(S);
        if (orc_tube_time_cost(N, D, r, S, K, mk, vl, tb, tb,
                               radii + static_cast<size_t>(b) * S * 2, 1e-10, 100, 500.0, 2, 0.1,
                               0, nullptr, nullptr, 100.0, 1.0e12, &c, g.data()))
          failed = 1;
        acc += std::isfinite(c) ? c : 0.0;
        ++n;
      } else if (kind == 4) {
        const int ders[2] = {1, 2};
        const double lims[2] = {3.0, 5.0};
        double c = 0.0;
        if (orc_soft_constraint_cost(N, D, S, coeffs[b].data(), tb, 2, ders, lims, 100.0, 1.0e12,
                                     nullptr, &c))
          failed = 1;
        acc += c;
        ++n;
      } else {
        double total_t = 0.0;
        for (int i = 0; i < S; ++i) total_t += tb[i];
        const int max_out = static_cast<int>(total_t / param_d) + 8;
        out.resize(static_cast<size_t>(max_out) * D);
        tout.resize(max_out);
        int cnt = 0;
        for (int dv = 0; dv <= param_i; ++dv) {
          if (orc_evaluate_range(N, D, S, coeffs[b].data(), tb, 0.0, total_t, param_d, dv,
                                 max_out, out.data(), tout.data(), &cnt))
            failed = 1;
          acc += out[0];
        }
        n += cnt;
      }
      if ((++iters & 3) == 0) {
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el >= min_seconds) break;
      }
    }
    total += n;
    sink = sink + acc;
  };
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) pool.emplace_back(worker, t);
  for (auto& th : pool) th.join();
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (units) *units = total.load();
  if (seconds) *seconds = el;
  return failed.load() ? -2 : 0;
}

int orc_bench_linear(int N, int D, int r, int S, int K, int B, const uint8_t* masks,
                     const double* vals, const double* times, int threads,
                     double min_seconds, int64_t* solves, double* seconds) {
  if (B < 1 || threads < 1 || !masks || !vals || !times) return -1;
  std::atomic<int64_t> total(0);
  std::atomic<int> failed(0);
  volatile double sink = 0.0;
  const size_t mstride = static_cast<size_t>(S + 1) * K;
  auto t0 = std::chrono::steady_clock::now();
  auto worker = [&](int tid) {
    int64_t n = 0;
    double acc = 0.0;
    for (int64_t it = tid;; it += threads) {
      const int b = static_cast<int>(it % B);
      LinearProblem lp;
      int rc = setupLinear(N, D, r, S, K, masks + b * mstride, vals + b * mstride * D,
                           times + static_cast<size_t>(b) * S, &lp);
      if (!rc) rc = lp.solveLinear();
      if (rc) failed = 1;
      acc += lp.computeCost();
      ++n;
      if ((n & 15) == 0) {
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el >= min_seconds) break;
      }
    }
    total += n;
    sink = sink + acc;
  };
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) pool.emplace_back(worker, t);
  for (auto& th : pool) th.join();
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (solves) *solves = total.load();
  if (seconds) *seconds = el;
  return failed.load() ? -2 : 0;
}


// ----------------------------------------------------------------------------
// Free-derivative objectives.
//
// mode 0: objectiveFunctionFreeConstraints (nonlinear_impl:1021-1113):
//   setFreeConstraints(d_p); J = J_d + [soft], J_d = sum_dim d^T R d from
//   getCostAndGradientDerivative (:1537-1606); gradient (when grad != NULL)
//   = 2 d_f^T R_pf^T + 2 d_p^T R_pp per dimension (:1591-1592), the soft term
//   is not differentiated there (:1100-1110).
// mode 1: objectiveFunctionTimeAndConstraints (:947-1019):
//   updateSegmentTimes(T); setFreeConstraints(d_p);
//   J = computeCost() + time_penalty (sum T)^2 + [soft]; no gradient.
// dp, grad: D x np (dimension-major, the x layout of :1040-1052).
static int freeCostImpl(LinearProblem& lp, const double* dp, int mode, double time_penalty,
                        const SoftSpec* soft, double* cost, double* grad) {
  const int D = lp.D, np = lp.np, nf = lp.nf;
  for (int d = 0; d < D; ++d)
    for (int i = 0; i < np; ++i) lp.dp[d][i] = dp[d * np + i];
  lp.updateSegmentsFromCompactConstraints();
  double J;
  if (mode == 0) {
    J = lp.costDerivativeJd();
    if (grad) {
      Mat R = lp.constructR();
      for (int d = 0; d < D; ++d)
        for (int i = 0; i < np; ++i) {
          double g = 0.0;
          for (int j = 0; j < nf; ++j) g += R(nf + i, j) * lp.df[d][j];
          for (int j = 0; j < np; ++j) g += R(nf + i, nf + j) * lp.dp[d][j];
          grad[d * np + i] = 2.0 * g;
        }
    }
  } else {
    double total = 0.0;
    for (double v : lp.times) total += v;
    J = lp.computeCost() + total * total * time_penalty;
  }
  if (soft && soft->n > 0) {
    double c = 0.0;
    orc_soft_constraint_cost(lp.N, D, lp.S, lp.coeffs.data(), lp.times.data(), soft->n,
                             soft->derivatives, soft->limits, soft->weight, soft->maximum_cost,
                             nullptr, &c);
    J += c;
  }
  if (cost) *cost = J;
  return 0;
}

int orc_free_cost(int N, int D, int r, int S, int K, const uint8_t* mask, const double* vals,
                  const double* times, const double* dp, int mode, double time_penalty,
                  int n_soft, const int* soft_derivatives, const double* soft_limits,
                  double soft_weight, double soft_maximum_cost, double* cost, double* grad) {
  if (!dp || mode < 0 || mode > 1) return -1;
  LinearProblem lp;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times, &lp);
  if (rc) return rc;
  const SoftSpec soft{n_soft, soft_derivatives, soft_limits, soft_weight, soft_maximum_cost};
  return freeCostImpl(lp, dp, mode, time_penalty, n_soft > 0 ? &soft : nullptr, cost,
                      mode == 0 ? grad : nullptr);
}

// The batched optimiser of mtg_free_optimize (free_optimize_kernel) on the
// mode-0 objective: d* = the unconstrained minimiser of J_d (solveLinear,
// linear_impl:337-379) is computed once; then projected steps
// d <- clamp(d + alpha (d* - d), lower, upper) with alpha = 1 initially,
// x1.5 (capped at 1) on a decrease of J, x0.5 otherwise, at most max_evals
// objective evaluations (NLopt maxeval, nonlinear_impl:101).  The direction
// d* - d is the Newton step of the quadratic J_d (its Hessian 2 R_pp is what
// the linear solve factors).  The loop also stops when a trial point moves
// no entry by more than 1e-13 (1 + |d_i|).  lower/upper: D x np or NULL
// (unbounded).
int orc_free_optimize(int N, int D, int r, int S, int K, const uint8_t* mask,
                      const double* vals, const double* times, double* dp_io,
                      const double* lower, const double* upper, int n_soft,
                      const int* soft_derivatives, const double* soft_limits,
                      double soft_weight, double soft_maximum_cost, int max_evals, double* cost,
                      int* evals) {
  if (!dp_io) return -1;
  LinearProblem lp;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times, &lp);
  if (rc) return rc;
  const int np = lp.np, n = D * np;
  if (lp.solveLinear() != 0) return -5;
  std::vector<double> dstar(n), d(dp_io, dp_io + n), trial(n);
  for (int k = 0; k < D; ++k)
    for (int i = 0; i < np; ++i) dstar[k * np + i] = lp.dp[k][i];
  const SoftSpec soft{n_soft, soft_derivatives, soft_limits, soft_weight, soft_maximum_cost};
  auto objective = [&](const std::vector<double>& x) {
    double J = 0.0;
    freeCostImpl(lp, x.data(), 0, 0.0, n_soft > 0 ? &soft : nullptr, &J, nullptr);
    return J;
  };
  double f = objective(d);
  int n_eval = 1;
  double alpha = 1.0;
  while (n_eval < max_evals && alpha > 1e-9) {
    bool same = true;
    for (int i = 0; i < n; ++i) {
      double x = d[i] + alpha * (dstar[i] - d[i]);
      if (lower) x = std::max(x, lower[i]);
      if (upper) x = std::min(x, upper[i]);
      trial[i] = x;
      same = same && std::fabs(x - d[i]) <= 1e-13 * (1.0 + std::fabs(d[i]));
    }
    if (same) break;
    const double ft = objective(trial);
    ++n_eval;
    if (ft < f) {
      d = trial;
      f = ft;
      alpha = std::min(alpha * 1.5, 1.0);
    } else {
      alpha *= 0.5;
    }
  }
  std::memcpy(dp_io, d.data(), sizeof(double) * n);
  if (cost) *cost = f;
  if (evals) *evals = n_eval;
  return 0;
}

// optimizeTimeAndFreeConstraints (nonlinear_impl:610-706) with the
// reference's default LN_SBPLX (orc_sbplx.cpp) over x = [T; d_p] (d_p
// dimension-major, :653-662) on objectiveFunctionTimeAndConstraints
// (:947-1019, freeCostImpl mode 1: no re-solve): bounds T in [0.1, 2 |T0|],
// d_p in [-2 |d0|, 2 |d0|], initial steps step_rel |x0| (:664-675), maxeval
// max_evals, ftol f_rel / f_abs.  NLopt rejects a zero initial step
// (nlopt_set_initial_step) before optimising, which the reference returns as
// nlopt::FAILURE (:681-691): result -1, no evaluation, x unchanged.
// dp_io: D x np, times_io: S; out NLopt's x; history (nullable, max_evals x
// (S + D np)) the evaluated points.
int orc_time_free_optimize_sbplx(int N, int D, int r, int S, int K, const uint8_t* mask,
                                 const double* vals, double* dp_io, double* times_io,
                                 double time_penalty, int n_soft, const int* soft_derivatives,
                                 const double* soft_limits, double soft_weight,
                                 double soft_maximum_cost, int max_evals, double f_rel,
                                 double f_abs, double step_rel, double* cost, int* evals,
                                 int* result, double* history) {
  if (!dp_io || !times_io || max_evals < 1) return -1;
  LinearProblem lp;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times_io, &lp);
  if (rc) return rc;
  const int np = lp.np, n = S + D * np;
  if (np < 1) return -1;
  const SoftSpec soft{n_soft, soft_derivatives, soft_limits, soft_weight, soft_maximum_cost};
  std::vector<double> x(n), lb(n), ub(n), step(n);
  for (int i = 0; i < S; ++i) x[i] = times_io[i];
  for (int i = 0; i < D * np; ++i) x[S + i] = dp_io[i];
  for (int i = 0; i < n; ++i) {
    const double a = std::fabs(x[i]);
    step[i] = step_rel * a;
    lb[i] = i < S ? 0.1 : -2.0 * a;
    ub[i] = 2.0 * a;
  }
  int k = 0;
  std::vector<double> t(S);
  auto objective = [&](const double* xp) {
    if (history && k < max_evals)
      std::memcpy(history + static_cast<size_t>(k) * n, xp, sizeof(double) * n);
    ++k;
    t.assign(xp, xp + S);
    lp.updateSegmentTimes(t);
    double J = 0.0;
    freeCostImpl(lp, xp + S, 1, time_penalty, n_soft > 0 ? &soft : nullptr, &J, nullptr);
    return J;
  };
  double minf = std::numeric_limits<double>::quiet_NaN();
  int nev = 0, res = kSbplxFailure;
  bool zero_step = false;
  for (double v : step) zero_step = zero_step || v == 0.0;
  if (!zero_step)
    res = orc_sbplx_run(n, objective, lb.data(), ub.data(), x.data(), &minf, step.data(),
                        max_evals, f_rel, f_abs, &nev);
  for (int i = 0; i < S; ++i) times_io[i] = x[i];
  for (int i = 0; i < D * np; ++i) dp_io[i] = x[S + i];
  if (cost) *cost = minf;
  if (evals) *evals = nev;
  if (result) *result = res;
  return 0;
}

// The mtg_time_free_optimize algorithm (time_free_optimize_kernel) restated on
// the oracle objective: optimizeTimeAndFreeConstraints (nonlinear_impl:
// 610-706) with objectiveFunctionTimeAndConstraints (:947-1019, mode 1 of
// freeCostImpl), bounds T in [0.1, 2|T0|], d in [-2|d0|, 2|d0|] (:660-677);
// block-alternating projected steps (see include/mtg_hip.h).  dp_io: D x np
// (in d0, out optimised), times_io: S (in T0, out optimised).
int orc_time_free_optimize(int N, int D, int r, int S, int K, const uint8_t* mask,
                           const double* vals, double* dp_io, double* times_io,
                           double time_penalty, double increment, int n_soft,
                           const int* soft_derivatives, const double* soft_limits,
                           double soft_weight, double soft_maximum_cost, int max_evals,
                           double* cost, int* evals) {
  if (!dp_io || !times_io || max_evals < 1) return -1;
  LinearProblem lp;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times_io, &lp);
  if (rc) return rc;
  const int np = lp.np, n = D * np;
  if (np < 1) return -1;
  const SoftSpec soft{n_soft, soft_derivatives, soft_limits, soft_weight, soft_maximum_cost};
  auto objective = [&](const std::vector<double>& t, const std::vector<double>& d) {
    lp.updateSegmentTimes(t);
    double J = 0.0;
    freeCostImpl(lp, d.data(), 1, time_penalty, n_soft > 0 ? &soft : nullptr, &J, nullptr);
    return J;
  };
  const std::vector<double> T0(times_io, times_io + S), d0(dp_io, dp_io + n);
  std::vector<double> T = T0, d = d0, g(S), Ttry(S), dtry(n), dstar(n);
  double f = objective(T, d);
  int n_eval = 1;
  double aT = 0.1, ad = 1.0;
  bool stale = true, dstar_ok = false;
  for (;;) {
    bool moved_round = false;
    if (stale) {
      stale = false;
      for (int k = 0; k < S; ++k) {
        std::vector<double> ts = T, tb = T;
        ts[k] = T[k] <= 0.1 ? 0.1 : T[k] - increment;
        tb[k] = T[k] <= 0.1 ? 0.1 : T[k] + increment;
        const double Js = objective(ts, d);
        const double Jb = objective(tb, d);
        g[k] = (Jb - Js) / (2.0 * increment);
      }
    }
    if (!(n_eval < max_evals)) break;
    if (aT > 1e-9) {  // T block
      double gmax = 0.0;
      for (int k = 0; k < S; ++k) gmax = std::max(gmax, std::fabs(g[k] * T0[k]));
      bool moved = false;
      if (gmax > 0.0)
        for (int k = 0; k < S; ++k) {
          const double x = T[k] - aT * T0[k] * (g[k] * T0[k]) / gmax;
          Ttry[k] = std::min(std::max(x, 0.1), 2.0 * std::fabs(T0[k]));
          moved = moved || Ttry[k] != T[k];
        }
      if (moved) {
        moved_round = true;
        const double ft = objective(Ttry, d);
        ++n_eval;
        if (ft < f) {
          f = ft;
          T = Ttry;
          aT = std::min(aT * 1.5, 1.0);
          stale = true;
          dstar_ok = false;
        } else {
          aT *= 0.5;
        }
      }
    }
    if (!(n_eval < max_evals)) break;
    if (ad > 1e-9) {  // d block
      if (!dstar_ok) {
        lp.updateSegmentTimes(T);
        lp.solveLinear();
        for (int k = 0; k < D; ++k)
          for (int i = 0; i < np; ++i) dstar[k * np + i] = lp.dp[k][i];
        dstar_ok = true;
      }
      bool moved = false;
      for (int i = 0; i < n; ++i) {
        const double bnd = 2.0 * std::fabs(d0[i]);
        double x = d[i] + ad * (dstar[i] - d[i]);
        x = std::min(std::max(x, -bnd), bnd);
        dtry[i] = x;
        moved = moved || std::fabs(x - d[i]) > 1e-13 * (1.0 + std::fabs(d[i]));
      }
      if (moved) {
        moved_round = true;
        const double ft = objective(T, dtry);
        ++n_eval;
        if (ft < f) {
          f = ft;
          d = dtry;
          ad = std::min(ad * 1.5, 1.0);
          stale = true;
        } else {
          ad *= 0.5;
        }
      }
    }
    if (!(n_eval < max_evals) || !moved_round) break;
  }
  std::memcpy(times_io, T.data(), sizeof(double) * S);
  std::memcpy(dp_io, d.data(), sizeof(double) * n);
  if (cost) *cost = f;
  if (evals) *evals = n_eval;
  return 0;
}

// ----------------------------------------------------------------------------
// Collision cost over a dense occupancy grid, restating
// getCostAndGradientCollision (nonlinear_impl:1609-1780) and
// getCostAndGradientPotentialOctree (:1782-1917) with the supereight octree
// replaced by a dense grid (occupied iff value >= 0, :2022-2027):
// findOccupiedVoxels (:1920-2018) keeps the voxels whose unit box overlaps the
// side^3 box at position_voxel - side/2 (supereight aabb_aabb_collision, the
// inclusive half-plane test !((a + a_edge < b) || (b + b_edge < a)));
// getDistanceOctree (:2031-2043) and getCostPotential (:2660-2684) as written.
// Coefficients from d_f and the given d_p (L = A^-1 M, :1650-1656), T and V
// by explicit powers and the derivative map (:1686-1706), eq. (14) gradient
// with T_all L_pp and T_all V_all L_pp (:1729-1747).
namespace {
struct CollMap {
  const float* occ;
  int nx, ny, nz;
  const double* prm;  // res, min[3], max[3], eps, radius, mult, dt
  int side;
  bool occupied(int x, int y, int z) const {
    if (x < 0 || y < 0 || z < 0 || x >= nx || y >= ny || z >= nz) return false;
    return occ[(static_cast<size_t>(z) * ny + y) * nx + x] >= 0.0f;
  }
};

double costPotential(double d, const double* prm, bool* coll) {
  const double eps = prm[7], radius = prm[8], mult = prm[9];
  *coll = false;
  d -= radius;
  if (d <= 0.0) {
    *coll = true;
    return mult * (-d) + 0.5 * eps;
  }
  if (d <= eps) return 0.5 * 1.0 / eps * (d - eps) * (d - eps);
  return 0.0;
}

bool axisOverlap(int a, int a_edge, int b, int b_edge) {
  return !((a + a_edge < b) || (b + b_edge < a));
}

// getCostAndGradientPotentialOctree on the dense map.
double potentialAt(const CollMap& mp, const double pos[3], double grad[3], bool* coll) {
  const double res = mp.prm[0];
  bool valid = true;
  for (int k = 0; k < 3; ++k)
    if (pos[k] < mp.prm[1 + k] + res || pos[k] > mp.prm[4 + k] - res) valid = false;
  int v[3];
  for (int k = 0; k < 3; ++k) v[k] = static_cast<int>(pos[k] / res);
  std::vector<std::array<int, 3>> occupied;
  const int half = mp.side / 2;
  for (int z = v[2] - half - 1; z <= v[2] - half + mp.side; ++z)
    for (int y = v[1] - half - 1; y <= v[1] - half + mp.side; ++y)
      for (int x = v[0] - half - 1; x <= v[0] - half + mp.side; ++x) {
        if (!(axisOverlap(v[0] - half, mp.side, x, 1) && axisOverlap(v[1] - half, mp.side, y, 1) &&
              axisOverlap(v[2] - half, mp.side, z, 1)))
          continue;
        if (mp.occupied(x, y, z)) occupied.push_back({x, y, z});
      }
  auto distance = [&](const int c[3]) {
    double m = std::numeric_limits<double>::max();
    for (const auto& o : occupied) {
      const double dx = o[0] - c[0], dy = o[1] - c[1], dz = o[2] - c[2];
      const double l = std::sqrt(dx * dx + dy * dy + dz * dz);
      if (l < m) m = l;
    }
    return m * res;
  };
  double dist = 0.0;
  if (valid) dist = distance(v);
  const double J = costPotential(dist, mp.prm, coll);

  if (!*coll && grad)
    for (int k = 0; k < 3; ++k) {
      int lo[3] = {v[0], v[1], v[2]}, hi[3] = {v[0], v[1], v[2]};
      lo[k] -= 1;
      hi[k] += 1;
      bool cl, cr;
      const double l = costPotential(valid ? distance(lo) : 0.0, mp.prm, &cl);
      const double r = costPotential(valid ? distance(hi) : 0.0, mp.prm, &cr);
      grad[k] = (r - l) / (2.0 * res);
    }
  return J;
}
}  // namespace

// L = blockdiag(A_s^-1) M (n_all x (nf + np)) at the problem's current times.
static Mat mappingL(const LinearProblem& lp) {
  const int S = lp.S, N = lp.N, nall = lp.nf + lp.np;
  Mat L(S * N, nall);
  for (int s = 0; s < S; ++s)
    for (int a = 0; a < N; ++a)
      for (int j = 0; j < nall; ++j) {
        double v = 0.0;
        for (int b = 0; b < N; ++b) v += lp.Ainv[s](a, b) * lp.M(s * N + b, j);
        L(s * N + a, j) = v;
      }
  return L;
}

// The walk of getCostAndGradientCollision (nonlinear_impl:1609-1780) over
// the problem's coefficients (lp.coeffs) sampled on the segment times `wt`
// (getSegmentTimes, :1646-1647; the time objective's gradient walks the same
// coefficients over perturbed times, :2532-2539).  With L the eq. (14)
// gradient rows accumulate into gc (S x D x N) and gf (D x np).  On a
// collision the walk stops with J_c = 0; the gradients keep what was
// accumulated: the zeroing loop of :1773-1777 iterates over copies
// (`for (Eigen::VectorXd gradients_k : *gradients)`), so it leaves the
// reference's gradient unchanged.
static double collisionWalk(const LinearProblem& lp, const Mat* L, const double* wt,
                            const CollMap& mp, bool* is_coll_out, std::vector<double>* gc,
                            std::vector<double>* gf) {
  const int N = lp.N, D = lp.D, S = lp.S, nf = lp.nf, np = lp.np;
  const double res = mp.prm[0], dt = mp.prm[10];
  double J = 0.0;
  bool is_coll = false;
  double prev[3] = {0, 0, 0}, time_sum = -1.0, dist_sum = 0.0, t = 0.0;
  for (int i = 0; i < S && !is_coll; ++i) {
    for (t = 0.0; t < wt[i]; t += dt) {
      double T[32], pos[3] = {0, 0, 0}, vel[3] = {0, 0, 0};
      for (int n = 0; n < N; ++n) T[n] = std::pow(t, n);
      for (int k = 0; k < D; ++k) {
        const double* c = lp.coeffs.data() + (static_cast<size_t>(i) * D + k) * N;
        for (int n = 0; n < N; ++n) pos[k] += T[n] * c[n];
        for (int n = 0; n + 1 < N; ++n) vel[k] += T[n] * (n + 1) * c[n + 1];  // T V p
      }
      if (time_sum < 0) {
        time_sum = 0.0;
        for (int k = 0; k < 3; ++k) prev[k] = pos[k];
        continue;
      }
      time_sum += dt;
      double dd = 0.0;
      for (int k = 0; k < 3; ++k) dd += (pos[k] - prev[k]) * (pos[k] - prev[k]);
      dist_sum += std::sqrt(dd);
      for (int k = 0; k < 3; ++k) prev[k] = pos[k];
      if (dist_sum < res) continue;
      bool pc = false;
      double gpot[3] = {0, 0, 0};
      const double c = potentialAt(mp, pos, L ? gpot : nullptr, &pc);
      if (pc) {
        is_coll = true;
        break;
      }
      const double vn = std::sqrt(vel[0] * vel[0] + vel[1] * vel[1] + vel[2] * vel[2]);
      J += c * vn * time_sum;
      if (L && vn > 1e-6) {
        // rows T_all L_pp and T_all V_all L_pp of eq. (14)
        std::vector<double> rT(np, 0.0), rV(np, 0.0);
        for (int p2 = 0; p2 < np; ++p2)
          for (int n = 0; n < N; ++n) {
            rT[p2] += T[n] * (*L)(i * N + n, nf + p2);
            if (n + 1 < N) rV[p2] += T[n] * (n + 1) * (*L)(i * N + n + 1, nf + p2);
          }
        for (int k = 0; k < D; ++k) {
          const double a = vn * time_sum * gpot[k], bc = time_sum * c * vel[k] / vn;
          for (int p2 = 0; p2 < np; ++p2) (*gf)[k * np + p2] += a * rT[p2] + bc * rV[p2];
          for (int n = 0; n < N; ++n)
            (*gc)[(static_cast<size_t>(i) * D + k) * N + n] +=
                a * T[n] + bc * (n > 0 ? n * T[n - 1] : 0.0);
        }
      }
      dist_sum = 0.0;
      time_sum = 0.0;
    }
    if (is_coll) break;
    time_sum += -dt + (wt[i] - t);
  }
  if (is_coll) J = 0.0;
  *is_coll_out = is_coll;
  return J;
}

int orc_collision_cost(int N, int D, int r, int S, int K, const uint8_t* mask,
                       const double* vals, const double* times, const double* dp,
                       const float* occupancy, int nx, int ny, int nz, const double* params,
                       int box_side, double* cost, int* collision, double* grad_coeffs,
                       double* grad_free) {
  if (D != 3 || !params) return -1;
  LinearProblem lp;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times, &lp);
  if (rc) return rc;
  const int np = lp.np;
  if (np > 0 && !dp) return -1;
  for (int d = 0; d < D; ++d)
    for (int i = 0; i < np; ++i) lp.dp[d][i] = dp[d * np + i];
  lp.updateSegmentsFromCompactConstraints();
  const Mat L = mappingL(lp);
  const CollMap mp{occupancy, nx, ny, nz, params, box_side};
  std::vector<double> gc(static_cast<size_t>(S) * D * N, 0.0), gf(static_cast<size_t>(D) * np, 0.0);
  bool is_coll = false;
  const double J = collisionWalk(lp, &L, times, mp, &is_coll, &gc, &gf);
  if (cost) *cost = J;
  if (collision) *collision = is_coll ? 1 : 0;
  if (grad_coeffs) std::memcpy(grad_coeffs, gc.data(), sizeof(double) * gc.size());
  if (grad_free) std::memcpy(grad_free, gf.data(), sizeof(double) * gf.size());
  return 0;
}

// ----------------------------------------------------------------------------
// Collision-driven objectives (the reference demo's path, src/main.cpp:77,
// 104-105), restated step by step:
//   mode 0  objectiveFunctionFreeConstraintsAndCollision (nonlinear_impl:
//           1115-1272), x = d_p;
//   mode 1  objectiveFunctionFreeConstraintsAndCollisionAndTime (:1274-1535),
//           x = [T; d_p].
// params (doubles): [0..10] the CollMap layout (res, min[3], max[3], epsilon,
// robot_radius, coll_pot_multiplier, coll_check_time_increment), [11] w_d,
// [12] w_c, [13] w_t, [14] w_sc, [15] add_coll_raise, [16] increment_time,
// [17] soft_constraint_weight, [18] soft maximum_cost, [19] f_rel,
// [20] f_abs, [21] x_rel, [22] x_abs.
// iparams: [0] box side, [1] is_collision_safe, [2] is_coll_raise_first_iter,
// [3] is_simple_numgrad_time, [4] is_simple_numgrad_constraints, [5] n_soft,
// [6] L-BFGS memory.
namespace {
struct CollObjective {
  LinearProblem lp;
  CollMap mp;
  const double* prm;
  const int* ip;
  SoftSpec soft;
  int mode = 0;
  double Jref0 = 0.0;  // total_cost_iter0_{}
  double Jlast = 0.0;  // optimization_info_ totals of the previous evaluation
  bool iter0 = true;

  double softCost() const {
    double c = 0.0;
    orc_soft_constraint_cost(lp.N, lp.D, lp.S, lp.coeffs.data(), lp.times.data(), soft.n,
                             soft.derivatives, soft.limits, soft.weight, soft.maximum_cost,
                             nullptr, &c);
    return c;
  }
  void setFree(const std::vector<double>& dp) {
    for (int d = 0; d < lp.D; ++d)
      for (int i = 0; i < lp.np; ++i) lp.dp[d][i] = dp[d * lp.np + i];
    lp.updateSegmentsFromCompactConstraints();
  }

  // The objective at x; grad (nullable) of length nv; terms[4] = w_d J_d,
  // w_c J_c (raised), w_t J_t, w_sc J_sc.  Returns NaN (no state change)
  // for a non-positive segment time.
  double eval(const std::vector<double>& x, double* grad, double* terms, int* collision) {
    const int S = lp.S, D = lp.D, np = lp.np, nfr = D * np, off = mode ? S : 0;
    const double h = prm[0], inc = prm[16];
    const double w_d = prm[11], w_c = prm[12], w_t = prm[13], w_sc = prm[14];
    if (mode == 1) {  // updateSegmentTimes (:1309)
      std::vector<double> T(x.begin(), x.begin() + S);
      for (double t : T)
        if (!(t > 0.0)) return std::numeric_limits<double>::quiet_NaN();
      lp.updateSegmentTimes(T);
    }
    std::vector<double> dp(x.begin() + off, x.end());
    setFree(dp);  // setFreeConstraints (:1143, 1310)
    const Mat L = mappingL(lp);  // L_ = A^-1 M (:539, 1313-1316)
    std::vector<double> gc(static_cast<size_t>(S) * D * lp.N, 0.0), gf(nfr, 0.0),
        gd(nfr, 0.0), gsc(nfr, 0.0), gt(S, 0.0);
    bool coll = false;
    const double Jc = collisionWalk(lp, grad ? &L : nullptr, lp.times.data(), mp, &coll, &gc, &gf);
    double Jd = 0.0, Jsc = 0.0, Jt = 0.0;
    if (!coll) {
      // getCostAndGradientDerivative (:1537-1606).
      Jd = lp.costDerivativeJd();
      if (grad) {
        const Mat R = lp.constructR();
        const int nf = lp.nf;
        for (int d = 0; d < D; ++d)
          for (int i = 0; i < np; ++i) {
            double a = 0.0, b = 0.0;
            for (int j = 0; j < nf; ++j) a += lp.df[d][j] * R(nf + i, j);
            for (int j = 0; j < np; ++j) b += lp.dp[d][j] * R(nf + j, nf + i);
            gd[d * np + i] = 2.0 * a + 2.0 * b;
          }
      }
      if (soft.n > 0) {
        const bool simple = mode == 1 && ip[4];
        if (simple) {  // getCostAndGradientSoftConstraintsSimple (:2434-2493)
          Jsc = softCost();
          if (grad) {
            for (int i = 0; i < nfr; ++i) {
              std::vector<double> right = dp;
              right[i] = dp[i] + h;
              setFree(right);
              gsc[i] = (softCost() - Jsc) / h;
            }
            setFree(dp);
          }
        } else {  // getCostAndGradientSoftConstraints (:2365-2432)
          if (grad) {
            for (int i = 0; i < nfr; ++i) {
              std::vector<double> left = dp, right = dp;
              left[i] = dp[i] - h;
              right[i] = dp[i] + h;
              setFree(left);
              const double cl = softCost();
              setFree(right);
              const double cr = softCost();
              gsc[i] = (cr - cl) / (2.0 * h);
            }
            setFree(dp);
          }
          Jsc = softCost();
        }
      }
      if (mode == 1) {
        // getCostAndGradientTime(Simple) (:2495-2584, 2586-2657): T_n moved
        // with d held; J_d at the new R, J_c walks the coefficients of T
        // (L_ is not refreshed) over the new times, J_sc reads the segments
        // that updateSegmentTimes leaves unchanged.
        const std::vector<double> T = lp.times;
        const std::vector<double> coeffs = lp.coeffs;
        const bool simple_t = ip[3] != 0;
        auto terms_at = [&](const std::vector<double>& t, double* jd, double* jc, double* jsc) {
          lp.updateSegmentTimes(t);
          *jd = lp.costDerivativeJd();
          bool c2 = false;
          std::vector<double> dummy_c, dummy_f;
          *jc = collisionWalk(lp, nullptr, t.data(), mp, &c2, &dummy_c, &dummy_f);
          // computeMaximumOfMagnitude reads the segments (coefficients and
          // their own times), which updateSegmentTimes leaves at T.
          *jsc = Jsc;
        };
        if (grad) {
          for (int n = 0; n < S; ++n) {
            std::vector<double> big = T;
            big[n] = T[n] <= 0.1 ? 0.1 : T[n] + inc;
            double jd_b, jc_b, jsc_b;
            terms_at(big, &jd_b, &jc_b, &jsc_b);
            double jd_s = Jd, jc_s = Jc, jsc_s = Jsc, den = inc;
            if (!simple_t) {
              std::vector<double> small = T;
              small[n] = T[n] <= 0.1 ? 0.1 : T[n] - inc;
              terms_at(small, &jd_s, &jc_s, &jsc_s);
              den = 2.0 * inc;
            }
            gt[n] = w_d * ((jd_b - jd_s) / den) + w_c * ((jc_b - jc_s) / den) +
                    w_sc * ((jsc_b - jsc_s) / den) + w_t * 1.0;
          }
          lp.updateSegmentTimes(T);
          lp.coeffs = coeffs;
        }
        Jt = 0.0;
        for (double t : T) Jt += t;
      }
    }
    const double ct = w_d * Jd, ctm = w_t * Jt, csc = w_sc * Jsc;
    double cc = w_c * Jc;
    const double total = ct + cc + ctm + csc;
    if (ip[1] && coll) {  // is_collision_safe (:1207-1226, 1432-1452)
      const double ref = ip[2] ? Jref0 : Jlast;
      cc = ref - (total - cc) + prm[15];
    }
    const double J = ct + cc + ctm + csc;
    if (iter0) {
      Jref0 = J;
      iter0 = false;
    }
    Jlast = J;
    if (terms) {
      terms[0] = ct;
      terms[1] = cc;
      terms[2] = ctm;
      terms[3] = csc;
    }
    if (collision) *collision = coll ? 1 : 0;
    if (grad) {
      for (int n = 0; n < off; ++n) grad[n] = gt[n];
      for (int i = 0; i < nfr; ++i) grad[off + i] = w_d * gd[i] + w_c * gf[i] + w_sc * gsc[i];
    }
    return J;
  }
};

int setupCollObjective(int N, int D, int r, int S, int K, const uint8_t* mask, const double* vals,
                       const double* times, int mode, const float* occ, int nx, int ny, int nz,
                       const double* params, const int* iparams, const int* soft_derivatives,
                       const double* soft_limits, CollObjective* o) {
  if (D != 3 || !params || !iparams || (mode != 0 && mode != 1)) return -1;
  int rc = setupLinear(N, D, r, S, K, mask, vals, times, &o->lp);
  if (rc) return rc;
  if (o->lp.np < 1) return -1;
  o->mp = CollMap{occ, nx, ny, nz, params, iparams[0]};
  o->prm = params;
  o->ip = iparams;
  o->mode = mode;
  o->soft = SoftSpec{iparams[5], soft_derivatives, soft_limits, params[17], params[18]};
  return 0;
}

// NLopt's relstop (util/stop.c).
bool relstopOracle(double vold, double vnew, double reltol, double abstol) {
  if (vold == vnew) return true;
  const double d = std::fabs(vnew - vold);
  return d < abstol || d < reltol * (std::fabs(vnew) + std::fabs(vold)) * 0.5;
}
}  // namespace

int orc_coll_cost(int N, int D, int r, int S, int K, const uint8_t* mask, const double* vals,
                  const double* times, int mode, const double* x, const float* occupancy, int nx,
                  int ny, int nz, const double* params, const int* iparams,
                  const int* soft_derivatives, const double* soft_limits, double raise_ref,
                  double* cost, double* grad, double* terms, int* collision) {
  CollObjective o;
  int rc = setupCollObjective(N, D, r, S, K, mask, vals, times, mode, occupancy, nx, ny, nz,
                              params, iparams, soft_derivatives, soft_limits, &o);
  if (rc) return rc;
  if (!x) return -1;
  const int nv = (mode ? S : 0) + D * o.lp.np;
  o.Jref0 = o.Jlast = raise_ref;
  const std::vector<double> xv(x, x + nv);
  const double J = o.eval(xv, grad, terms, collision);
  if (cost) *cost = J;
  return 0;
}

// The mtg_coll_optimize algorithm restated: projected L-BFGS with Armijo
// backtracking by safeguarded quadratic interpolation, every trial one
// counted evaluation (NLopt maxeval), NLopt's ftol / xtol tests on accepted
// steps; it stands in for NLopt's LD_LBFGS (absent; parity unpinned).
int orc_coll_optimize(int N, int D, int r, int S, int K, const uint8_t* mask, const double* vals,
                      const double* times, int mode, const float* occupancy, int nx, int ny,
                      int nz, const double* params, const int* iparams,
                      const int* soft_derivatives, const double* soft_limits,
                      const double* lower, const double* upper, const double* initial_step,
                      int max_evals, double* x_io, double* cost, int* evals, int* result,
                      double* terms) {
  CollObjective o;
  int rc = setupCollObjective(N, D, r, S, K, mask, vals, times, mode, occupancy, nx, ny, nz,
                              params, iparams, soft_derivatives, soft_limits, &o);
  if (rc) return rc;
  if (!x_io || max_evals < 1) return -1;
  const int nv = (mode ? S : 0) + D * o.lp.np;
  const int m = iparams[6];
  if (m < 1 || m > 16) return -1;
  auto lo = [&](int i) { return lower ? lower[i] : -HUGE_VAL; };
  auto hi = [&](int i) { return upper ? upper[i] : HUGE_VAL; };
  std::vector<double> x(nv), g(nv), xt(nv), G(nv), d(nv);
  double step0 = 0.0;
  for (int i = 0; i < nv; ++i) {
    x[i] = std::min(std::max(x_io[i], lo(i)), hi(i));
    step0 = std::max(step0, std::fabs(initial_step ? initial_step[i] : 0.1 * std::fabs(x_io[i])));
  }
  std::vector<std::vector<double>> Sh(m, std::vector<double>(nv)), Yh = Sh;
  std::vector<double> rho(m);
  int cnt = 0, head = 0;
  double best_terms[4] = {NAN, NAN, NAN, NAN}, tt[4];
  auto held = [&](int i) {
    return (x[i] <= lo(i) && g[i] > 0.0) || (x[i] >= hi(i) && g[i] < 0.0);
  };
  // Two-loop recursion on the free variables (see coll direction on the
  // device); returns max |q|.
  auto direction = [&](bool reset) {
    if (reset) cnt = head = 0;
    std::vector<double> q(nv);
    double qmax = 0.0;
    for (int i = 0; i < nv; ++i) {
      q[i] = held(i) ? 0.0 : g[i];
      qmax = std::max(qmax, std::fabs(q[i]));
    }
    if (!(qmax > 0.0)) return qmax;
    std::vector<double> a(m);
    for (int c = 0; c < cnt; ++c) {
      const int k = (head - 1 - c + m) % m;
      double sq = 0.0;
      for (int i = 0; i < nv; ++i) sq += Sh[k][i] * q[i];
      a[c] = rho[k] * sq;
      for (int i = 0; i < nv; ++i) q[i] -= a[c] * Yh[k][i];
    }
    double gamma;
    if (cnt > 0) {
      const int k = (head - 1 + m) % m;
      double sy = 0.0, yy = 0.0;
      for (int i = 0; i < nv; ++i) {
        sy += Sh[k][i] * Yh[k][i];
        yy += Yh[k][i] * Yh[k][i];
      }
      gamma = sy / yy;
    } else {
      gamma = (step0 > 0.0 ? step0 : 1.0) / qmax;
    }
    for (int i = 0; i < nv; ++i) q[i] *= gamma;
    for (int c = cnt - 1; c >= 0; --c) {
      const int k = (head - 1 - c + m) % m;
      double yr = 0.0;
      for (int i = 0; i < nv; ++i) yr += Yh[k][i] * q[i];
      const double beta = rho[k] * yr;
      for (int i = 0; i < nv; ++i) q[i] += (a[c] - beta) * Sh[k][i];
    }
    double gp = 0.0;
    for (int i = 0; i < nv; ++i) {
      d[i] = held(i) ? 0.0 : -q[i];
      gp += g[i] * d[i];
    }
    if (!(gp < 0.0)) {
      cnt = head = 0;
      const double g0 = (step0 > 0.0 ? step0 : 1.0) / qmax;
      for (int i = 0; i < nv; ++i) d[i] = held(i) ? 0.0 : -g0 * g[i];
    }
    return qmax;
  };
  double f = o.eval(x, g.data(), tt, nullptr);
  int n_eval = 1, res = 0;
  double alpha = 1.0;
  if (!std::isfinite(f)) {
    res = -1;
  } else {
    std::copy(tt, tt + 4, best_terms);
    if (!(direction(true) > 0.0)) res = 1;
  }
  while (res == 0) {
    if (n_eval >= max_evals) {
      res = 5;
      break;
    }
    bool moved = false;
    for (int i = 0; i < nv; ++i) {
      xt[i] = std::min(std::max(x[i] + alpha * d[i], lo(i)), hi(i));
      moved = moved || xt[i] != x[i];
    }
    if (!moved) {
      res = 4;
      break;
    }
    const double J = o.eval(xt, G.data(), tt, nullptr);
    ++n_eval;
    double dd = 0.0;
    for (int i = 0; i < nv; ++i) dd += g[i] * (xt[i] - x[i]);
    if (std::isfinite(J) && J < f && J <= f + 1e-4 * dd) {
      double sy = 0.0, ss = 0.0, yy = 0.0;
      bool xstop = true;
      for (int i = 0; i < nv; ++i) {
        const double s2 = xt[i] - x[i], y = G[i] - g[i];
        sy += s2 * y;
        ss += s2 * s2;
        yy += y * y;
        xstop = xstop && relstopOracle(x[i], xt[i], params[21], params[22]);
      }
      const bool fstop = relstopOracle(f, J, params[19], params[20]);
      if (sy > 1e-12 * std::sqrt(ss * yy)) {
        for (int i = 0; i < nv; ++i) {
          Sh[head][i] = xt[i] - x[i];
          Yh[head][i] = G[i] - g[i];
        }
        rho[head] = 1.0 / sy;
        head = (head + 1) % m;
        cnt = std::min(cnt + 1, m);
      }
      x = xt;
      g = G;
      f = J;
      std::copy(tt, tt + 4, best_terms);
      if (fstop) {
        res = 3;
      } else if (xstop) {
        res = 4;
      } else {
        if (!(direction(false) > 0.0)) res = 1;
        alpha = 1.0;
      }
    } else {
      double an = 0.5 * alpha;
      const double den = 2.0 * (J - f - dd);
      if (std::isfinite(J) && den > 0.0)
        an = std::min(std::max(-dd * alpha / den, 0.1 * alpha), 0.5 * alpha);
      alpha = an;
      if (alpha < 1e-10) {
        if (cnt > 0) {
          if (!(direction(true) > 0.0)) res = 1;
          alpha = 1.0;
        } else {
          res = 4;
        }
      }
    }
  }
  if (std::isfinite(f)) std::copy(x.begin(), x.end(), x_io);
  if (cost) *cost = f;
  if (evals) *evals = n_eval;
  if (result) *result = res;
  if (terms) std::copy(best_terms, best_terms + 4, terms);
  return 0;
}

// CPU baseline of bench.py's collision workload: orc_coll_optimize (mode 0,
// unbounded, default initial step) cycling over the B starts X0 [B][nv] of
// one problem, `threads` std::threads, until min_seconds have passed.
int orc_bench_coll(int N, int D, int r, int S, int K, const uint8_t* mask, const double* vals,
                   const double* times, const float* occupancy, int nx, int ny, int nz,
                   const double* params, const int* iparams, const int* soft_derivatives,
                   const double* soft_limits, int B, int nv, const double* X0, int max_evals,
                   int threads, double min_seconds, int64_t* units, double* seconds) {
  if (B < 1 || nv < 1 || threads < 1 || !X0) return -1;
  std::atomic<int> failed(0);
  std::atomic<int64_t> total(0);
  volatile double sink = 0.0;
  const auto t0 = std::chrono::steady_clock::now();
  auto worker = [&](int tid) {
    int64_t n = 0;
    double acc = 0.0;
    std::vector<double> x(nv);
    for (int64_t it = tid;; it += threads) {
      const int b = static_cast<int>(it % B);
      std::copy(X0 + static_cast<size_t>(b) * nv, X0 + static_cast<size_t>(b + 1) * nv,
                x.begin());
      double c = 0.0, terms[4];
      int ev = 0, res = 0;
      if (orc_coll_optimize(N, D, r, S, K, mask, vals, times, 0, occupancy, nx, ny, nz, params,
                            iparams, soft_derivatives, soft_limits, nullptr, nullptr, nullptr,
                            max_evals, x.data(), &c, &ev, &res, terms))
        failed = 1;
      acc += c;
      ++n;
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0)
                            .count();
      if (el >= min_seconds || failed) break;
    }
    total += n;
    sink = sink + acc;
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(worker, t);
  worker(0);
  for (auto& th : pool) th.join();
  *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *units = total;
  return failed ? -2 : 0;
}

}  // extern "C"
