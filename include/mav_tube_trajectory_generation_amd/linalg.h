// linalg.h — minimal dense FP64 vector / matrix types standing in for the
// Eigen::VectorXd / Eigen::MatrixXd of the reference's public API
// (vertex.h:45, polynomial.h:61; Eigen is not available in this image,
// SURVEY.md §8b).  Only the operations the API surface needs; column vectors,
// and matrices stored column-major as Eigen's default MatrixXd is, so a
// caller copying getM() / getA() / getAInverse() / getMpinv() through
// data() reads the same order it would from Eigen; operator()(i, j)
// indexing as in Eigen.
#ifndef MAV_TUBE_TRAJECTORY_GENERATION_AMD_LINALG_H_
#define MAV_TUBE_TRAJECTORY_GENERATION_AMD_LINALG_H_

#include <cmath>
#include <complex>
#include <cstddef>
#include <initializer_list>
#include <ostream>
#include <stdexcept>
#include <vector>

namespace mav_trajectory_generation {

class VectorXd {
 public:
  VectorXd() {}
  explicit VectorXd(long n) : v_(static_cast<size_t>(n), 0.0) {}
  VectorXd(std::initializer_list<double> l) : v_(l) {}
  explicit VectorXd(const std::vector<double>& v) : v_(v) {}

  static VectorXd Zero(long n) { return VectorXd(n); }
  static VectorXd Constant(long n, double x) {
    VectorXd r(n);
    for (double& e : r.v_) e = x;
    return r;
  }

  long size() const { return static_cast<long>(v_.size()); }
  long rows() const { return size(); }
  void resize(long n) { v_.assign(static_cast<size_t>(n), 0.0); }
  void setZero() {
    for (double& e : v_) e = 0.0;
  }
  double& operator[](long i) { return v_[static_cast<size_t>(i)]; }
  double operator[](long i) const { return v_[static_cast<size_t>(i)]; }
  double& operator()(long i) { return v_[static_cast<size_t>(i)]; }
  double operator()(long i) const { return v_[static_cast<size_t>(i)]; }
  double* data() { return v_.data(); }
  const double* data() const { return v_.data(); }

  double squaredNorm() const {
    double s = 0.0;
    for (double e : v_) s += e * e;
    return s;
  }
  double norm() const { return std::sqrt(squaredNorm()); }
  double dot(const VectorXd& o) const {
    check(o);
    double s = 0.0;
    for (size_t i = 0; i < v_.size(); ++i) s += v_[i] * o.v_[i];
    return s;
  }
  double sum() const {
    double s = 0.0;
    for (double e : v_) s += e;
    return s;
  }
  VectorXd head(long n) const {
    return VectorXd(std::vector<double>(v_.begin(), v_.begin() + n));
  }
  VectorXd segment(long start, long n) const {
    return VectorXd(std::vector<double>(v_.begin() + start, v_.begin() + start + n));
  }
  VectorXd tail(long n) const {
    return VectorXd(std::vector<double>(v_.end() - n, v_.end()));
  }

  VectorXd operator+(const VectorXd& o) const {
    check(o);
    VectorXd r(*this);
    for (size_t i = 0; i < v_.size(); ++i) r.v_[i] += o.v_[i];
    return r;
  }
  VectorXd operator-(const VectorXd& o) const {
    check(o);
    VectorXd r(*this);
    for (size_t i = 0; i < v_.size(); ++i) r.v_[i] -= o.v_[i];
    return r;
  }
  VectorXd& operator+=(const VectorXd& o) {
    check(o);
    for (size_t i = 0; i < v_.size(); ++i) v_[i] += o.v_[i];
    return *this;
  }
  VectorXd operator*(double s) const {
    VectorXd r(*this);
    for (double& e : r.v_) e *= s;
    return r;
  }
  bool operator==(const VectorXd& o) const { return v_ == o.v_; }
  bool operator!=(const VectorXd& o) const { return v_ != o.v_; }
  // Eigen's isZero(tol): every |entry| <= tol.
  bool isZero(double tol) const {
    for (double e : v_)
      if (std::fabs(e) > tol) return false;
    return true;
  }

 private:
  void check(const VectorXd& o) const {
    if (o.v_.size() != v_.size()) throw std::invalid_argument("VectorXd size mismatch");
  }
  std::vector<double> v_;
};

inline VectorXd operator*(double s, const VectorXd& v) { return v * s; }

// Eigen::Vector3d (the x, y, z triples of
// PolynomialOptimizationNonLinear::getFreeConstraints,
// polynomial_optimization_nonlinear.h:293): a VectorXd of size 3.
class Vector3d : public VectorXd {
 public:
  Vector3d() : VectorXd(3) {}
  Vector3d(double x, double y, double z) : VectorXd({x, y, z}) {}
  double x() const { return (*this)[0]; }
  double y() const { return (*this)[1]; }
  double z() const { return (*this)[2]; }
};

inline std::ostream& operator<<(std::ostream& os, const VectorXd& v) {
  for (long i = 0; i < v.size(); ++i) os << (i ? " " : "") << v[i];
  return os;
}

// Complex column vector (Eigen::VectorXcd of Polynomial::getRoots,
// polynomial.h:153; findRootsJenkinsTraub, rpoly_ak1.h:26).
class VectorXcd {
 public:
  typedef std::complex<double> Scalar;
  VectorXcd() {}
  explicit VectorXcd(long n) : v_(static_cast<size_t>(n)) {}
  long size() const { return static_cast<long>(v_.size()); }
  long rows() const { return size(); }
  void resize(long n) { v_.assign(static_cast<size_t>(n), Scalar()); }
  Scalar& operator[](long i) { return v_[static_cast<size_t>(i)]; }
  const Scalar& operator[](long i) const { return v_[static_cast<size_t>(i)]; }
  Scalar& operator()(long i) { return v_[static_cast<size_t>(i)]; }
  const Scalar& operator()(long i) const { return v_[static_cast<size_t>(i)]; }
  Scalar* data() { return v_.data(); }
  const Scalar* data() const { return v_.data(); }
  VectorXd real() const {
    VectorXd r(size());
    for (long i = 0; i < size(); ++i) r[i] = v_[static_cast<size_t>(i)].real();
    return r;
  }
  VectorXd imag() const {
    VectorXd r(size());
    for (long i = 0; i < size(); ++i) r[i] = v_[static_cast<size_t>(i)].imag();
    return r;
  }

 private:
  std::vector<Scalar> v_;
};

class MatrixXd {
 public:
  MatrixXd() {}
  MatrixXd(long r, long c) : r_(r), c_(c), a_(static_cast<size_t>(r * c), 0.0) {}
  static MatrixXd Zero(long r, long c) { return MatrixXd(r, c); }
  static MatrixXd Identity(long n) {
    MatrixXd m(n, n);
    for (long i = 0; i < n; ++i) m(i, i) = 1.0;
    return m;
  }
  long rows() const { return r_; }
  long cols() const { return c_; }
  void resize(long r, long c) {
    r_ = r;
    c_ = c;
    a_.assign(static_cast<size_t>(r * c), 0.0);
  }
  void setZero() {
    for (double& e : a_) e = 0.0;
  }
  // Column-major: entry (i, j) at data()[j * rows() + i] (Eigen's default).
  double& operator()(long i, long j) { return a_[static_cast<size_t>(j * r_ + i)]; }
  double operator()(long i, long j) const { return a_[static_cast<size_t>(j * r_ + i)]; }
  double* data() { return a_.data(); }
  const double* data() const { return a_.data(); }

  MatrixXd transpose() const {
    MatrixXd t(c_, r_);
    for (long i = 0; i < r_; ++i)
      for (long j = 0; j < c_; ++j) t(j, i) = (*this)(i, j);
    return t;
  }
  MatrixXd operator*(const MatrixXd& o) const {
    if (c_ != o.r_) throw std::invalid_argument("MatrixXd product size mismatch");
    MatrixXd p(r_, o.c_);
    for (long i = 0; i < r_; ++i)
      for (long k = 0; k < c_; ++k) {
        const double a = (*this)(i, k);
        if (a == 0.0) continue;
        for (long j = 0; j < o.c_; ++j) p(i, j) += a * o(k, j);
      }
    return p;
  }
  VectorXd operator*(const VectorXd& v) const {
    if (c_ != v.size()) throw std::invalid_argument("MatrixXd * VectorXd size mismatch");
    VectorXd y(r_);
    for (long i = 0; i < r_; ++i) {
      double s = 0.0;
      for (long j = 0; j < c_; ++j) s += (*this)(i, j) * v[j];
      y[i] = s;
    }
    return y;
  }
  MatrixXd operator-(const MatrixXd& o) const {
    MatrixXd d(*this);
    for (size_t i = 0; i < a_.size(); ++i) d.a_[i] -= o.a_[i];
    return d;
  }
  double maxAbs() const {
    double m = 0.0;
    for (double e : a_) m = std::fabs(e) > m ? std::fabs(e) : m;
    return m;
  }

 private:
  long r_ = 0, c_ = 0;
  std::vector<double> a_;
};

}  // namespace mav_trajectory_generation

#endif  // MAV_TUBE_TRAJECTORY_GENERATION_AMD_LINALG_H_
