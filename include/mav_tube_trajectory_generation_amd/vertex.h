// vertex.h — Vertex constraint map and the vertex/time generators of the
// host API (reference: include/mav_tube_trajectory_generation/vertex.h:42-174,
// src/vertex.cpp).
#ifndef MAV_TUBE_TRAJECTORY_GENERATION_AMD_VERTEX_H_
#define MAV_TUBE_TRAJECTORY_GENERATION_AMD_VERTEX_H_

#include <cmath>
#include <map>
#include <ostream>
#include <random>
#include <utility>
#include <vector>

#include "mav_tube_trajectory_generation_amd/check.h"
#include "mav_tube_trajectory_generation_amd/linalg.h"
#include "mav_tube_trajectory_generation_amd/motion_defines.h"

namespace mav_trajectory_generation {

// A support point of a path with per-derivative constraints, the same value
// dimension D for every constraint (vertex.h:42-112).
class Vertex {
 public:
  typedef std::vector<Vertex> Vector;
  typedef VectorXd ConstraintValue;
  typedef std::pair<int, ConstraintValue> Constraint;
  typedef std::map<int, ConstraintValue> Constraints;

  explicit Vertex(size_t dimension) : D_(static_cast<int>(dimension)) {}
  int D() const { return D_; }

  void addConstraint(int derivative_order, double value) {
    constraints_[derivative_order] = ConstraintValue::Constant(D_, value);
  }
  void addConstraint(int derivative_order, const VectorXd& constraint) {
    MTG_CHECK(constraint.size() == D_, "constraint dimension " << constraint.size()
                                                               << " != " << D_);
    constraints_[derivative_order] = constraint;
  }
  bool removeConstraint(int type) { return constraints_.erase(type) > 0; }

  // Position plus zero derivatives 1..up_to_derivative (vertex.cpp:147-153).
  void makeStartOrEnd(const VectorXd& constraint, int up_to_derivative) {
    addConstraint(derivative_order::POSITION, constraint);
    for (int i = 1; i <= up_to_derivative; ++i) constraints_[i] = ConstraintValue::Zero(D_);
  }
  void makeStartOrEnd(double value, int up_to_derivative) {
    makeStartOrEnd(VectorXd::Constant(D_, value), up_to_derivative);
  }

  bool hasConstraint(int derivative_order) const {
    return constraints_.count(derivative_order) > 0;
  }
  bool getConstraint(int derivative_order, VectorXd* value) const {
    MTG_CHECK(value != nullptr, "value must not be null");
    auto it = constraints_.find(derivative_order);
    if (it == constraints_.end()) return false;
    *value = it->second;
    return true;
  }
  Constraints::const_iterator cBegin() const { return constraints_.begin(); }
  Constraints::const_iterator cEnd() const { return constraints_.end(); }
  size_t getNumberOfConstraints() const { return constraints_.size(); }

  bool isEqualTol(const Vertex& rhs, double tol) const {
    if (constraints_.size() != rhs.constraints_.size()) return false;
    for (const auto& kv : constraints_) {
      auto it = rhs.constraints_.find(kv.first);
      if (it == rhs.constraints_.end()) return false;
      if (!(kv.second - it->second).isZero(tol)) return false;
    }
    return true;
  }

  bool getSubdimension(const std::vector<size_t>& subdimensions, int max_derivative_order,
                       Vertex* subvertex) const {
    MTG_CHECK(subvertex != nullptr, "subvertex must not be null");
    *subvertex = Vertex(subdimensions.size());
    for (size_t s : subdimensions)
      if (static_cast<int>(s) >= D_) return false;
    for (const auto& kv : constraints_) {
      if (kv.first > max_derivative_order) continue;
      VectorXd sub(static_cast<long>(subdimensions.size()));
      for (size_t i = 0; i < subdimensions.size(); ++i) sub[i] = kv.second[subdimensions[i]];
      subvertex->addConstraint(kv.first, sub);
    }
    return true;
  }

 private:
  int D_;
  Constraints constraints_;
};

inline std::ostream& operator<<(std::ostream& os, const Vertex& v) {
  os << "constraints: " << std::endl;
  for (auto it = v.cBegin(); it != v.cEnd(); ++it)
    os << "  type: " << positionDerivativeToString(it->first) << "  value: [" << it->second
       << "]" << std::endl;
  return os;
}

inline int getHighestDerivativeFromN(int N) { return N / 2 - 1; }  // vertex.h:147

// t = 2 d / v_max (1 + c v_max / a_max exp(-2 d / v_max)) (vertex.cpp:252-269).
inline std::vector<double> estimateSegmentTimesNfabian(const Vertex::Vector& vertices,
                                                       double v_max, double a_max,
                                                       double magic_fabian_constant = 6.5) {
  MTG_CHECK(vertices.size() >= 2, "need at least two vertices");
  std::vector<double> times;
  times.reserve(vertices.size() - 1);
  for (size_t i = 0; i + 1 < vertices.size(); ++i) {
    VectorXd a, b;
    vertices[i].getConstraint(derivative_order::POSITION, &a);
    vertices[i + 1].getConstraint(derivative_order::POSITION, &b);
    const double d = (b - a).norm();
    times.push_back(d / v_max * 2 *
                    (1.0 + magic_fabian_constant * v_max / a_max * std::exp(-d / v_max * 2)));
  }
  return times;
}

// Rest-to-rest bang-coast-bang time (vertex.cpp:271-287).
inline double computeTimeVelocityRamp(const VectorXd& start, const VectorXd& goal,
                                      double v_max, double a_max) {
  const double distance = (start - goal).norm();
  const double acc_time = v_max / a_max;
  const double acc_distance = 0.5 * v_max * acc_time;
  if (distance < 2.0 * acc_distance) return 2.0 * std::sqrt(distance / a_max);
  return 2.0 * acc_time + (distance - 2.0 * acc_distance) / v_max;
}

// vertex.cpp:233-250 (time_factor scaling of vertex.h:131-134).
inline std::vector<double> estimateSegmentTimesVelocityRamp(const Vertex::Vector& vertices,
                                                            double v_max, double a_max,
                                                            double time_factor = 1.0) {
  MTG_CHECK(vertices.size() >= 2, "need at least two vertices");
  std::vector<double> times;
  for (size_t i = 0; i + 1 < vertices.size(); ++i) {
    VectorXd a, b;
    vertices[i].getConstraint(derivative_order::POSITION, &a);
    vertices[i + 1].getConstraint(derivative_order::POSITION, &b);
    times.push_back(computeTimeVelocityRamp(a, b, v_max, a_max) * time_factor);
  }
  return times;
}

// Current preferred method (vertex.cpp:228-231).
inline std::vector<double> estimateSegmentTimes(const Vertex::Vector& vertices, double v_max,
                                                double a_max) {
  return estimateSegmentTimesNfabian(vertices, v_max, a_max);
}

// Random vertices (vertex.cpp:27-82): std::mt19937(seed), one
// uniform_real_distribution<double> per dimension, consecutive vertices more
// than 0.2 apart, start/end fixed up to maximum_derivative.  Bit-identical to
// the reference generator on libstdc++.
inline Vertex::Vector createRandomVertices(int maximum_derivative, size_t n_segments,
                                           const VectorXd& minimum_position,
                                           const VectorXd& maximum_position,
                                           size_t seed = 0) {
  MTG_CHECK(n_segments >= 1, "need at least one segment");
  MTG_CHECK(minimum_position.size() == maximum_position.size(), "bounds dimension mismatch");
  MTG_CHECK((maximum_position - minimum_position).norm() >= 0.2, "bounds too small");
  MTG_CHECK(maximum_derivative > 0, "maximum_derivative must be > 0");
  const long D = minimum_position.size();
  std::mt19937 gen(static_cast<std::mt19937::result_type>(seed));
  std::vector<std::uniform_real_distribution<double>> dist;
  for (long d = 0; d < D; ++d)
    dist.emplace_back(minimum_position[d], maximum_position[d]);
  constexpr double kMinDistance = 0.2;
  VectorXd last(D);
  for (long d = 0; d < D; ++d) last[d] = dist[d](gen);
  Vertex::Vector vertices;
  vertices.reserve(n_segments + 1);
  vertices.emplace_back(static_cast<size_t>(D));
  vertices.front().makeStartOrEnd(last, maximum_derivative);
  for (size_t i = 1; i <= n_segments; ++i) {
    VectorXd pos(D);
    do {
      for (long d = 0; d < D; ++d) pos[d] = dist[d](gen);
    } while (!((pos - last).norm() > kMinDistance));
    Vertex v(static_cast<size_t>(D));
    v.addConstraint(derivative_order::POSITION, pos);
    vertices.push_back(v);
    last = pos;
  }
  vertices.back().makeStartOrEnd(last, maximum_derivative);
  return vertices;
}

inline Vertex::Vector createRandomVertices1D(int maximum_derivative, size_t n_segments,
                                             double minimum_position, double maximum_position,
                                             size_t seed = 0) {
  return createRandomVertices(maximum_derivative, n_segments,
                              VectorXd::Constant(1, minimum_position),
                              VectorXd::Constant(1, maximum_position), seed);
}

// Square loops (vertex.cpp:84-120).
inline Vertex::Vector createSquareVertices(int maximum_derivative, const VectorXd& center,
                                           double side_length, int rounds) {
  MTG_CHECK(center.size() == 3, "center must be 3D");
  const double h = side_length / 2.0;
  VectorXd p1{center[0] - h, center[1] - h, center[2]};
  VectorXd p2{center[0] - h, center[1] + h, center[2]};
  VectorXd p3{center[0] + h, center[1] + h, center[2]};
  VectorXd p4{center[0] + h, center[1] - h, center[2]};
  auto at = [](const VectorXd& p) {
    Vertex v(3);
    v.addConstraint(derivative_order::POSITION, p);
    return v;
  };
  Vertex::Vector vs;
  vs.push_back(at(p1));
  vs.front().makeStartOrEnd(p1, maximum_derivative);
  for (int i = 0; i < rounds; ++i) {
    vs.push_back(at(p2));
    vs.push_back(at(p3));
    vs.push_back(at(p4));
    vs.push_back(at(p1));
  }
  vs.back().makeStartOrEnd(p1, maximum_derivative);
  return vs;
}

}  // namespace mav_trajectory_generation

#endif  // MAV_TUBE_TRAJECTORY_GENERATION_AMD_VERTEX_H_
