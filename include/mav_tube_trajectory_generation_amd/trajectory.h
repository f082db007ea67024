// trajectory.h — Trajectory = sequence of segments (reference:
// include/mav_tube_trajectory_generation/trajectory.h:32-130,
// src/trajectory.cpp:24-134).
#ifndef MAV_TUBE_TRAJECTORY_GENERATION_AMD_TRAJECTORY_H_
#define MAV_TUBE_TRAJECTORY_GENERATION_AMD_TRAJECTORY_H_

#include <vector>

#include "mav_tube_trajectory_generation_amd/segment.h"
#include "mav_tube_trajectory_generation_amd/vertex.h"

namespace mav_trajectory_generation {

class Trajectory {
 public:
  Trajectory() : D_(0), N_(0), max_time_(0.0) {}

  bool operator==(const Trajectory& rhs) const { return segments_ == rhs.segments_; }
  bool operator!=(const Trajectory& rhs) const { return !operator==(rhs); }

  int D() const { return D_; }
  int N() const { return N_; }
  int K() const { return static_cast<int>(segments_.size()); }
  bool empty() const { return segments_.empty(); }
  void clear() {
    segments_.clear();
    D_ = N_ = 0;
    max_time_ = 0.0;
  }

  // trajectory.h:54-73.
  void setSegments(const Segment::Vector& segments) {
    MTG_CHECK(!segments.empty(), "segments must not be empty");
    D_ = segments.front().D();
    N_ = segments.front().N();
    max_time_ = 0.0;
    segments_.clear();
    addSegments(segments);
  }
  void addSegments(const Segment::Vector& segments) {
    for (const Segment& s : segments) {
      MTG_CHECK(s.D() == D_, "segment dimension mismatch");
      MTG_CHECK(s.N() == N_, "segment order mismatch");
      max_time_ += s.getTime();
    }
    segments_.insert(segments_.end(), segments.begin(), segments.end());
  }
  void getSegments(Segment::Vector* segments) const {
    MTG_CHECK(segments != nullptr, "segments must not be null");
    *segments = segments_;
  }
  const Segment::Vector& segments() const { return segments_; }

  double getMinTime() const { return 0.0; }
  double getMaxTime() const { return max_time_; }
  std::vector<double> getSegmentTimes() const {
    std::vector<double> t;
    for (const Segment& s : segments_) t.push_back(s.getTime());
    return t;
  }

  // Right-continuous segment lookup (trajectory.cpp:41-72).
  VectorXd evaluate(double t, int derivative_order = derivative_order::POSITION) const {
    double acc = 0.0;
    size_t i = 0;
    for (i = 0; i < segments_.size(); ++i) {
      acc += segments_[i].getTime();
      if (acc > t) break;
    }
    if (t > acc) {
      internal::warn("Time out of range of the trajectory!");
      return VectorXd::Zero(D_);
    }
    if (i >= segments_.size()) i = segments_.size() - 1;
    acc -= segments_[i].getTime();
    return segments_[i].evaluate(t - acc, derivative_order);
  }

  // trajectory.cpp:74-134.
  void evaluateRange(double t_start, double t_end, double dt, int derivative_order,
                     std::vector<VectorXd>* result,
                     std::vector<double>* sampling_times = nullptr) const {
    result->clear();
    if (sampling_times) sampling_times->clear();
    double acc = 0.0;
    size_t i = 0;
    for (i = 0; i < segments_.size(); ++i) {
      acc += segments_[i].getTime();
      if (acc > t_start) break;
    }
    if (t_start > acc) {
      internal::warn("Start time out of range of the trajectory!");
      return;
    }
    acc -= segments_[i].getTime();
    double tin = t_start - acc;
    while (acc < t_end) {
      if (tin > segments_[i].getTime()) {
        tin -= segments_[i].getTime();
        ++i;
        if (i >= segments_.size()) break;
        continue;
      }
      result->push_back(segments_[i].evaluate(tin, derivative_order));
      if (sampling_times) sampling_times->push_back(acc);
      tin += dt;
      acc += dt;
    }
  }

  // Vertex at time t with derivatives 0..max_derivative_order
  // (trajectory.cpp:222-240).
  Vertex getVertexAtTime(double t, int max_derivative_order) const {
    Vertex v(D_);
    for (int k = 0; k <= max_derivative_order; ++k) v.addConstraint(k, evaluate(t, k));
    return v;
  }
  Vertex getStartVertex(int max_derivative_order) const {
    return getVertexAtTime(getMinTime(), max_derivative_order);
  }
  Vertex getGoalVertex(int max_derivative_order) const {
    return getVertexAtTime(getMaxTime(), max_derivative_order);
  }

 private:
  int D_;
  int N_;
  double max_time_;
  Segment::Vector segments_;
};

}  // namespace mav_trajectory_generation

#endif  // MAV_TUBE_TRAJECTORY_GENERATION_AMD_TRAJECTORY_H_
