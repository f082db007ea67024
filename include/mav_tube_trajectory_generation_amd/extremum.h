// extremum.h — Extremum {time, value, segment_idx}, compared by value
// (reference include/mav_tube_trajectory_generation/extremum.h:28-45).
#ifndef MAV_TUBE_TRAJECTORY_GENERATION_AMD_EXTREMUM_H_
#define MAV_TUBE_TRAJECTORY_GENERATION_AMD_EXTREMUM_H_

#include <ostream>

namespace mav_trajectory_generation {

struct Extremum {
  Extremum() : time(0.0), value(0.0), segment_idx(0) {}
  Extremum(double t, double v, int seg) : time(t), value(v), segment_idx(seg) {}

  bool operator<(const Extremum& rhs) const { return value < rhs.value; }
  bool operator>(const Extremum& rhs) const { return value > rhs.value; }

  double time;       // relative to the start of segment segment_idx
  double value;
  int segment_idx;
};

inline std::ostream& operator<<(std::ostream& os, const Extremum& e) {
  os << "time: " << e.time << ", value: " << e.value << ", segment idx: " << e.segment_idx
     << std::endl;
  return os;
}

}  // namespace mav_trajectory_generation

#endif  // MAV_TUBE_TRAJECTORY_GENERATION_AMD_EXTREMUM_H_
