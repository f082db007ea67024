// motion_defines.h — derivative order constants (reference:
// include/mav_tube_trajectory_generation/motion_defines.h:28-41,
// src/motion_defines.cpp).
#ifndef MAV_TUBE_TRAJECTORY_GENERATION_AMD_MOTION_DEFINES_H_
#define MAV_TUBE_TRAJECTORY_GENERATION_AMD_MOTION_DEFINES_H_

#include <string>

namespace mav_trajectory_generation {
namespace derivative_order {
static constexpr int POSITION = 0;
static constexpr int VELOCITY = 1;
static constexpr int ACCELERATION = 2;
static constexpr int JERK = 3;
static constexpr int SNAP = 4;

static constexpr int ORIENTATION = 0;
static constexpr int ANGULAR_VELOCITY = 1;
static constexpr int ANGULAR_ACCELERATION = 2;

static constexpr int INVALID = -1;
static constexpr int kINVALID = -1;
}  // namespace derivative_order

inline std::string positionDerivativeToString(int derivative) {
  switch (derivative) {
    case derivative_order::POSITION: return "position";
    case derivative_order::VELOCITY: return "velocity";
    case derivative_order::ACCELERATION: return "acceleration";
    case derivative_order::JERK: return "jerk";
    case derivative_order::SNAP: return "snap";
    default: return "invalid";
  }
}

inline int positionDerivativeToInt(const std::string& s) {
  if (s == "position") return derivative_order::POSITION;
  if (s == "velocity") return derivative_order::VELOCITY;
  if (s == "acceleration") return derivative_order::ACCELERATION;
  if (s == "jerk") return derivative_order::JERK;
  if (s == "snap") return derivative_order::SNAP;
  return derivative_order::INVALID;
}

}  // namespace mav_trajectory_generation

#endif  // MAV_TUBE_TRAJECTORY_GENERATION_AMD_MOTION_DEFINES_H_
