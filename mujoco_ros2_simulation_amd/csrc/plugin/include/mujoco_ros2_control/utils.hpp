// get_sensor_from_info (reference include/mujoco_ros2_control/utils.hpp:30-42)
#pragma once
#include <map>
#include <optional>
#include <string>
#include "hardware_interface/hardware_info.hpp"

namespace mujoco_ros2_control {

inline std::optional<hardware_interface::ComponentInfo> get_sensor_from_info(
    const hardware_interface::HardwareInfo& info, const std::string& name) {
  for (const auto& s : info.sensors)
    if (s.name == name) return s;
  return std::nullopt;
}

// ROS 2 parameter file (--params-file) flattened to dotted names under ros__parameters; repeated
// keys merge (defined in mujoco_system_interface.cpp)
std::map<std::string, std::string> load_ros_params_file(const std::string& path);

}  // namespace mujoco_ros2_control
