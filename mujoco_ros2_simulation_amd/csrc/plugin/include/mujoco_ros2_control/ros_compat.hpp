// The three places the plugin touches rclcpp beyond the API common to ROS 2 and the build-time shim
// (csrc/plugin/ros_shim): node creation with the PID parameter file, the robot-description fallback
// and the simulated clock.  MRS_WITH_ROS is defined by the colcon build (csrc/plugin/CMakeLists.txt).
#pragma once

#include <optional>
#include <string>

#include "mujoco_ros2_control/utils.hpp"
#include "rclcpp/rclcpp.hpp"

#ifdef MRS_WITH_ROS
#include <chrono>
#include <mutex>
#include <rcl/arguments.h>
#include <std_msgs/msg/string.hpp>
#endif

namespace mujoco_ros2_control::compat {

#ifdef MRS_WITH_ROS

// reference :653-675: use_sim_time plus --ros-args --params-file <pids_config_file>
inline rclcpp::Node::SharedPtr make_node(const std::string& name, const std::optional<std::string>& params_file,
                                         const std::map<std::string, std::string>& extra = {}) {
  rclcpp::NodeOptions options;
  options.append_parameter_override("use_sim_time", rclcpp::ParameterValue(true));
  for (const auto& kv : extra) options.append_parameter_override(kv.first, rclcpp::ParameterValue(kv.second));
  if (params_file) {
    auto args = options.arguments();
    args.insert(args.end(), {RCL_ROS_ARGS_FLAG, RCL_PARAM_FILE_FLAG, *params_file});
    options.arguments(args);
  }
  return std::make_shared<rclcpp::Node>(name, options);
}

// reference :358-413: the MJCF string from the transient-local /mujoco_robot_description topic
inline std::optional<std::string> robot_description(const rclcpp::Node::SharedPtr& node) {
  std::mutex mu;
  std::optional<std::string> xml;
  auto sub = node->create_subscription<std_msgs::msg::String>(
      "/mujoco_robot_description", rclcpp::QoS(1).transient_local(),
      [&](const std_msgs::msg::String::SharedPtr m) { std::lock_guard<std::mutex> l(mu); xml = m->data; });
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(10);
  while (std::chrono::steady_clock::now() < deadline) {
    rclcpp::spin_some(node);
    std::lock_guard<std::mutex> l(mu);
    if (xml) break;
  }
  return xml;
}

// with use_sim_time the node clock follows /clock by itself
inline void set_sim_time(const rclcpp::Node::SharedPtr&, const rclcpp::Time&) {}

#else  // build-time shim

inline rclcpp::Node::SharedPtr make_node(const std::string& name, const std::optional<std::string>& params_file,
                                         std::map<std::string, std::string> extra = {}) {
  if (params_file) {
    auto p = load_ros_params_file(*params_file);
    extra.insert(p.begin(), p.end());
  }
  return std::make_shared<rclcpp::Node>(name, extra);
}

// the shim has no topics to wait on: the description is a node parameter
inline std::optional<std::string> robot_description(const rclcpp::Node::SharedPtr& node) {
  return node->get_parameter("mujoco_robot_description");
}

inline void set_sim_time(const rclcpp::Node::SharedPtr& node, const rclcpp::Time& t) { node->set_now(t); }

#endif

}  // namespace mujoco_ros2_control::compat
