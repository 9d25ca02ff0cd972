// Host-side state containers of the plugin (mirror of the reference's
// include/mujoco_ros2_control/data.hpp:43-112).  Field addresses are exported to the controller
// manager as raw double* (StateInterface / CommandInterface), so containers must not reallocate
// after export.  Vec3/Quat replace the Eigen types (Eigen is not a dependency here); x()/y()/z()/w()
// return references exactly like Eigen's accessors, so `&data.x()` is the exported address.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "control_toolbox/pid_ros.hpp"

namespace mujoco_ros2_control {

// same enumerators and order as the reference (data.hpp:43-51); mrs_actuator_type() uses it
enum class ActuatorType { UNKNOWN, MOTOR, POSITION, VELOCITY, CUSTOM };

struct Vec3 {
  double v[3] = {0, 0, 0};
  double& x() { return v[0]; }
  double& y() { return v[1]; }
  double& z() { return v[2]; }
};
struct Quat {
  double v[4] = {1, 0, 0, 0};  // w, x, y, z storage; accessors by name
  double& w() { return v[0]; }
  double& x() { return v[1]; }
  double& y() { return v[2]; }
  double& z() { return v[3]; }
};

struct JointState {
  std::string name;
  double position = 0, velocity = 0, effort = 0;
  std::shared_ptr<control_toolbox::PidROS> pos_pid, vel_pid;
  ActuatorType actuator_type = ActuatorType::UNKNOWN;
  double position_command = 0, velocity_command = 0, effort_command = 0;
  bool is_mimic = false;
  int mimicked_joint_index = -1;
  double mimic_multiplier = 1.0;
  int mj_joint_type = -1, mj_pos_adr = -1, mj_vel_adr = -1, mj_actuator_id = -1;
  bool is_position_control_enabled = false, is_position_pid_control_enabled = false;
  bool is_velocity_pid_control_enabled = false, is_velocity_control_enabled = false;
  bool is_effort_control_enabled = false;
  bool has_pos_pid = false, has_vel_pid = false;
};

template <typename T>
struct SensorData {
  std::string name;
  T data;
  int mj_sensor_index = -1;
};

struct FTSensorData {
  std::string name;
  SensorData<Vec3> force, torque;
};

struct IMUSensorData {
  std::string name;
  SensorData<Quat> orientation;
  SensorData<Vec3> angular_velocity, linear_acceleration;
  std::vector<double> orientation_covariance, angular_velocity_covariance, linear_acceleration_covariance;
};

}  // namespace mujoco_ros2_control
