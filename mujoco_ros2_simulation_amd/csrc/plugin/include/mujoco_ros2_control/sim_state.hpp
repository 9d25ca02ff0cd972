// Host mirror of one environment's mjData fields the plugin exchanges with the GPU batch (the
// "mj_data_" / "mj_data_control_" double buffer of the reference, src/mujoco_system_interface.cpp:
// 684-688, 1756-1762).  Guarded by the plugin's sim mutex.
#pragma once
#include <vector>

namespace mujoco_ros2_control {

struct SimState {
  std::vector<double> qpos, qvel, ctrl, qfrc_applied, qfrc_actuator, sensordata;
  double time = 0;
};

}  // namespace mujoco_ros2_control
