// mujoco_ros2_control/MujocoSystemInterface backed by the MI355X batch simulator.
//
// Public API identical to the reference (include/mujoco_ros2_control/mujoco_system_interface.hpp:
// 61-100), get_model/get_data/set_data included: mjModel / mjData are this library's own
// (mujoco_ros2_control/mj_types.hpp, MuJoCo field names).  MuJoCo is not linked: the physics is
// libmrs (include/mrs.h), env 0 of a batch is the ROS-visible robot.
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "hardware_interface/handle.hpp"
#include "hardware_interface/hardware_info.hpp"
#include "hardware_interface/system_interface.hpp"
#include "hardware_interface/types/hardware_interface_return_values.hpp"
#include "mrs.h"
#include "mujoco_ros2_control/data.hpp"
#include "mujoco_ros2_control/mujoco_cameras.hpp"
#include "mujoco_ros2_control/mujoco_lidar.hpp"
#include "mujoco_ros2_control/mj_types.hpp"
#include "rclcpp/rclcpp.hpp"
#include "rclcpp_lifecycle/state.hpp"
#include "realtime_tools/realtime_publisher.hpp"
#include "rosgraph_msgs/msg/clock.hpp"

namespace mujoco_ros2_control {

class MujocoSystemInterface : public hardware_interface::SystemInterface {
 public:
  MujocoSystemInterface();
  ~MujocoSystemInterface() override;

  hardware_interface::CallbackReturn on_init(const hardware_interface::HardwareComponentInterfaceParams& params) override;
  std::vector<hardware_interface::StateInterface> export_state_interfaces() override;
  std::vector<hardware_interface::CommandInterface> export_command_interfaces() override;
  hardware_interface::CallbackReturn on_activate(const rclcpp_lifecycle::State& previous_state) override;
  hardware_interface::CallbackReturn on_deactivate(const rclcpp_lifecycle::State& previous_state) override;
  hardware_interface::return_type perform_command_mode_switch(const std::vector<std::string>& start_interfaces,
                                                              const std::vector<std::string>& stop_interfaces) override;
  hardware_interface::return_type read(const rclcpp::Time& time, const rclcpp::Duration& period) override;
  hardware_interface::return_type write(const rclcpp::Time& time, const rclcpp::Duration& period) override;

  // deep copies under the sim mutex (reference :1794-1814); dest == nullptr allocates (the caller
  // frees with mj_deleteModel / mj_deleteData)
  void get_model(mjModel*& dest);
  void get_data(mjData*& dest);
  void set_data(mjData* mj_data);

  // --- additions (not in the reference API) used by the test harness and tools
  rclcpp::Node::SharedPtr node() const { return mujoco_node_; }
  mrs_batch* batch() const { return batch_; }
  double sim_time() const;
  // advance the sim synchronously by n physics steps with the current control buffer (the body of
  // one PhysicsLoop iteration without wall-clock pacing); requires physics_thread=false
  bool step_physics(int n);
  MujocoLidar* lidar() const { return lidar_sensors_.get(); }
  MujocoCameras* cameras() const { return cameras_.get(); }
  const std::vector<JointState>& joint_states() const { return joint_states_; }

 private:
  void register_joints(const hardware_interface::HardwareInfo& info);
  void register_sensors(const hardware_interface::HardwareInfo& info);
  bool set_override_start_positions(const std::string& override_start_position_file);
  void set_initial_pose();
  void PhysicsLoop();
  void publish_clock();
  rclcpp::Logger get_logger() const { return logger_; }

  // control -> sim, n steps, sim -> control (caller holds sim_mutex_); false if diverged
  bool advance_locked(int n);
  void pull_state_locked();

  std::string model_path_;
  mjModel* mj_model_ = nullptr;         // owns the compiled model
  mrs_model* model_ = nullptr;          // mj_model_->handle
  mrs_batch* batch_ = nullptr;
  mrs_model_view view_{};
  mjData* mj_data_ = nullptr;           // latest state of env 0
  mjData* mj_data_control_ = nullptr;   // buffer read()/write() use
  rclcpp::Logger logger_ = rclcpp::get_logger("MujocoSystemInterface");
  double sim_speed_factor_ = -1;
  bool run_ = true;
  std::atomic_bool exit_request_{false};
  bool use_physics_thread_ = true;
  std::thread physics_thread_;
  std::shared_ptr<rclcpp::Node> mujoco_node_;
  std::shared_ptr<rclcpp::Publisher<rosgraph_msgs::msg::Clock>> clock_publisher_;
  realtime_tools::RealtimePublisher<rosgraph_msgs::msg::Clock>::SharedPtr clock_realtime_publisher_;
  std::unique_ptr<MujocoCameras> cameras_;
  std::unique_ptr<MujocoLidar> lidar_sensors_;
  mutable std::recursive_mutex sim_mutex_;
  std::unordered_map<std::string, hardware_interface::ComponentInfo> joint_hw_info_;
  std::unordered_map<std::string, hardware_interface::ComponentInfo> sensors_hw_info_;
  std::vector<JointState> joint_states_;
  std::vector<FTSensorData> ft_sensor_data_;
  std::vector<IMUSensorData> imu_sensor_data_;
  std::string load_error_;
};

}  // namespace mujoco_ros2_control
