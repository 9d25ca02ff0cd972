// Lidar wrapper: groups rangefinder sensors "<name>-<digits>" into LaserScan messages
// (API of the reference's include/mujoco_ros2_control/mujoco_lidar.hpp; the rays themselves are cast
// on the GPU by the step kernel, this class only gathers and filters sensordata of env 0).
#pragma once

#include <atomic>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "hardware_interface/hardware_info.hpp"
#include "mrs.h"
#include "mujoco_ros2_control/mj_types.hpp"
#include "rclcpp/rclcpp.hpp"
#include "sensor_msgs/msg/laser_scan.hpp"

namespace mujoco_ros2_control {

struct LidarData {
  std::string name;
  std::string frame_name;
  int num_rangefinders = 0;
  double min_angle = 0, max_angle = 0, angle_increment = 0, range_min = 0, range_max = 0;
  // sensor_indexes[k] = sensordata address of rangefinder "<name>-k"
  std::vector<int> sensor_indexes;
  std::string laserscan_topic;
  sensor_msgs::msg::LaserScan laser_scan_msg;
  rclcpp::Publisher<sensor_msgs::msg::LaserScan>::SharedPtr scan_pub;
};

// "<name>-<digits>" -> (name, index); (name or whole string, -1) if not of that form
std::pair<std::string, int> parse_lidar_name(const std::string& sensor_name);
// LidarData from the ros2_control <sensor name=...> parameters; nullopt if a required one is missing
std::optional<LidarData> get_lidar_data(const hardware_interface::HardwareInfo& hardware_info,
                                        const std::string& name);

class MujocoLidar {
 public:
  MujocoLidar(rclcpp::Node::SharedPtr& node, std::recursive_mutex* sim_mutex, mjData* mujoco_data,
              mjModel* mujoco_model, double lidar_publish_rate);
  ~MujocoLidar() { close(); }
  void init();
  void close();
  bool register_lidar(const hardware_interface::HardwareInfo& hardware_info);
  void update();  // one gather + filter + publish (public so a test can drive it synchronously)
  const std::vector<LidarData>& lidars() const { return lidar_sensors_; }

 private:
  void update_loop();
  rclcpp::Node::SharedPtr node_;
  std::recursive_mutex* sim_mutex_;
  mjData* mj_data_;
  mjModel* mj_model_;
  double lidar_publish_rate_;
  std::vector<double> snapshot_;
  std::vector<LidarData> lidar_sensors_;
  std::thread thread_;
  std::atomic_bool publish_lidar_{false};
};

}  // namespace mujoco_ros2_control
