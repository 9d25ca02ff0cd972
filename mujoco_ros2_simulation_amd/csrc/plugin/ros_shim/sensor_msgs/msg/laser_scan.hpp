// ros_shim: sensor_msgs/msg/LaserScan fields
#pragma once
#include <string>
#include <vector>
#include "rclcpp/rclcpp.hpp"
namespace std_msgs { namespace msg { struct Header { rclcpp::Time stamp; std::string frame_id; }; } }
namespace sensor_msgs { namespace msg {
struct LaserScan {
  std_msgs::msg::Header header;
  float angle_min = 0, angle_max = 0, angle_increment = 0, time_increment = 0, scan_time = 0;
  float range_min = 0, range_max = 0;
  std::vector<float> ranges, intensities;
};
} }
