// ros_shim: sensor_msgs/msg/CameraInfo fields
#pragma once
#include <array>
#include <string>
#include <vector>
#include "sensor_msgs/msg/laser_scan.hpp"
namespace sensor_msgs { namespace msg {
struct CameraInfo {
  std_msgs::msg::Header header;
  uint32_t height = 0, width = 0;
  std::string distortion_model;
  std::vector<double> d;
  std::array<double, 9> k{};
  std::array<double, 9> r{};
  std::array<double, 12> p{};
};
} }
