// ros_shim: sensor_msgs/msg/Image fields
#pragma once
#include <cstdint>
#include <string>
#include <vector>
#include "sensor_msgs/msg/laser_scan.hpp"
namespace sensor_msgs { namespace msg {
struct Image {
  std_msgs::msg::Header header;
  uint32_t height = 0, width = 0;
  std::string encoding;
  uint8_t is_bigendian = 0;
  uint32_t step = 0;
  std::vector<uint8_t> data;
};
} }
namespace sensor_msgs { namespace image_encodings {
constexpr char RGB8[] = "rgb8";
constexpr char TYPE_32FC1[] = "32FC1";
} }
