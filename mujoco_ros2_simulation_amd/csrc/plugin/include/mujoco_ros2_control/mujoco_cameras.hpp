// Camera wrapper: per-camera intrinsics + depth images rendered by the HIP depth kernel for env 0
// (API of the reference's include/mujoco_ros2_control/mujoco_cameras.hpp).  RGB rendering is out of
// scope: the colour topic carries a zero image of the right size and encoding.
#pragma once

#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hardware_interface/hardware_info.hpp"
#include "mrs.h"
#include "rclcpp/rclcpp.hpp"
#include "sensor_msgs/msg/camera_info.hpp"
#include "sensor_msgs/msg/image.hpp"

namespace mujoco_ros2_control {

struct CameraData {
  int cam_id = -1;
  std::string name, frame_name, info_topic, image_topic, depth_topic;
  uint32_t width = 0, height = 0;
  std::vector<float> depth;  // H*W, ROS row order, eye-space metres
  sensor_msgs::msg::Image image, depth_image;
  sensor_msgs::msg::CameraInfo camera_info;
  rclcpp::Publisher<sensor_msgs::msg::Image>::SharedPtr image_pub, depth_image_pub;
  rclcpp::Publisher<sensor_msgs::msg::CameraInfo>::SharedPtr camera_info_pub;
};

class MujocoCameras {
 public:
  MujocoCameras(rclcpp::Node::SharedPtr& node, std::recursive_mutex* sim_mutex, mrs_batch* batch,
                const mrs_model* model, double camera_publish_rate);
  ~MujocoCameras() { close(); }
  void init();
  void close();
  void register_cameras(const hardware_interface::HardwareInfo& hardware_info);
  void update();
  const std::vector<CameraData>& cameras() const { return cameras_; }

 private:
  void update_loop();
  rclcpp::Node::SharedPtr node_;
  std::recursive_mutex* sim_mutex_;
  mrs_batch* batch_;
  const mrs_model* model_;
  double camera_publish_rate_;
  std::vector<CameraData> cameras_;
  std::thread thread_;
  std::atomic_bool publish_images_{false};
};

}  // namespace mujoco_ros2_control
