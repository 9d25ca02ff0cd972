// Camera wrapper (behaviour of the reference's src/mujoco_cameras.cpp).  Depth and colour come from
// the HIP ray-cast kernel (mrs_batch_render_rgbd, env 0) — already in ROS row order, depth in linear
// eye-space metres, so the reference's OpenGL readback, flip and linearisation loops (:211-250) have
// no counterpart.  Colour is flat headlight shading of geom rgba, not an OpenGL raster match.  No GL context: init() cannot fail for lack of a display.
#include "mujoco_ros2_control/mujoco_cameras.hpp"

#include <cmath>
#include <cstring>

#include "mujoco_ros2_control/utils.hpp"

namespace mujoco_ros2_control {

MujocoCameras::MujocoCameras(rclcpp::Node::SharedPtr& node, std::recursive_mutex* sim_mutex, mrs_batch* batch,
                             const mrs_model* model, double camera_publish_rate)
    : node_(node), sim_mutex_(sim_mutex), batch_(batch), model_(model), camera_publish_rate_(camera_publish_rate) {}

void MujocoCameras::register_cameras(const hardware_interface::HardwareInfo& hardware_info) {
  cameras_.clear();
  mrs_model_view v{};
  mrs_model_view_get(model_, &v);
  for (int i = 0; i < v.ncam; ++i) {
    CameraData cam;
    const char* name = mrs_id2name(model_, MRS_OBJ_CAMERA, i);
    cam.cam_id = i;
    cam.name = name ? name : "";
    cam.width = static_cast<uint32_t>(v.cam_resolution[2 * i]);
    cam.height = static_cast<uint32_t>(v.cam_resolution[2 * i + 1]);
    if (auto info = get_sensor_from_info(hardware_info, cam.name)) {
      // all four required once the camera is named in ros2_control (.at() in the reference :59-62)
      cam.frame_name = info->parameters.at("frame_name");
      cam.info_topic = info->parameters.at("info_topic");
      cam.image_topic = info->parameters.at("image_topic");
      cam.depth_topic = info->parameters.at("depth_topic");
    } else {
      cam.frame_name = cam.name + "_frame";
      cam.info_topic = cam.name + "/camera_info";
      cam.image_topic = cam.name + "/color";
      cam.depth_topic = cam.name + "/depth";
    }
    RCLCPP_INFO_STREAM(node_->get_logger(), "Adding camera: " << cam.name << " (" << cam.width << "x" << cam.height << ")");
    cam.camera_info_pub = node_->create_publisher<sensor_msgs::msg::CameraInfo>(cam.info_topic, 1);
    cam.image_pub = node_->create_publisher<sensor_msgs::msg::Image>(cam.image_topic, 1);
    cam.depth_image_pub = node_->create_publisher<sensor_msgs::msg::Image>(cam.depth_topic, 1);

    cam.image.header.frame_id = cam.frame_name;
    cam.image.width = cam.width;
    cam.image.height = cam.height;
    cam.image.step = cam.width * 3;
    cam.image.encoding = sensor_msgs::image_encodings::RGB8;
    cam.image.data.assign(size_t(cam.width) * cam.height * 3, 0);

    cam.depth.assign(size_t(cam.width) * cam.height, 0.0f);
    cam.depth_image.header.frame_id = cam.frame_name;
    cam.depth_image.width = cam.width;
    cam.depth_image.height = cam.height;
    cam.depth_image.step = cam.width * sizeof(float);
    cam.depth_image.encoding = sensor_msgs::image_encodings::TYPE_32FC1;
    cam.depth_image.data.assign(cam.depth.size() * sizeof(float), 0);

    // pinhole intrinsics from the vertical field of view (reference :104-117)
    auto& ci = cam.camera_info;
    ci.header.frame_id = cam.frame_name;
    ci.width = cam.width;
    ci.height = cam.height;
    ci.distortion_model = "plumb_bob";
    ci.d.assign(5, 0.0);
    ci.k.fill(0.0);
    ci.r.fill(0.0);
    ci.p.fill(0.0);
    const double f = cam.height / 2.0 / std::tan(v.cam_fovy[i] * M_PI / 180.0 / 2.0);
    ci.k[0] = ci.p[0] = f;
    ci.k[4] = ci.p[5] = f;
    ci.k[2] = ci.p[2] = cam.width / 2.0;
    ci.k[5] = ci.p[6] = cam.height / 2.0;
    ci.k[8] = ci.p[10] = 1.0;
    cameras_.push_back(std::move(cam));
  }
}

void MujocoCameras::init() {
  if (cameras_.empty() || publish_images_) return;
  publish_images_ = true;
  thread_ = std::thread([this] { update_loop(); });
}

void MujocoCameras::close() {
  publish_images_ = false;
  if (thread_.joinable()) thread_.join();
}

void MujocoCameras::update_loop() {
  rclcpp::Rate rate(camera_publish_rate_);
  while (rclcpp::ok() && publish_images_) {
    update();
    rate.sleep();
  }
}

void MujocoCameras::update() {
  {
    // the depth kernel reads the batch's current geom/camera poses; holding the sim mutex keeps
    // the physics thread from stepping underneath it (mjv_copyData under the lock, reference :199-203)
    std::lock_guard<std::recursive_mutex> lock(*sim_mutex_);
    for (auto& cam : cameras_)
      if (mrs_batch_render_rgbd(batch_, cam.cam_id, 0, 1, cam.depth.data(), cam.image.data.data()) != MRS_OK)
        RCLCPP_ERROR(node_->get_logger(), "render of camera %s failed: %s", cam.name.c_str(), mrs_last_error());
  }
  for (auto& cam : cameras_) {
    std::memcpy(cam.depth_image.data.data(), cam.depth.data(), cam.depth_image.data.size());
    const auto t = node_->now();
    cam.image.header.stamp = cam.depth_image.header.stamp = cam.camera_info.header.stamp = t;
    cam.image_pub->publish(cam.image);
    cam.depth_image_pub->publish(cam.depth_image);
    cam.camera_info_pub->publish(cam.camera_info);
  }
}

}  // namespace mujoco_ros2_control
