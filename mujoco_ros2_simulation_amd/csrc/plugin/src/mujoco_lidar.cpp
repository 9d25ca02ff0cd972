// Lidar wrapper (behaviour of the reference's src/mujoco_lidar.cpp).  The 1-D rangefinder rays are
// cast by the GPU step kernel into sensordata; this class groups them into LaserScan messages.
#include "mujoco_ros2_control/mujoco_lidar.hpp"

#include <algorithm>
#include <cctype>

#include "mujoco_ros2_control/utils.hpp"

namespace mujoco_ros2_control {

std::pair<std::string, int> parse_lidar_name(const std::string& sensor_name) {
  // "<name>-<digits>" as produced by <replicate> (reference :29-47)
  const auto dash = sensor_name.rfind('-');
  if (dash == std::string::npos) return {sensor_name, -1};
  const std::string digits = sensor_name.substr(dash + 1);
  const bool numeric = !digits.empty() &&
                       std::all_of(digits.begin(), digits.end(), [](unsigned char c) { return std::isdigit(c); });
  return {sensor_name.substr(0, dash), numeric ? std::stoi(digits) : -1};
}

std::optional<LidarData> get_lidar_data(const hardware_interface::HardwareInfo& hardware_info,
                                        const std::string& name) {
  // required: frame_name, min_angle, max_angle, angle_increment (reference :52-112)
  const auto info = get_sensor_from_info(hardware_info, name);
  if (!info) return std::nullopt;
  auto p = [&](const char* key) -> std::optional<std::string> {
    auto it = info->parameters.find(key);
    if (it == info->parameters.end()) return std::nullopt;
    return it->second;
  };
  const auto frame = p("frame_name"), amin = p("min_angle"), amax = p("max_angle"), inc = p("angle_increment");
  if (!frame || !amin || !amax || !inc) return std::nullopt;

  LidarData d;
  d.name = name;
  d.frame_name = *frame;
  d.min_angle = std::stod(*amin);
  d.max_angle = std::stod(*amax);
  d.angle_increment = std::stod(*inc);
  d.num_rangefinders = static_cast<int>((d.max_angle - d.min_angle) / d.angle_increment) + 1;
  d.laserscan_topic = p("laserscan_topic").value_or("/scan");
  d.range_min = p("range_min") ? std::stod(*p("range_min")) : 0.0;
  d.range_max = p("range_max") ? std::stod(*p("range_max")) : 1000.0;
  // scan indices no rangefinder maps to keep address 0 and so publish sensordata[0], as the
  // reference's value-initialised resize does (reference :98, read at :261-263)
  d.sensor_indexes.assign(std::max(0, d.num_rangefinders), 0);

  auto& msg = d.laser_scan_msg;
  msg.header.frame_id = d.frame_name;
  msg.time_increment = 0.0f;
  msg.angle_min = static_cast<float>(d.min_angle);
  msg.angle_max = static_cast<float>(d.max_angle);
  msg.angle_increment = static_cast<float>(d.angle_increment);
  msg.range_min = static_cast<float>(d.range_min);
  msg.range_max = static_cast<float>(d.range_max);
  msg.ranges.assign(d.sensor_indexes.size(), 0.0f);
  msg.intensities.clear();
  return d;
}

MujocoLidar::MujocoLidar(rclcpp::Node::SharedPtr& node, std::recursive_mutex* sim_mutex, mjData* mujoco_data,
                         mjModel* mujoco_model, double lidar_publish_rate)
    : node_(node), sim_mutex_(sim_mutex), mj_data_(mujoco_data), mj_model_(mujoco_model), lidar_publish_rate_(lidar_publish_rate) {}

bool MujocoLidar::register_lidar(const hardware_interface::HardwareInfo& hardware_info) {
  lidar_sensors_.clear();
  const mjModel& v = *mj_model_;
  for (int i = 0; i < v.nsensor; ++i) {
    if (v.sensor_type[i] != MRS_SENS_RANGEFINDER) continue;
    const char* raw = mrs_id2name(mj_model_->handle, MRS_OBJ_SENSOR, i);
    if (!raw) {
      RCLCPP_WARN_STREAM(node_->get_logger(), "Cannot find a name for lidar sensor at index: " << i << ", skipping!");
      continue;
    }
    const auto [lidar_name, idx] = parse_lidar_name(raw);
    if (idx == -1) {
      RCLCPP_WARN_STREAM(node_->get_logger(), "Failed to parse lidar sensor name: " << raw << ", skipping!");
      continue;
    }
    auto it = std::find_if(lidar_sensors_.begin(), lidar_sensors_.end(),
                           [&](const LidarData& d) { return d.name == lidar_name; });
    if (it == lidar_sensors_.end()) {
      auto data = get_lidar_data(hardware_info, lidar_name);
      if (!data) {
        RCLCPP_ERROR_STREAM(node_->get_logger(), "Failed to parse required configuration from ros2_control xacro: " << lidar_name);
        return false;
      }
      data->scan_pub = node_->create_publisher<sensor_msgs::msg::LaserScan>(data->laserscan_topic, 1);
      data->laser_scan_msg.scan_time = static_cast<float>(1.0 / lidar_publish_rate_);
      RCLCPP_INFO_STREAM(node_->get_logger(), "Adding lidar sensor: " << data->name << ", num_rangefinders: "
                                                                      << data->num_rangefinders);
      lidar_sensors_.push_back(std::move(*data));
      it = lidar_sensors_.end() - 1;
    }
    // the reference writes sensor_indexes[idx] unchecked; rays beyond the configured scan width are
    // dropped here (the scan is truncated to num_rangefinders, same published message)
    if (idx < static_cast<int>(it->sensor_indexes.size()))
      it->sensor_indexes[idx] = v.sensor_adr[i];
    else
      RCLCPP_WARN_STREAM(node_->get_logger(), "Rangefinder " << raw << " is beyond the configured scan width of "
                                                             << it->name << ", ignored");
  }
  return true;
}

void MujocoLidar::init() {
  if (lidar_sensors_.empty() || publish_lidar_) return;
  publish_lidar_ = true;
  thread_ = std::thread([this] { update_loop(); });
}

void MujocoLidar::close() {
  publish_lidar_ = false;
  if (thread_.joinable()) thread_.join();
}

void MujocoLidar::update_loop() {
  rclcpp::Rate rate(lidar_publish_rate_);
  while (rclcpp::ok() && publish_lidar_) {
    update();
    rate.sleep();
  }
}

void MujocoLidar::update() {
  {
    std::lock_guard<std::recursive_mutex> lock(*sim_mutex_);
    snapshot_.assign(mj_data_->sensordata, mj_data_->sensordata + mj_data_->nsensordata);
  }
  for (auto& lidar : lidar_sensors_) {
    auto& ranges = lidar.laser_scan_msg.ranges;
    for (size_t k = 0; k < lidar.sensor_indexes.size(); ++k) {
      const int adr = lidar.sensor_indexes[k];
      const double r = adr >= 0 && adr < static_cast<int>(snapshot_.size()) ? snapshot_[adr] : -1.0;
      // out-of-range readings (including MuJoCo's -1 "no hit") become -1 (reference :265-269)
      ranges[k] = static_cast<float>((r < lidar.range_min || r > lidar.range_max) ? -1.0 : r);
    }
  }
  for (auto& lidar : lidar_sensors_) {
    lidar.laser_scan_msg.header.stamp = node_->now();
    lidar.scan_pub->publish(lidar.laser_scan_msg);
  }
}

}  // namespace mujoco_ros2_control
