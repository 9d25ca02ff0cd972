// MujocoSystemInterface on the MI355X batch simulator (libmrs, include/mrs.h).
//
// Behaviour follows the reference plugin (src/mujoco_system_interface.cpp); line references below
// point at the reference.  Differences, all deliberate:
//  * physics is a GPU batch (env 0 is the robot); the physics thread advances it in fused launches
//    sized to catch up with the wall clock instead of one mj_step per loop iteration;
//  * read()/write() and the physics thread exchange data through a mutex-guarded double buffer (the
//    reference reads/writes mj_data_control_ without the lock);
//  * qfrc_applied is copied to the sim with length nv (the reference copies nu, :1689,1729);
//  * there is no Simulate UI: `headless` is accepted, a UI request is logged and ignored.
#include "mujoco_ros2_control/mujoco_system_interface.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>

#include "hardware_interface/lexical_casts.hpp"
#include "hardware_interface/types/hardware_interface_type_values.hpp"
#include "mujoco_ros2_control/ros_compat.hpp"
#include "mujoco_ros2_control/utils.hpp"

namespace mujoco_ros2_control {

namespace hi = hardware_interface;
using Clock = std::chrono::steady_clock;

namespace {

constexpr double kSyncMisalign = 0.1;       // s of sim time before re-sync (reference :55)
constexpr double kSimRefreshFraction = 0.7;  // share of a 60 Hz frame the loop may spend (reference :56)
constexpr double kRefreshRate = 60.0;

std::vector<double> parse_numbers(const std::string& s) {
  std::vector<double> v;
  std::stringstream ss(s);
  double x;
  while (ss >> x) v.push_back(x);
  return v;
}

// attribute value of the first <key ...> element of a keyframe file (start_positions.xml format)
std::optional<std::string> key_attribute(const std::string& text, const std::string& attr) {
  const auto k = text.find("<key");
  if (k == std::string::npos) return std::nullopt;
  const auto end = text.find('>', k);
  const std::string elem = text.substr(k, end == std::string::npos ? std::string::npos : end - k);
  size_t p = 0;
  while ((p = elem.find(attr, p)) != std::string::npos) {
    const bool boundary = p > 0 && std::isspace(static_cast<unsigned char>(elem[p - 1]));
    size_t q = p + attr.size();
    while (q < elem.size() && std::isspace(static_cast<unsigned char>(elem[q]))) ++q;
    if (boundary && q < elem.size() && elem[q] == '=') {
      const auto a = elem.find_first_of("\"'", q);
      if (a == std::string::npos) return std::nullopt;
      const auto b = elem.find(elem[a], a + 1);
      if (b == std::string::npos) return std::nullopt;
      return elem.substr(a + 1, b - a - 1);
    }
    p += attr.size();
  }
  return std::nullopt;
}

bool is_effort_name(const std::string& n) {
  return n == hi::HW_IF_EFFORT || n == hi::HW_IF_TORQUE || n == hi::HW_IF_FORCE;
}

}  // namespace

// ---- ROS parameter file (the --params-file the reference hands to rclcpp, :659-670), flattened to
// dotted names under ros__parameters: "pid_gains.position.joint1.p" -> "100.0".  Repeated keys at the
// same level merge, as rcl's YAML parser does (test/config/mujoco_pid.yaml repeats "pid_gains").
std::map<std::string, std::string> load_ros_params_file(const std::string& path) {
  std::ifstream f(path);
  std::map<std::string, std::string> out;
  std::vector<std::pair<int, std::string>> stack;  // (indent, key)
  std::string line;
  while (std::getline(f, line)) {
    auto hash = line.find('#');
    if (hash != std::string::npos) line = line.substr(0, hash);
    if (line.find_first_not_of(" \t\r") == std::string::npos) continue;
    const int indent = static_cast<int>(line.find_first_not_of(' '));
    std::string body = line.substr(indent);
    while (!body.empty() && (body.back() == ' ' || body.back() == '\r')) body.pop_back();
    const auto colon = body.find(':');
    if (colon == std::string::npos) continue;
    std::string key = body.substr(0, colon), value = body.substr(colon + 1);
    value.erase(0, value.find_first_not_of(' '));
    while (!stack.empty() && stack.back().first >= indent) stack.pop_back();
    if (value.empty()) {
      stack.emplace_back(indent, key);
      continue;
    }
    std::string name;
    bool under_params = false;
    for (auto& kv : stack) {
      if (kv.second == "ros__parameters") { under_params = true; name.clear(); continue; }
      if (under_params) name += kv.second + ".";
    }
    if (!under_params) continue;
    if (value.size() >= 2 && (value.front() == '"' || value.front() == '\'')) value = value.substr(1, value.size() - 2);
    out[name + key] = value;
  }
  return out;
}

MujocoSystemInterface::MujocoSystemInterface() = default;

MujocoSystemInterface::~MujocoSystemInterface() {
  if (cameras_) cameras_->close();
  if (lidar_sensors_) lidar_sensors_->close();
  exit_request_ = true;
  if (physics_thread_.joinable()) physics_thread_.join();
  if (batch_) mrs_batch_free(batch_);
  mj_deleteData(mj_data_);
  mj_deleteData(mj_data_control_);
  mj_deleteModel(mj_model_);
}

hi::CallbackReturn MujocoSystemInterface::on_init(const hi::HardwareComponentInterfaceParams& params) {
  if (hi::SystemInterface::on_init(params) != hi::CallbackReturn::SUCCESS) return hi::CallbackReturn::ERROR;
  const auto& hw = get_hardware_info().hardware_parameters;
  auto param = [&](const std::string& key) -> std::optional<std::string> {
    auto it = hw.find(key);
    if (it == hw.end()) return std::nullopt;
    return it->second;
  };

  model_path_ = param("mujoco_model").value_or("");
  sim_speed_factor_ = std::stod(param("sim_speed_factor").value_or("-1"));
  const double camera_publish_rate = std::stod(param("camera_publish_rate").value_or("5.0"));
  const double lidar_publish_rate = std::stod(param("lidar_publish_rate").value_or("5.0"));
  const bool headless = hi::parse_bool(param("headless").value_or("false"));
  if (!headless) RCLCPP_WARN(get_logger(), "The Simulate UI is not part of this build; running headless.");
  // additions (defaults reproduce the reference): GPU, batch size, threaded physics
  const int device = std::stoi(param("device").value_or("0"));
  const int num_envs = std::stoi(param("num_envs").value_or("1"));
  use_physics_thread_ = hi::parse_bool(param("physics_thread").value_or("true"));

  // ROS node with the PID parameter file (reference :653-675)
  const auto pids = param("pids_config_file");
  if (pids && !std::filesystem::exists(*pids)) {
    RCLCPP_FATAL(get_logger(), "PID config file '%s' does not exist!", pids->c_str());
    return hi::CallbackReturn::ERROR;
  }
  std::map<std::string, std::string> extra;
  if (auto desc = param("mujoco_robot_description")) extra["mujoco_robot_description"] = *desc;
  mujoco_node_ = compat::make_node("mujoco_node", pids, extra);

  // model: file, else the /mujoco_robot_description string (reference :415, :358-413)
  char err[1024] = "";
  mrs_model* compiled = nullptr;
  if (!model_path_.empty()) {
    compiled = mrs_model_load_xml(model_path_.c_str(), err, sizeof err);
  } else if (auto xml = compat::robot_description(mujoco_node_)) {
    compiled = mrs_model_load_xml_string(xml->c_str(), ".", err, sizeof err);
  } else {
    std::snprintf(err, sizeof err, "no 'mujoco_model' parameter and no /mujoco_robot_description");
  }
  if (!compiled) {
    load_error_ = err;
    RCLCPP_FATAL(get_logger(), "Failed to load the model: %s", err);
    return hi::CallbackReturn::ERROR;
  }
  mj_model_ = mj_wrapModel(compiled);
  model_ = compiled;
  view_ = *mj_model_;
  batch_ = mrs_batch_create(model_, std::max(1, num_envs), device);
  if (!batch_) {
    RCLCPP_FATAL(get_logger(), "Could not create the simulation batch: %s", mrs_last_error());
    return hi::CallbackReturn::ERROR;
  }
  mj_data_ = mj_makeData(mj_model_);
  mj_data_control_ = mj_makeData(mj_model_);
  {
    std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
    pull_state_locked();
  }

  register_joints(get_hardware_info());
  register_sensors(get_hardware_info());
  set_initial_pose();

  clock_publisher_ = mujoco_node_->create_publisher<rosgraph_msgs::msg::Clock>("/clock", 1);
  clock_realtime_publisher_ =
      std::make_shared<realtime_tools::RealtimePublisher<rosgraph_msgs::msg::Clock>>(clock_publisher_);

  cameras_ = std::make_unique<MujocoCameras>(mujoco_node_, &sim_mutex_, batch_, model_, camera_publish_rate);
  cameras_->register_cameras(get_hardware_info());
  lidar_sensors_ = std::make_unique<MujocoLidar>(mujoco_node_, &sim_mutex_, mj_data_, mj_model_, lidar_publish_rate);
  if (!lidar_sensors_->register_lidar(get_hardware_info())) {
    RCLCPP_INFO(get_logger(), "Failed to initialize lidar, exiting...");
    return hi::CallbackReturn::FAILURE;
  }

  {
    std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
    mrs_batch_forward(batch_);  // initial mj_forward (reference :741)
    mrs_batch_sync(batch_);
    pull_state_locked();
  }
  publish_clock();
  if (use_physics_thread_) physics_thread_ = std::thread([this] { PhysicsLoop(); });
  return hi::CallbackReturn::SUCCESS;
}

std::vector<hi::StateInterface> MujocoSystemInterface::export_state_interfaces() {
  std::vector<hi::StateInterface> out;
  for (auto& joint : joint_states_) {
    auto it = joint_hw_info_.find(joint.name);
    if (it == joint_hw_info_.end()) continue;
    for (const auto& si : it->second.state_interfaces) {
      if (si.name == hi::HW_IF_POSITION) out.emplace_back(joint.name, hi::HW_IF_POSITION, &joint.position);
      else if (si.name == hi::HW_IF_VELOCITY) out.emplace_back(joint.name, hi::HW_IF_VELOCITY, &joint.velocity);
      else if (is_effort_name(si.name)) out.emplace_back(joint.name, si.name, &joint.effort);
    }
  }
  for (auto& s : ft_sensor_data_) {
    auto it = sensors_hw_info_.find(s.name);
    if (it == sensors_hw_info_.end()) continue;
    const std::map<std::string, double*> slots = {
        {"force.x", &s.force.data.x()},   {"force.y", &s.force.data.y()},   {"force.z", &s.force.data.z()},
        {"torque.x", &s.torque.data.x()}, {"torque.y", &s.torque.data.y()}, {"torque.z", &s.torque.data.z()}};
    for (const auto& si : it->second.state_interfaces) {
      auto slot = slots.find(si.name);
      if (slot != slots.end()) out.emplace_back(s.name, si.name, slot->second);
    }
  }
  for (auto& s : imu_sensor_data_) {
    auto it = sensors_hw_info_.find(s.name);
    if (it == sensors_hw_info_.end()) continue;
    const std::map<std::string, double*> slots = {
        {"orientation.x", &s.orientation.data.x()},         {"orientation.y", &s.orientation.data.y()},
        {"orientation.z", &s.orientation.data.z()},         {"orientation.w", &s.orientation.data.w()},
        {"angular_velocity.x", &s.angular_velocity.data.x()}, {"angular_velocity.y", &s.angular_velocity.data.y()},
        {"angular_velocity.z", &s.angular_velocity.data.z()},
        {"linear_acceleration.x", &s.linear_acceleration.data.x()},
        {"linear_acceleration.y", &s.linear_acceleration.data.y()},
        {"linear_acceleration.z", &s.linear_acceleration.data.z()}};
    for (const auto& si : it->second.state_interfaces) {
      auto slot = slots.find(si.name);
      if (slot != slots.end()) { out.emplace_back(s.name, si.name, slot->second); continue; }
      // covariance interfaces "<field>_covariance<idx>" (reference :871-908), zeros
      const std::pair<const char*, std::vector<double>*> covs[] = {
          {"orientation_covariance", &s.orientation_covariance},
          {"angular_velocity_covariance", &s.angular_velocity_covariance},
          {"linear_acceleration_covariance", &s.linear_acceleration_covariance}};
      for (auto& cv : covs) {
        const std::string prefix = cv.first;
        if (si.name.rfind(prefix, 0) == 0 && si.name.size() > prefix.size()) {
          const size_t idx = std::stoul(si.name.substr(prefix.size() + (si.name[prefix.size()] == '_' ? 1 : 0)));
          if (idx < cv.second->size()) out.emplace_back(s.name, si.name, &(*cv.second)[idx]);
        }
      }
    }
  }
  return out;
}

std::vector<hi::CommandInterface> MujocoSystemInterface::export_command_interfaces() {
  std::vector<hi::CommandInterface> out;
  for (auto& joint : joint_states_) {
    auto it = joint_hw_info_.find(joint.name);
    if (it == joint_hw_info_.end()) continue;
    for (const auto& ci : it->second.command_interfaces) {
      if (ci.name.find(hi::HW_IF_POSITION) != std::string::npos) {
        if (joint.is_position_control_enabled || joint.is_position_pid_control_enabled)
          out.emplace_back(joint.name, hi::HW_IF_POSITION, &joint.position_command);
      } else if (ci.name.find(hi::HW_IF_VELOCITY) != std::string::npos) {
        if (joint.is_velocity_control_enabled || joint.is_velocity_pid_control_enabled)
          out.emplace_back(joint.name, hi::HW_IF_VELOCITY, &joint.velocity_command);
      } else if (is_effort_name(ci.name)) {
        if (joint.is_effort_control_enabled) out.emplace_back(joint.name, ci.name, &joint.effort_command);
      }
    }
  }
  return out;
}

hi::CallbackReturn MujocoSystemInterface::on_activate(const rclcpp_lifecycle::State&) {
  cameras_->init();
  lidar_sensors_->init();
  return hi::CallbackReturn::SUCCESS;
}

hi::CallbackReturn MujocoSystemInterface::on_deactivate(const rclcpp_lifecycle::State&) {
  return hi::CallbackReturn::SUCCESS;
}

hi::return_type MujocoSystemInterface::perform_command_mode_switch(const std::vector<std::string>& start,
                                                                   const std::vector<std::string>& stop) {
  auto apply = [this](const std::string& full, bool enable) {
    const auto slash = full.find('/');
    if (slash == std::string::npos) {
      RCLCPP_ERROR(get_logger(), "Invalid interface name format: %s", full.c_str());
      return;
    }
    const std::string joint_name = full.substr(0, slash), iface = full.substr(slash + 1);
    auto j = std::find_if(joint_states_.begin(), joint_states_.end(),
                          [&](const JointState& s) { return s.name == joint_name; });
    if (j == joint_states_.end()) {
      RCLCPP_WARN(get_logger(), "Joint %s not found in joint_states_", joint_name.c_str());
      return;
    }
    if (!enable) {
      if (iface == hi::HW_IF_POSITION) j->is_position_control_enabled = j->is_position_pid_control_enabled = false;
      else if (iface == hi::HW_IF_VELOCITY) j->is_velocity_control_enabled = j->is_velocity_pid_control_enabled = false;
      else if (is_effort_name(iface)) j->is_effort_control_enabled = false;
      return;
    }
    // one mode at a time: clear everything, then enable the requested one
    j->is_position_control_enabled = j->is_velocity_control_enabled = j->is_effort_control_enabled = false;
    j->is_position_pid_control_enabled = j->is_velocity_pid_control_enabled = false;
    if (iface == hi::HW_IF_POSITION) {
      if (j->actuator_type == ActuatorType::POSITION) j->is_position_control_enabled = true;
      else if (j->has_pos_pid) j->is_position_pid_control_enabled = true;
    } else if (iface == hi::HW_IF_VELOCITY) {
      if (j->actuator_type == ActuatorType::VELOCITY) j->is_velocity_control_enabled = true;
      else if (j->has_vel_pid) j->is_velocity_pid_control_enabled = true;
    } else if (is_effort_name(iface)) {
      j->is_effort_control_enabled = true;
    }
  };
  for (const auto& s : stop) apply(s, false);
  for (const auto& s : start) apply(s, true);
  return hi::return_type::OK;
}

hi::return_type MujocoSystemInterface::read(const rclcpp::Time&, const rclcpp::Duration&) {
  std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
  const mjData& c = *mj_data_control_;
  for (auto& j : joint_states_) {
    if (j.mj_pos_adr < 0) continue;
    j.position = c.qpos[j.mj_pos_adr];
    j.velocity = c.qvel[j.mj_vel_adr];
    j.effort = c.qfrc_actuator[j.mj_vel_adr];
  }
  for (auto& s : imu_sensor_data_) {
    const double* q = &c.sensordata[s.orientation.mj_sensor_index];  // framequat is (w, x, y, z)
    s.orientation.data.w() = q[0];
    s.orientation.data.x() = q[1];
    s.orientation.data.y() = q[2];
    s.orientation.data.z() = q[3];
    for (int k = 0; k < 3; ++k) {
      s.angular_velocity.data.v[k] = c.sensordata[s.angular_velocity.mj_sensor_index + k];
      s.linear_acceleration.data.v[k] = c.sensordata[s.linear_acceleration.mj_sensor_index + k];
    }
  }
  for (auto& s : ft_sensor_data_)  // MuJoCo reports the force the child exerts: negate (reference :1088-1094)
    for (int k = 0; k < 3; ++k) {
      s.force.data.v[k] = -c.sensordata[s.force.mj_sensor_index + k];
      s.torque.data.v[k] = -c.sensordata[s.torque.mj_sensor_index + k];
    }
  return hi::return_type::OK;
}

hi::return_type MujocoSystemInterface::write(const rclcpp::Time&, const rclcpp::Duration& period) {
  for (auto& j : joint_states_) {
    if (!j.is_mimic) continue;
    const JointState& src = joint_states_.at(j.mimicked_joint_index);
    j.position_command = j.mimic_multiplier * src.position_command;
    j.velocity_command = j.mimic_multiplier * src.velocity_command;
    j.effort_command = j.mimic_multiplier * src.effort_command;
  }
  std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
  for (auto& j : joint_states_) {
    if (j.mj_actuator_id == -1) continue;
    if (j.is_position_control_enabled) {
      mj_data_control_->ctrl[j.mj_actuator_id] = j.position_command;
    } else if (j.is_position_pid_control_enabled) {
      const double error = j.position_command - mj_data_->qpos[j.mj_pos_adr];  // live sim state (:1133)
      mj_data_control_->qfrc_applied[j.mj_vel_adr] = j.pos_pid->compute_command(error, period);
    } else if (j.is_velocity_control_enabled) {
      mj_data_control_->ctrl[j.mj_actuator_id] = j.velocity_command;
    } else if (j.is_velocity_pid_control_enabled) {
      const double error = j.velocity_command - mj_data_->qvel[j.mj_vel_adr];
      mj_data_control_->qfrc_applied[j.mj_vel_adr] = j.vel_pid->compute_command(error, period);
    } else if (j.is_effort_control_enabled) {
      mj_data_control_->ctrl[j.mj_actuator_id] = j.effort_command;
    }
  }
  return hi::return_type::OK;
}

void MujocoSystemInterface::register_joints(const hi::HardwareInfo& info) {
  joint_states_.resize(info.joints.size());
  bool override_start = false;
  auto it = info.hardware_parameters.find("override_start_position_file");
  if (it != info.hardware_parameters.end() && !it->second.empty()) {
    override_start = set_override_start_positions(it->second);
    if (!override_start)
      RCLCPP_ERROR(get_logger(), "Failed to load override start positions from %s. Falling back to urdf initial positions.",
                   it->second.c_str());
  }
  for (size_t k = 0; k < info.joints.size(); ++k) {
    const auto& joint = info.joints[k];
    const int jid = mrs_name2id(model_, MRS_OBJ_JOINT, joint.name.c_str());
    if (jid == -1) {
      RCLCPP_ERROR_STREAM(get_logger(), "Failed to find joint in mujoco model, joint name: " << joint.name);
      continue;
    }
    // actuator: first joint-transmission actuator on this joint, else one named like the joint
    int aid = -1;
    for (int a = 0; a < view_.nu && aid == -1; ++a)
      if (view_.actuator_trntype[a] == MRS_TRN_JOINT && view_.actuator_trnid[2 * a] == jid) aid = a;
    if (aid == -1) aid = mrs_name2id(model_, MRS_OBJ_ACTUATOR, joint.name.c_str());
    joint_hw_info_.insert({joint.name, joint});

    JointState& js = joint_states_[k];
    js = JointState();
    js.name = joint.name;
    js.mj_joint_type = view_.jnt_type[jid];
    js.mj_pos_adr = view_.jnt_qposadr[jid];
    js.mj_vel_adr = view_.jnt_dofadr[jid];
    js.mj_actuator_id = aid;

    if (auto m = joint.parameters.find("mimic"); m != joint.parameters.end()) {
      auto src = std::find_if(info.joints.begin(), info.joints.end(),
                              [&](const hi::ComponentInfo& c) { return c.name == m->second; });
      if (src == info.joints.end()) throw std::runtime_error("Mimicked joint '" + m->second + "' not found");
      js.is_mimic = true;
      js.mimicked_joint_index = static_cast<int>(std::distance(info.joints.begin(), src));
      auto mult = joint.parameters.find("multiplier");
      js.mimic_multiplier = mult != joint.parameters.end() ? std::stod(mult->second) : 1.0;
    }
    auto initial = [](const hi::InterfaceInfo& ii) { return ii.initial_value.empty() ? 0.0 : std::stod(ii.initial_value); };
    for (const auto& si : joint.state_interfaces) {
      if (si.name == hi::HW_IF_POSITION) js.position = override_start ? mj_data_->qpos[js.mj_pos_adr] : initial(si);
      else if (si.name == hi::HW_IF_VELOCITY) js.velocity = override_start ? mj_data_->qvel[js.mj_vel_adr] : initial(si);
      else if (is_effort_name(si.name)) js.effort = initial(si);
    }
    if (aid == -1) {
      RCLCPP_WARN_STREAM(get_logger(), "No actuator found for joint: " << joint.name);
      continue;
    }
    js.actuator_type = static_cast<ActuatorType>(mrs_actuator_type(model_, aid));
    const bool motor_like = js.actuator_type == ActuatorType::MOTOR || js.actuator_type == ActuatorType::CUSTOM;
    const double ctrl0 = override_start ? mj_data_->ctrl[aid] : 0.0;
    auto make_pid = [&](const std::string& kind) {
      auto pid = std::make_shared<control_toolbox::PidROS>(mujoco_node_, "pid_gains." + kind + "." + joint.name, "", false);
      const bool ok = pid->initialize_from_ros_parameters();
      return std::make_pair(pid, ok);
    };
    for (const auto& ci : joint.command_interfaces) {
      if (ci.name.find(hi::HW_IF_POSITION) != std::string::npos) {
        if (js.actuator_type == ActuatorType::POSITION) {
          js.is_position_control_enabled = true;
          js.position_command = override_start ? ctrl0 : js.position;
        } else {
          auto [pid, ok] = make_pid("position");
          js.pos_pid = pid;
          js.has_pos_pid = ok;
          if (ok) {
            js.is_position_pid_control_enabled = true;
            js.position_command = js.position;
          } else {
            RCLCPP_ERROR(get_logger(), "Position command interface for the joint : %s is not supported with velocity or motor actuator without defining the PIDs",
                         joint.name.c_str());
          }
        }
      } else if (ci.name.find(hi::HW_IF_VELOCITY) != std::string::npos) {
        if (js.actuator_type == ActuatorType::POSITION)
          RCLCPP_ERROR(get_logger(), "Velocity command interface for the joint : %s is not supported with position actuator",
                       joint.name.c_str());
        if (js.actuator_type == ActuatorType::VELOCITY) {
          js.is_velocity_control_enabled = true;
          js.velocity_command = override_start ? ctrl0 : js.velocity;
        } else if (motor_like) {
          auto [pid, ok] = make_pid("velocity");
          js.vel_pid = pid;
          js.has_vel_pid = ok;
          if (ok) {
            js.is_velocity_pid_control_enabled = true;
            js.velocity_command = js.velocity;
          } else {
            RCLCPP_ERROR(get_logger(), "Velocity command interface for the joint : %s is not supported with motor or custom actuator without defining the PIDs",
                         joint.name.c_str());
          }
        }
      } else if (ci.name.find(hi::HW_IF_EFFORT) != std::string::npos ||
                 ci.name.find(hi::HW_IF_TORQUE) != std::string::npos ||
                 ci.name.find(hi::HW_IF_FORCE) != std::string::npos) {
        if (motor_like) {
          js.is_effort_control_enabled = true;
          js.effort_command = override_start ? ctrl0 : js.effort;
        } else {
          RCLCPP_ERROR(get_logger(), "Effort command interface for the joint : %s is not supported with position or velocity actuator.Skipping it.",
                       joint.name.c_str());
        }
      }
    }
    if (!joint.command_interfaces.empty() && !js.is_position_control_enabled && !js.is_velocity_control_enabled &&
        !js.is_effort_control_enabled && !js.is_position_pid_control_enabled && !js.is_velocity_pid_control_enabled)
      throw std::runtime_error("Joint '" + joint.name + "' has an unsupported command interface for the specified MuJoCo actuator");
  }
  // the reference calls set_initial_pose() once per joint (:1440-1443); once after the loop is equivalent
  if (!override_start) set_initial_pose();
}

void MujocoSystemInterface::register_sensors(const hi::HardwareInfo& info) {
  for (const auto& sensor : info.sensors) {
    auto type_it = sensor.parameters.find("mujoco_type");
    if (type_it == sensor.parameters.end()) {
      RCLCPP_INFO_STREAM(get_logger(), "Not adding hardware interface for sensor in ros2_control xacro: " << sensor.name);
      continue;
    }
    // suffix parameters: the sensor's own block first, then the hardware block (where the reference
    // looks them up, :1449-1457)
    auto suffix = [&](const std::string& key, const std::string& def) {
      if (auto s = sensor.parameters.find(key); s != sensor.parameters.end()) return s->second;
      if (auto h = info.hardware_parameters.find(key); h != info.hardware_parameters.end()) return h->second;
      return def;
    };
    auto mj_name_it = sensor.parameters.find("mujoco_sensor_name");
    const std::string base = mj_name_it == sensor.parameters.end() ? sensor.name : mj_name_it->second;
    sensors_hw_info_.insert({sensor.name, sensor});
    auto adr = [&](const std::string& n) {
      const int id = mrs_name2id(model_, MRS_OBJ_SENSOR, n.c_str());
      return id < 0 ? -1 : view_.sensor_adr[id];
    };
    if (type_it->second == "fts") {
      FTSensorData d;
      d.name = sensor.name;
      d.force.name = base + suffix("force_mjcf_suffix", "_force");
      d.torque.name = base + suffix("torque_mjcf_suffix", "_torque");
      d.force.mj_sensor_index = adr(d.force.name);
      d.torque.mj_sensor_index = adr(d.torque.name);
      if (d.force.mj_sensor_index < 0 || d.torque.mj_sensor_index < 0) {
        RCLCPP_ERROR_STREAM(get_logger(), "Failed to find force/torque sensor in mujoco model, sensor name: " << sensor.name);
        continue;
      }
      ft_sensor_data_.push_back(d);
    } else if (type_it->second == "imu") {
      IMUSensorData d;
      d.name = sensor.name;
      d.orientation.name = base + suffix("orientation_mjcf_suffix", "_quat");
      d.angular_velocity.name = base + suffix("angular_velocity_mjcf_suffix", "_gyro");
      d.linear_acceleration.name = base + suffix("linear_acceleration_mjcf_suffix", "_accel");
      d.orientation_covariance.assign(9, 0.0);
      d.angular_velocity_covariance.assign(9, 0.0);
      d.linear_acceleration_covariance.assign(9, 0.0);
      d.orientation.mj_sensor_index = adr(d.orientation.name);
      d.angular_velocity.mj_sensor_index = adr(d.angular_velocity.name);
      d.linear_acceleration.mj_sensor_index = adr(d.linear_acceleration.name);
      if (d.orientation.mj_sensor_index < 0 || d.angular_velocity.mj_sensor_index < 0 ||
          d.linear_acceleration.mj_sensor_index < 0) {
        RCLCPP_ERROR_STREAM(get_logger(), "Failed to find IMU sensor in mujoco model, sensor name: " << sensor.name);
        continue;
      }
      imu_sensor_data_.push_back(d);
    } else {
      RCLCPP_ERROR_STREAM(get_logger(), "Invalid mujoco_type passed to the mujoco hardware interface: " << type_it->second);
    }
  }
}

bool MujocoSystemInterface::set_override_start_positions(const std::string& file) {
  std::ifstream f(file);
  if (!f) {
    RCLCPP_ERROR_STREAM(get_logger(), "Failed to load override start position file " << file << ".");
    return false;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  if (text.find("<key") == std::string::npos) {
    RCLCPP_ERROR_STREAM(get_logger(), "<key> element not found in override start position file.");
    return false;
  }
  std::vector<double> v[3];
  const char* names[3] = {"qpos", "qvel", "ctrl"};
  for (int i = 0; i < 3; ++i) {
    auto a = key_attribute(text, names[i]);
    if (!a) {
      RCLCPP_ERROR_STREAM(get_logger(), "Attribute '" << names[i] << "' not found in override start position file.");
      return false;
    }
    v[i] = parse_numbers(*a);
  }
  if (v[0].empty() || v[1].empty() || v[2].empty()) return false;
  if (v[0].size() != static_cast<size_t>(view_.nq) || v[1].size() != static_cast<size_t>(view_.nv) ||
      v[2].size() != static_cast<size_t>(view_.nu)) {
    RCLCPP_ERROR_STREAM(get_logger(), "Mismatch in data types in override starting positions. Numbers are: qpos "
                                          << v[0].size() << "/" << view_.nq << ", qvel " << v[1].size() << "/"
                                          << view_.nv << ", ctrl " << v[2].size() << "/" << view_.nu);
    return false;
  }
  std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
  std::copy(v[0].begin(), v[0].end(), mj_data_->qpos);
  std::copy(v[1].begin(), v[1].end(), mj_data_->qvel);
  std::copy(v[2].begin(), v[2].end(), mj_data_->ctrl);
  std::copy(v[2].begin(), v[2].end(), mj_data_control_->ctrl);
  mrs_batch_set_field(batch_, MRS_FIELD_QPOS, mj_data_->qpos, 0, 1);
  mrs_batch_set_field(batch_, MRS_FIELD_QVEL, mj_data_->qvel, 0, 1);
  mrs_batch_set_field(batch_, MRS_FIELD_CTRL, mj_data_->ctrl, 0, 1);
  return true;
}

void MujocoSystemInterface::set_initial_pose() {
  std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
  for (const auto& j : joint_states_)
    if (j.mj_pos_adr >= 0) mj_data_->qpos[j.mj_pos_adr] = j.position;
  mrs_batch_set_field(batch_, MRS_FIELD_QPOS, mj_data_->qpos, 0, 1);
  mrs_batch_forward(batch_);
  mrs_batch_sync(batch_);
  pull_state_locked();
}

void MujocoSystemInterface::pull_state_locked() {
  mrs_batch_get_field(batch_, MRS_FIELD_QPOS, mj_data_->qpos, 0, 1);
  mrs_batch_get_field(batch_, MRS_FIELD_QVEL, mj_data_->qvel, 0, 1);
  mrs_batch_get_field(batch_, MRS_FIELD_QFRC_ACTUATOR, mj_data_->qfrc_actuator, 0, 1);
  if (view_.nsensordata > 0) mrs_batch_get_field(batch_, MRS_FIELD_SENSORDATA, mj_data_->sensordata, 0, 1);
  if (view_.nv > 0) {
    mrs_batch_get_field(batch_, MRS_FIELD_QACC, mj_data_->qacc, 0, 1);
    mrs_batch_get_field(batch_, MRS_FIELD_QACC_WARMSTART, mj_data_->qacc_warmstart, 0, 1);
  }
  mrs_batch_get_field(batch_, MRS_FIELD_TIME, &mj_data_->time, 0, 1);
  // sim -> control copy of the outputs (mj_copyData(control <- sim), reference :1759); the control
  // inputs ctrl / qfrc_applied stay what write() put there
  const mjData& d = *mj_data_;
  mjData& c = *mj_data_control_;
  std::copy(d.qpos, d.qpos + d.nq, c.qpos);
  std::copy(d.qvel, d.qvel + d.nv, c.qvel);
  std::copy(d.qacc, d.qacc + d.nv, c.qacc);
  std::copy(d.qacc_warmstart, d.qacc_warmstart + d.nv, c.qacc_warmstart);
  std::copy(d.qfrc_actuator, d.qfrc_actuator + d.nv, c.qfrc_actuator);
  std::copy(d.sensordata, d.sensordata + d.nsensordata, c.sensordata);
  c.time = d.time;
}

bool MujocoSystemInterface::advance_locked(int n) {
  // control -> sim (reference :1688-1689, with nv for qfrc_applied)
  std::copy(mj_data_control_->ctrl, mj_data_control_->ctrl + view_.nu, mj_data_->ctrl);
  std::copy(mj_data_control_->qfrc_applied, mj_data_control_->qfrc_applied + view_.nv, mj_data_->qfrc_applied);
  if (view_.nu > 0) mrs_batch_set_field(batch_, MRS_FIELD_CTRL, mj_data_->ctrl, 0, 1);
  if (view_.nv > 0) mrs_batch_set_field(batch_, MRS_FIELD_QFRC_APPLIED, mj_data_->qfrc_applied, 0, 1);
  double before[4], after[4];
  mrs_batch_get_field(batch_, MRS_FIELD_WARNING, before, 0, 1);
  if (mrs_batch_step(batch_, n) != MRS_OK || mrs_batch_sync(batch_) != MRS_OK) {
    RCLCPP_ERROR(get_logger(), "batch step failed: %s", mrs_last_error());
    return false;
  }
  mrs_batch_get_field(batch_, MRS_FIELD_WARNING, after, 0, 1);
  pull_state_locked();
  // Diverged() (reference :281-294): only reported when auto-reset is disabled
  if ((view_.disableflags & MRS_DSBL_AUTORESET) &&
      (after[0] > before[0] || after[1] > before[1] || after[2] > before[2])) {
    load_error_ = "Simulation diverged (bad qpos/qvel/qacc); paused";
    return false;
  }
  return true;
}

void MujocoSystemInterface::PhysicsLoop() {
  Clock::time_point sync_cpu{};
  double sync_sim = 0;
  bool synced = false;
  const double h = view_.timestep;
  while (!exit_request_) {
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
    {
      std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
      if (run_) {
        const auto start_cpu = Clock::now();
        const double elapsed_cpu = std::chrono::duration<double>(start_cpu - sync_cpu).count();
        const double elapsed_sim = mj_data_->time - sync_sim;
        const double slowdown = sim_speed_factor_ > 0 ? 1.0 / sim_speed_factor_ : 1.0;  // UI default 100%
        const bool misaligned = std::abs(elapsed_cpu / slowdown - elapsed_sim) > kSyncMisalign;
        int n = 0;
        if (!synced || elapsed_sim < 0 || misaligned) {
          // out of sync: re-sync and take one step (reference :1679-1703)
          sync_cpu = start_cpu;
          sync_sim = mj_data_->time;
          synced = true;
          n = 1;
        } else {
          // in sync: the steps that bring sim time level with the paced wall clock, within the
          // refresh budget (reference :1715-1752 steps them one by one; here one fused launch)
          const double lag = elapsed_cpu / slowdown - elapsed_sim;
          const double budget = kSimRefreshFraction / kRefreshRate / slowdown;
          n = static_cast<int>(std::ceil(std::min(lag, budget) / h - 1e-9));
        }
        if (n > 0 && !advance_locked(n)) run_ = false;
      } else {
        mrs_batch_forward(batch_);  // paused: keep outputs fresh (reference :1766-1773)
        mrs_batch_sync(batch_);
        pull_state_locked();
      }
    }
    publish_clock();
  }
}

bool MujocoSystemInterface::step_physics(int n) {
  bool ok;
  {
    std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
    ok = advance_locked(n);
  }
  publish_clock();
  return ok;
}

double MujocoSystemInterface::sim_time() const {
  std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
  return mj_data_->time;
}

void MujocoSystemInterface::publish_clock() {
  const double t = sim_time();
  const int32_t sec = static_cast<int32_t>(std::floor(t));
  const uint32_t nsec = static_cast<uint32_t>((t - sec) * 1e9);
  rosgraph_msgs::msg::Clock msg;
  msg.clock = rclcpp::Time(sec, nsec);
  compat::set_sim_time(mujoco_node_, msg.clock);
  clock_realtime_publisher_->try_publish(msg);
}

void MujocoSystemInterface::get_model(mjModel*& dest) {
  std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
  dest = mj_copyModel(dest, mj_model_);
}

void MujocoSystemInterface::get_data(mjData*& dest) {
  std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
  if (dest == nullptr) dest = mj_makeData(mj_model_);
  mj_copyData(dest, mj_model_, mj_data_);
}

// mj_copyData(mj_data_ <- mj_data) (reference :1810-1814), then the arrays go to env 0 and a forward
// pass recomputes the outputs (qacc, qfrc_actuator, sensordata) from the new state
void MujocoSystemInterface::set_data(mjData* mj_data) {
  std::lock_guard<std::recursive_mutex> lock(sim_mutex_);
  if (!mj_copyData(mj_data_, mj_model_, mj_data)) {
    RCLCPP_ERROR(get_logger(), "set_data: mjData was made for a different model");
    return;
  }
  mrs_batch_set_field(batch_, MRS_FIELD_QPOS, mj_data_->qpos, 0, 1);
  if (view_.nv > 0) {
    mrs_batch_set_field(batch_, MRS_FIELD_QVEL, mj_data_->qvel, 0, 1);
    mrs_batch_set_field(batch_, MRS_FIELD_QACC_WARMSTART, mj_data_->qacc_warmstart, 0, 1);
    mrs_batch_set_field(batch_, MRS_FIELD_QFRC_APPLIED, mj_data_->qfrc_applied, 0, 1);
  }
  if (view_.nu > 0) mrs_batch_set_field(batch_, MRS_FIELD_CTRL, mj_data_->ctrl, 0, 1);
  mrs_batch_set_field(batch_, MRS_FIELD_TIME, &mj_data_->time, 0, 1);
  mrs_batch_forward(batch_);
  mrs_batch_sync(batch_);
  pull_state_locked();
}

}  // namespace mujoco_ros2_control

#ifdef MRS_WITH_ROS
#include <pluginlib/class_list_macros.hpp>
// class name "mujoco_ros2_control/MujocoSystemInterface" (csrc/plugin/mujoco_system_interface_plugin.xml)
PLUGINLIB_EXPORT_CLASS(mujoco_ros2_control::MujocoSystemInterface, hardware_interface::SystemInterface)
#endif
