// C entry points of the plugin host (include/mrs_plugin.h): URDF <ros2_control> parsing with the
// xacro subset the reference's test robot uses, lifecycle and read/write driving.
#include "mrs_plugin.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../mjcf/xml.h"
#include "mujoco_ros2_control/mujoco_system_interface.hpp"
#include "mujoco_ros2_control/utils.hpp"

namespace hi = hardware_interface;
using mujoco_ros2_control::MujocoSystemInterface;

struct mrsp_system {
  hi::HardwareInfo info;
  std::unique_ptr<MujocoSystemInterface> plugin;
  std::vector<hi::StateInterface> states;
  std::vector<hi::CommandInterface> commands;
};

namespace {

thread_local std::string g_error;

int fail(const std::string& msg, int code = -1) {
  g_error = msg;
  return code;
}

int copy_out(const std::string& s, char* buf, int len) {
  if (!buf || len <= 0) return static_cast<int>(s.size());
  std::snprintf(buf, static_cast<size_t>(len), "%s", s.c_str());
  return static_cast<int>(s.size());
}

std::map<std::string, std::string> split_pairs(const char* text, char sep, const std::string& assign) {
  std::map<std::string, std::string> out;
  if (!text) return out;
  std::string s(text), item;
  std::stringstream ss(s);
  while (std::getline(ss, item, sep)) {
    const auto p = item.find(assign);
    if (item.find_first_not_of(" \t") == std::string::npos || p == std::string::npos) continue;
    auto trim = [](std::string t) {
      t.erase(0, t.find_first_not_of(" \t"));
      t.erase(t.find_last_not_of(" \t") + 1);
      return t;
    };
    out[trim(item.substr(0, p))] = trim(item.substr(p + assign.size()));
  }
  return out;
}

// $(arg x) and $(find pkg) substitution (xacro's substitution_args subset)
struct Xacro {
  std::map<std::string, std::string> args, packages;
  std::string subst(const std::string& in) const {
    std::string out;
    size_t i = 0;
    while (i < in.size()) {
      const auto a = in.find("$(", i);
      if (a == std::string::npos) { out += in.substr(i); break; }
      out += in.substr(i, a - i);
      const auto b = in.find(')', a);
      if (b == std::string::npos) throw std::runtime_error("unterminated $( in '" + in + "'");
      std::stringstream ss(in.substr(a + 2, b - a - 2));
      std::string verb, name;
      ss >> verb >> name;
      if (verb == "arg") {
        auto it = args.find(name);
        if (it == args.end()) throw std::runtime_error("undefined substitution argument " + name);
        out += it->second;
      } else if (verb == "find") {
        auto it = packages.find(name);
        if (it == packages.end()) throw std::runtime_error("package not found: " + name);
        out += it->second;
      } else {
        throw std::runtime_error("unsupported substitution $(" + verb + ")");
      }
      i = b + 1;
    }
    return out;
  }
  bool truth(const std::string& v) const {
    const std::string s = subst(v);
    if (s == "true" || s == "True" || s == "1") return true;
    if (s == "false" || s == "False" || s == "0") return false;
    throw std::runtime_error("xacro:if value must be a boolean, got '" + s + "'");
  }
  // children with xacro:if / xacro:unless resolved in place
  void expand(const mrs::XmlElement& e, std::vector<const mrs::XmlElement*>& out) const {
    for (const auto& c : e.children) {
      if (c->tag == "xacro:if" || c->tag == "xacro:unless") {
        const std::string* v = c->attr("value");
        if (!v) throw std::runtime_error(c->tag + " without value");
        if (truth(*v) == (c->tag == "xacro:if")) expand(*c, out);
      } else {
        out.push_back(c.get());
      }
    }
  }
  std::vector<const mrs::XmlElement*> kids(const mrs::XmlElement& e) const {
    std::vector<const mrs::XmlElement*> out;
    expand(e, out);
    return out;
  }
};

// <command_interface>/<state_interface> (hardware_interface component_parser semantics)
hi::InterfaceInfo parse_interface(const Xacro& x, const mrs::XmlElement& e) {
  hi::InterfaceInfo ii;
  if (const auto* n = e.attr("name")) ii.name = x.subst(*n);
  for (const auto* p : x.kids(e)) {
    if (p->tag != "param") continue;
    const auto* n = p->attr("name");
    if (!n) continue;
    const std::string key = x.subst(*n), val = x.subst(p->text);
    if (key == "min") ii.min = val;
    else if (key == "max") ii.max = val;
    else if (key == "initial_value") ii.initial_value = val;
    else if (key == "data_type") ii.data_type = val;
    else if (key == "size") ii.size = std::stoi(val);
    else ii.parameters[key] = val;
  }
  return ii;
}

hi::ComponentInfo parse_component(const Xacro& x, const mrs::XmlElement& e) {
  hi::ComponentInfo c;
  if (const auto* n = e.attr("name")) c.name = x.subst(*n);
  c.type = e.tag;
  for (const auto* k : x.kids(e)) {
    if (k->tag == "command_interface") c.command_interfaces.push_back(parse_interface(x, *k));
    else if (k->tag == "state_interface") c.state_interfaces.push_back(parse_interface(x, *k));
    else if (k->tag == "param" && k->attr("name")) c.parameters[x.subst(*k->attr("name"))] = x.subst(k->text);
  }
  return c;
}

const mrs::XmlElement* find_tag(const Xacro& x, const mrs::XmlElement& e, const std::string& tag) {
  for (const auto* k : x.kids(e)) {
    if (k->tag == tag) return k;
    if (const auto* d = find_tag(x, *k, tag)) return d;
  }
  return nullptr;
}

}  // namespace

extern "C" {

const char* mrsp_last_error(void) { return g_error.c_str(); }

mrsp_system* mrsp_load_urdf(const char* urdf_path, const char* xacro_args, const char* package_dirs) {
  try {
    auto root = mrs::xml_parse(mrs::read_file(urdf_path), urdf_path);
    Xacro x;
    x.packages = split_pairs(package_dirs, ';', "=");
    for (const auto& c : root->children)
      if (c->tag == "xacro:arg" && c->attr("name"))
        x.args[*c->attr("name")] = c->attr("default") ? *c->attr("default") : "";
    for (auto& kv : split_pairs(xacro_args, ' ', ":=")) x.args[kv.first] = kv.second;
    const mrs::XmlElement* rc = find_tag(x, *root, "ros2_control");
    if (!rc) throw std::runtime_error("no <ros2_control> block in " + std::string(urdf_path));
    auto s = std::make_unique<mrsp_system>();
    s->info.name = rc->attr("name") ? x.subst(*rc->attr("name")) : "";
    s->info.type = rc->attr("type") ? x.subst(*rc->attr("type")) : "";
    for (const auto* k : x.kids(*rc)) {
      if (k->tag == "hardware") {
        for (const auto* h : x.kids(*k)) {
          if (h->tag == "plugin") s->info.hardware_plugin_name = x.subst(h->text);
          else if (h->tag == "param" && h->attr("name"))
            s->info.hardware_parameters[x.subst(*h->attr("name"))] = x.subst(h->text);
        }
      } else if (k->tag == "joint") {
        s->info.joints.push_back(parse_component(x, *k));
      } else if (k->tag == "sensor") {
        s->info.sensors.push_back(parse_component(x, *k));
      } else if (k->tag == "gpio") {
        s->info.gpios.push_back(parse_component(x, *k));
      }
    }
    return s.release();
  } catch (const std::exception& e) {
    fail(e.what());
    return nullptr;
  }
}

void mrsp_free(mrsp_system* s) { delete s; }

int mrsp_set_hardware_param(mrsp_system* s, const char* key, const char* value) {
  if (!s || !key || !value) return fail("null argument");
  s->info.hardware_parameters[key] = value;
  return 0;
}

int mrsp_get_hardware_param(const mrsp_system* s, const char* key, char* buf, int len) {
  if (!s || !key) return fail("null argument");
  auto it = s->info.hardware_parameters.find(key);
  if (it == s->info.hardware_parameters.end()) return fail(std::string("no hardware parameter ") + key);
  return copy_out(it->second, buf, len);
}

int mrsp_num_joints(const mrsp_system* s) { return s ? static_cast<int>(s->info.joints.size()) : -1; }
int mrsp_num_sensors(const mrsp_system* s) { return s ? static_cast<int>(s->info.sensors.size()) : -1; }

int mrsp_on_init(mrsp_system* s) {
  if (!s) return fail("null system");
  try {
    s->plugin = std::make_unique<MujocoSystemInterface>();
    hi::HardwareComponentInterfaceParams params;
    params.hardware_info = s->info;
    const auto r = s->plugin->on_init(params);
    if (r == hi::CallbackReturn::SUCCESS) {
      s->states = s->plugin->export_state_interfaces();
      s->commands = s->plugin->export_command_interfaces();
    }
    return static_cast<int>(r);
  } catch (const std::exception& e) {
    return fail(e.what());
  }
}

#define NEED_PLUGIN(s) \
  if (!(s) || !(s)->plugin) return fail("plugin not initialised")

int mrsp_on_activate(mrsp_system* s) {
  NEED_PLUGIN(s);
  return static_cast<int>(s->plugin->on_activate(rclcpp_lifecycle::State()));
}

int mrsp_num_state_interfaces(const mrsp_system* s) { return s ? static_cast<int>(s->states.size()) : -1; }
int mrsp_num_command_interfaces(const mrsp_system* s) { return s ? static_cast<int>(s->commands.size()) : -1; }

int mrsp_state_interface_name(const mrsp_system* s, int i, char* buf, int len) {
  if (!s || i < 0 || i >= static_cast<int>(s->states.size())) return fail("state interface index out of range");
  return copy_out(s->states[i].get_name(), buf, len);
}

int mrsp_command_interface_name(const mrsp_system* s, int i, char* buf, int len) {
  if (!s || i < 0 || i >= static_cast<int>(s->commands.size())) return fail("command interface index out of range");
  return copy_out(s->commands[i].get_name(), buf, len);
}

double mrsp_get_state(const mrsp_system* s, int i) {
  if (!s || i < 0 || i >= static_cast<int>(s->states.size())) return fail("index out of range"), 0.0 / 0.0;
  return s->states[i].get_value();
}

double mrsp_get_command(const mrsp_system* s, int i) {
  if (!s || i < 0 || i >= static_cast<int>(s->commands.size())) return fail("index out of range"), 0.0 / 0.0;
  return s->commands[i].get_value();
}

int mrsp_set_command(mrsp_system* s, int i, double value) {
  if (!s || i < 0 || i >= static_cast<int>(s->commands.size())) return fail("command interface index out of range");
  s->commands[i].set_value(value);
  return 0;
}

int mrsp_switch_mode(mrsp_system* s, const char* start, const char* stop) {
  NEED_PLUGIN(s);
  auto split = [](const char* t) {
    std::vector<std::string> v;
    std::string item;
    std::stringstream ss(t ? t : "");
    while (std::getline(ss, item, ';'))
      if (!item.empty()) v.push_back(item);
    return v;
  };
  return static_cast<int>(s->plugin->perform_command_mode_switch(split(start), split(stop)));
}

int mrsp_read(mrsp_system* s) {
  NEED_PLUGIN(s);
  return static_cast<int>(s->plugin->read(rclcpp::Time(), rclcpp::Duration()));
}

int mrsp_write(mrsp_system* s, double period_s) {
  NEED_PLUGIN(s);
  return static_cast<int>(s->plugin->write(rclcpp::Time(), rclcpp::Duration::from_seconds(period_s)));
}

int mrsp_step(mrsp_system* s, int n_steps) {
  NEED_PLUGIN(s);
  try {
    return s->plugin->step_physics(n_steps) ? 0 : 1;
  } catch (const std::exception& e) {
    return fail(e.what());
  }
}

double mrsp_sim_time(const mrsp_system* s) { return s && s->plugin ? s->plugin->sim_time() : -1.0; }

int mrsp_get_model(mrsp_system* s, int* sizes, double* timestep) {
  if (!s || !s->plugin) return fail("plugin not initialised");
  mjModel* m = nullptr;
  s->plugin->get_model(m);
  if (!m) return fail("get_model failed");
  if (sizes) {
    sizes[0] = m->nq;
    sizes[1] = m->nv;
    sizes[2] = m->nu;
    sizes[3] = m->nsensordata;
  }
  if (timestep) *timestep = m->opt.timestep;
  mj_deleteModel(m);
  return 0;
}

int mrsp_get_data(mrsp_system* s, double* qpos, double* qvel, double* ctrl, double* sensordata, double* time) {
  if (!s || !s->plugin) return fail("plugin not initialised");
  mjData* d = nullptr;
  s->plugin->get_data(d);
  if (!d) return fail("get_data failed");
  if (qpos) std::copy(d->qpos, d->qpos + d->nq, qpos);
  if (qvel) std::copy(d->qvel, d->qvel + d->nv, qvel);
  if (ctrl) std::copy(d->ctrl, d->ctrl + d->nu, ctrl);
  if (sensordata) std::copy(d->sensordata, d->sensordata + d->nsensordata, sensordata);
  if (time) *time = d->time;
  mj_deleteData(d);
  return 0;
}

int mrsp_set_data(mrsp_system* s, const double* qpos, const double* qvel, double time) {
  if (!s || !s->plugin) return fail("plugin not initialised");
  mjData* d = nullptr;
  s->plugin->get_data(d);
  if (!d) return fail("get_data failed");
  if (qpos) std::copy(qpos, qpos + d->nq, d->qpos);
  if (qvel) std::copy(qvel, qvel + d->nv, d->qvel);
  d->time = time;
  s->plugin->set_data(d);
  mj_deleteData(d);
  return 0;
}

double mrsp_clock(const mrsp_system* s, long* count) {
  if (!s || !s->plugin) return -1.0;
  auto pub = s->plugin->node()->find_publisher<rosgraph_msgs::msg::Clock>("/clock");
  if (!pub) return -1.0;
  if (count) *count = static_cast<long>(pub->count());
  auto m = pub->last();
  return m ? m->clock.seconds() : -1.0;
}

int mrsp_lidar_update(mrsp_system* s) {
  NEED_PLUGIN(s);
  s->plugin->lidar()->update();
  return 0;
}

int mrsp_last_scan(const mrsp_system* s, const char* topic, float* ranges, int max, float* meta) {
  NEED_PLUGIN(s);
  auto pub = s->plugin->node()->find_publisher<sensor_msgs::msg::LaserScan>(topic);
  if (!pub) return fail(std::string("no publisher on ") + topic);
  auto m = pub->last();
  if (!m) return fail(std::string("nothing published on ") + topic);
  const int n = static_cast<int>(m->ranges.size());
  if (ranges) std::memcpy(ranges, m->ranges.data(), sizeof(float) * std::min(n, max));
  if (meta) {
    const float v[7] = {m->angle_min, m->angle_max, m->angle_increment, m->range_min,
                        m->range_max, m->scan_time, m->time_increment};
    std::memcpy(meta, v, sizeof v);
  }
  return n;
}

int mrsp_camera_update(mrsp_system* s) {
  NEED_PLUGIN(s);
  s->plugin->cameras()->update();
  return 0;
}

int mrsp_last_depth(const mrsp_system* s, const char* topic, float* depth, int max, int* wh) {
  NEED_PLUGIN(s);
  auto pub = s->plugin->node()->find_publisher<sensor_msgs::msg::Image>(topic);
  if (!pub) return fail(std::string("no publisher on ") + topic);
  auto m = pub->last();
  if (!m) return fail(std::string("nothing published on ") + topic);
  const int n = static_cast<int>(m->data.size() / sizeof(float));
  if (depth) std::memcpy(depth, m->data.data(), sizeof(float) * std::min(n, max));
  if (wh) { wh[0] = static_cast<int>(m->width); wh[1] = static_cast<int>(m->height); }
  return n;
}

int mrsp_last_camera_info(const mrsp_system* s, const char* topic, double* k9, double* p12, int* wh) {
  NEED_PLUGIN(s);
  auto pub = s->plugin->node()->find_publisher<sensor_msgs::msg::CameraInfo>(topic);
  if (!pub) return fail(std::string("no publisher on ") + topic);
  auto m = pub->last();
  if (!m) return fail(std::string("nothing published on ") + topic);
  if (k9) std::memcpy(k9, m->k.data(), sizeof(double) * 9);
  if (p12) std::memcpy(p12, m->p.data(), sizeof(double) * 12);
  if (wh) { wh[0] = static_cast<int>(m->width); wh[1] = static_cast<int>(m->height); }
  return 0;
}

int mrsp_last_image(const mrsp_system* s, const char* topic, int* wh_step, char* encoding, int len) {
  NEED_PLUGIN(s);
  auto pub = s->plugin->node()->find_publisher<sensor_msgs::msg::Image>(topic);
  if (!pub) return fail(std::string("no publisher on ") + topic);
  auto m = pub->last();
  if (!m) return fail(std::string("nothing published on ") + topic);
  if (wh_step) { wh_step[0] = static_cast<int>(m->width); wh_step[1] = static_cast<int>(m->height); wh_step[2] = static_cast<int>(m->step); }
  copy_out(m->encoding, encoding, len);
  return static_cast<int>(m->data.size());
}

int mrsp_last_image_data(const mrsp_system* s, const char* topic, unsigned char* out, int max) {
  NEED_PLUGIN(s);
  auto pub = s->plugin->node()->find_publisher<sensor_msgs::msg::Image>(topic);
  if (!pub) return fail(std::string("no publisher on ") + topic);
  auto m = pub->last();
  if (!m) return fail(std::string("nothing published on ") + topic);
  const int n = static_cast<int>(m->data.size());
  if (out) std::memcpy(out, m->data.data(), static_cast<size_t>(std::min(n, std::max(max, 0))));
  return n;
}

int mrsp_parse_lidar_name(const char* sensor_name, char* buf, int len) {
  if (!sensor_name) return fail("null name");
  const auto [name, idx] = mujoco_ros2_control::parse_lidar_name(sensor_name);
  copy_out(name, buf, len);
  return idx;
}

int mrsp_lidar_config(const mrsp_system* s, const char* name, double* out, char* topic, int len) {
  if (!s || !name) return fail("null argument");
  try {
    auto d = mujoco_ros2_control::get_lidar_data(s->info, name);
    if (!d) return fail(std::string("lidar ") + name + ": missing sensor or required parameter");
    if (out) {
      const double v[6] = {d->min_angle, d->max_angle, d->angle_increment, d->range_min, d->range_max,
                           static_cast<double>(d->num_rangefinders)};
      std::memcpy(out, v, sizeof v);
    }
    copy_out(d->laserscan_topic, topic, len);
    return 0;
  } catch (const std::exception& e) {
    return fail(e.what());
  }
}

int mrsp_ros_param(const char* params_file, const char* key, char* buf, int len) {
  if (!params_file || !key) return fail("null argument");
  const auto params = mujoco_ros2_control::load_ros_params_file(params_file);
  auto it = params.find(key);
  if (it == params.end()) return fail(std::string("no parameter ") + key);
  return copy_out(it->second, buf, len);
}

struct mrs_batch* mrsp_batch(mrsp_system* s) { return s && s->plugin ? s->plugin->batch() : nullptr; }

}  // extern "C"
