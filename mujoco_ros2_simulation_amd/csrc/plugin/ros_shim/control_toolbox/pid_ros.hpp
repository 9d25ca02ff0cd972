// ros_shim: control_toolbox::PidROS subset (gains from "<prefix>.{p,i,d,u_clamp_*,i_clamp_*}"
// node parameters, legacy anti-windup: clamped integral, clamped output).
#pragma once
#include <algorithm>
#include <cmath>
#include <limits>
#include <memory>
#include <string>
#include "rclcpp/rclcpp.hpp"

namespace control_toolbox {

struct AntiWindupStrategy {
  double i_max = std::numeric_limits<double>::infinity();
  double i_min = -std::numeric_limits<double>::infinity();
  std::string to_string() const { return "legacy"; }
};

struct Gains {
  double p_gain_ = std::numeric_limits<double>::quiet_NaN();
  double i_gain_ = std::numeric_limits<double>::quiet_NaN();
  double d_gain_ = std::numeric_limits<double>::quiet_NaN();
  double u_max_ = std::numeric_limits<double>::infinity();
  double u_min_ = -std::numeric_limits<double>::infinity();
  AntiWindupStrategy antiwindup_strat_;
};

class PidROS {
 public:
  PidROS(rclcpp::Node::SharedPtr node, std::string prefix, std::string /*topic_prefix*/, bool /*activate_state_publisher*/)
      : node_(std::move(node)), prefix_(std::move(prefix)) {}
  bool initialize_from_ros_parameters() {
    auto get = [&](const char* k, double& dst) {
      auto v = node_->get_parameter(prefix_ + "." + k);
      if (v) dst = std::stod(*v);
    };
    get("p", g_.p_gain_);
    get("i", g_.i_gain_);
    get("d", g_.d_gain_);
    get("u_clamp_max", g_.u_max_);
    get("u_clamp_min", g_.u_min_);
    get("i_clamp_max", g_.antiwindup_strat_.i_max);
    get("i_clamp_min", g_.antiwindup_strat_.i_min);
    return std::isfinite(g_.p_gain_) && std::isfinite(g_.i_gain_) && std::isfinite(g_.d_gain_);
  }
  Gains get_gains() const { return g_; }
  double compute_command(double error, const rclcpp::Duration& period) {
    const double dt = period.seconds();
    if (!(dt > 0) || !std::isfinite(error)) return 0.0;
    // derivative of the error against the previous call's error (0 after reset), as Pid does
    const double error_dot = (error - last_error_) / dt;
    last_error_ = error;
    i_term_ = std::clamp(i_term_ + g_.i_gain_ * dt * error, g_.antiwindup_strat_.i_min, g_.antiwindup_strat_.i_max);
    const double u = g_.p_gain_ * error + i_term_ + g_.d_gain_ * error_dot;
    return std::clamp(u, g_.u_min_, g_.u_max_);
  }
  void reset() { i_term_ = 0; last_error_ = 0; }
 private:
  rclcpp::Node::SharedPtr node_;
  std::string prefix_;
  Gains g_;
  double i_term_ = 0, last_error_ = 0;
};

}  // namespace control_toolbox
