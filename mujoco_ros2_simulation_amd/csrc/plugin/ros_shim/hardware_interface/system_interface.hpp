// ros_shim: hardware_interface::SystemInterface base class (lifecycle + hardware info holder)
#pragma once
#include <string>
#include <vector>

#include "hardware_interface/handle.hpp"
#include "hardware_interface/hardware_info.hpp"
#include "hardware_interface/types/hardware_interface_return_values.hpp"
#include "rclcpp/rclcpp.hpp"
#include "rclcpp_lifecycle/state.hpp"

namespace hardware_interface {

class SystemInterface {
 public:
  virtual ~SystemInterface() = default;
  virtual CallbackReturn on_init(const HardwareComponentInterfaceParams& params) {
    info_ = params.hardware_info;
    return CallbackReturn::SUCCESS;
  }
  virtual std::vector<StateInterface> export_state_interfaces() = 0;
  virtual std::vector<CommandInterface> export_command_interfaces() = 0;
  virtual CallbackReturn on_activate(const rclcpp_lifecycle::State&) { return CallbackReturn::SUCCESS; }
  virtual CallbackReturn on_deactivate(const rclcpp_lifecycle::State&) { return CallbackReturn::SUCCESS; }
  virtual return_type perform_command_mode_switch(const std::vector<std::string>&, const std::vector<std::string>&) {
    return return_type::OK;
  }
  virtual return_type read(const rclcpp::Time& time, const rclcpp::Duration& period) = 0;
  virtual return_type write(const rclcpp::Time& time, const rclcpp::Duration& period) = 0;
  const HardwareInfo& get_hardware_info() const { return info_; }
 protected:
  HardwareInfo info_;
};

}  // namespace hardware_interface
