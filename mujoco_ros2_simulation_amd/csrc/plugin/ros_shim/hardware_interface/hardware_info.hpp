// ros_shim: hardware_interface::HardwareInfo / ComponentInfo / InterfaceInfo (jazzy field names)
#pragma once
#include <string>
#include <unordered_map>
#include <vector>

namespace hardware_interface {

struct InterfaceInfo {
  std::string name;
  std::string min, max;
  std::string initial_value;
  std::string data_type = "double";
  int size = 0;
  std::unordered_map<std::string, std::string> parameters;
};

struct ComponentInfo {
  std::string name;
  std::string type;
  std::vector<InterfaceInfo> command_interfaces;
  std::vector<InterfaceInfo> state_interfaces;
  std::unordered_map<std::string, std::string> parameters;
};

struct HardwareInfo {
  std::string name;
  std::string type;
  std::string hardware_plugin_name;
  std::unordered_map<std::string, std::string> hardware_parameters;
  std::vector<ComponentInfo> joints;
  std::vector<ComponentInfo> sensors;
  std::vector<ComponentInfo> gpios;
};

struct HardwareComponentInterfaceParams {
  HardwareInfo hardware_info;
};

}  // namespace hardware_interface
