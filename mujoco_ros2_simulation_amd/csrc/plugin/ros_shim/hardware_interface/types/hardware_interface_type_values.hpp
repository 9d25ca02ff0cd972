// ros_shim: interface name constants (hardware_interface/types/hardware_interface_type_values.hpp)
#pragma once
namespace hardware_interface {
constexpr char HW_IF_POSITION[] = "position";
constexpr char HW_IF_VELOCITY[] = "velocity";
constexpr char HW_IF_ACCELERATION[] = "acceleration";
constexpr char HW_IF_EFFORT[] = "effort";
constexpr char HW_IF_TORQUE[] = "torque";
constexpr char HW_IF_FORCE[] = "force";
}  // namespace hardware_interface
