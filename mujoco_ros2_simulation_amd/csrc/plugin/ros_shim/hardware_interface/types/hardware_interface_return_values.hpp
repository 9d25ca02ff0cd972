// ros_shim (see ../../README.md)
#pragma once
namespace hardware_interface {
enum class return_type { OK = 0, ERROR = 1 };
enum class CallbackReturn { SUCCESS = 0, FAILURE = 1, ERROR = 2 };
}  // namespace hardware_interface
