// ros_shim: hardware_interface::StateInterface / CommandInterface (name + raw double* handle)
#pragma once
#include <string>

namespace hardware_interface {

class Handle {
 public:
  Handle(std::string prefix, std::string iface, double* ptr)
      : prefix_(std::move(prefix)), iface_(std::move(iface)), ptr_(ptr) {}
  std::string get_name() const { return prefix_ + "/" + iface_; }
  const std::string& get_interface_name() const { return iface_; }
  const std::string& get_prefix_name() const { return prefix_; }
  double get_value() const { return *ptr_; }
  double* get_ptr() const { return ptr_; }
 protected:
  std::string prefix_, iface_;
  double* ptr_;
};

class StateInterface : public Handle { public: using Handle::Handle; };
class CommandInterface : public Handle {
 public:
  using Handle::Handle;
  void set_value(double v) { *ptr_ = v; }
};

}  // namespace hardware_interface
