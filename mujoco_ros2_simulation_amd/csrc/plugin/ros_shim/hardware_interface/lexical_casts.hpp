// ros_shim: hardware_interface::parse_bool
#pragma once
#include <algorithm>
#include <cctype>
#include <string>
namespace hardware_interface {
inline bool parse_bool(const std::string& s) {
  std::string t = s;
  std::transform(t.begin(), t.end(), t.begin(), [](unsigned char c) { return std::tolower(c); });
  return t == "true";
}
}  // namespace hardware_interface
