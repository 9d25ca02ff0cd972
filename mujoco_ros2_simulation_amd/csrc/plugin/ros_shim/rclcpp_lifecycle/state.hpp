// ros_shim: rclcpp_lifecycle::State (see ../README.md)
#pragma once
namespace rclcpp_lifecycle { class State { public: State() = default; }; }
