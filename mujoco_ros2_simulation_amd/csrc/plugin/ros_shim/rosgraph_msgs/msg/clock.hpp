// ros_shim: rosgraph_msgs/msg/Clock
#pragma once
#include "rclcpp/rclcpp.hpp"
namespace rosgraph_msgs { namespace msg { struct Clock { rclcpp::Time clock; }; } }
