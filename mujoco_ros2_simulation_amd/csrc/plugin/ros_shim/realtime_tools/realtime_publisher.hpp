// ros_shim: realtime_tools::RealtimePublisher (try_publish forwards to the wrapped publisher)
#pragma once
#include <memory>
#include "rclcpp/rclcpp.hpp"
namespace realtime_tools {
template <class MsgT>
class RealtimePublisher {
 public:
  using SharedPtr = std::shared_ptr<RealtimePublisher<MsgT>>;
  explicit RealtimePublisher(typename rclcpp::Publisher<MsgT>::SharedPtr pub) : pub_(std::move(pub)) {}
  bool try_publish(const MsgT& msg) { pub_->publish(msg); return true; }
 private:
  typename rclcpp::Publisher<MsgT>::SharedPtr pub_;
};
}  // namespace realtime_tools
