// ros_shim: minimal rclcpp surface (Time, Duration, Logger + RCLCPP_* macros, Node with parameters
// and recording publishers, Rate).  See ../README.md.
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace rclcpp {

class Duration {
 public:
  Duration(int32_t sec = 0, uint32_t nsec = 0) : ns_(int64_t(sec) * 1000000000LL + nsec) {}
  static Duration from_seconds(double s) { Duration d; d.ns_ = int64_t(s * 1e9); return d; }
  double seconds() const { return ns_ * 1e-9; }
  int64_t nanoseconds() const { return ns_; }
 private:
  int64_t ns_ = 0;
};

class Time {
 public:
  Time(int32_t sec = 0, uint32_t nsec = 0, int clock_type = 0) : ns_(int64_t(sec) * 1000000000LL + nsec) { (void)clock_type; }
  double seconds() const { return ns_ * 1e-9; }
  int64_t nanoseconds() const { return ns_; }
 private:
  int64_t ns_;
};

class Logger {
 public:
  explicit Logger(std::string name = "") : name_(std::move(name)) {}
  const std::string& name() const { return name_; }
 private:
  std::string name_;
};
inline Logger get_logger(const std::string& name) { return Logger(name); }

inline bool& verbose_logging() { static bool v = false; return v; }

namespace detail {
inline void log(const char* level, const Logger& l, const std::string& msg) {
  if (verbose_logging() || level[0] == 'E' || level[0] == 'F')
    std::fprintf(stderr, "[%s] [%s]: %s\n", level, l.name().c_str(), msg.c_str());
}
template <class... A>
std::string fmt(const char* f, A... a) {
  char buf[2048];
  std::snprintf(buf, sizeof buf, f, a...);
  return buf;
}
inline std::string fmt(const char* f) { return f; }
}  // namespace detail

struct QoS {
  explicit QoS(size_t depth = 1) : depth(depth) {}
  size_t depth;
};

template <class MsgT>
class Publisher {
 public:
  using SharedPtr = std::shared_ptr<Publisher<MsgT>>;
  explicit Publisher(std::string topic) : topic_(std::move(topic)) {}
  void publish(const MsgT& msg) {
    std::lock_guard<std::mutex> lk(mu_);
    last_ = msg;
    ++count_;
  }
  const std::string& get_topic_name() const { return topic_; }
  // shim-only introspection for tests
  std::optional<MsgT> last() const { std::lock_guard<std::mutex> lk(mu_); return last_; }
  size_t count() const { std::lock_guard<std::mutex> lk(mu_); return count_; }
 private:
  std::string topic_;
  mutable std::mutex mu_;
  std::optional<MsgT> last_;
  size_t count_ = 0;
};

class Node {
 public:
  using SharedPtr = std::shared_ptr<Node>;
  explicit Node(std::string name, std::map<std::string, std::string> params = {})
      : name_(std::move(name)), params_(std::move(params)) {}
  template <class MsgT>
  typename Publisher<MsgT>::SharedPtr create_publisher(const std::string& topic, size_t /*qos*/) {
    auto p = std::make_shared<Publisher<MsgT>>(topic);
    std::lock_guard<std::mutex> lk(mu_);
    publishers_[topic] = p;
    return p;
  }
  template <class MsgT>
  typename Publisher<MsgT>::SharedPtr find_publisher(const std::string& topic) const {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = publishers_.find(topic);
    return it == publishers_.end() ? nullptr : std::static_pointer_cast<Publisher<MsgT>>(it->second);
  }
  Logger get_logger() const { return Logger(name_); }
  // simulated ROS time (use_sim_time=true): driven by the plugin's /clock
  Time now() const { std::lock_guard<std::mutex> lk(mu_); return now_; }
  void set_now(const Time& t) { std::lock_guard<std::mutex> lk(mu_); now_ = t; }
  std::optional<std::string> get_parameter(const std::string& key) const {
    auto it = params_.find(key);
    if (it == params_.end()) return std::nullopt;
    return it->second;
  }
  const std::string& get_name() const { return name_; }
 private:
  std::string name_;
  std::map<std::string, std::string> params_;
  mutable std::mutex mu_;
  std::map<std::string, std::shared_ptr<void>> publishers_;
  Time now_;
};

inline bool ok() { return true; }

class Rate {
 public:
  explicit Rate(double hz) : period_(std::chrono::duration<double>(1.0 / hz)), next_(std::chrono::steady_clock::now()) {}
  void sleep() {
    next_ += std::chrono::duration_cast<std::chrono::steady_clock::duration>(period_);
    std::this_thread::sleep_until(next_);
  }
 private:
  std::chrono::duration<double> period_;
  std::chrono::steady_clock::time_point next_;
};

}  // namespace rclcpp

#define RCLCPP_INFO(logger, ...) ::rclcpp::detail::log("INFO", logger, ::rclcpp::detail::fmt(__VA_ARGS__))
#define RCLCPP_WARN(logger, ...) ::rclcpp::detail::log("WARN", logger, ::rclcpp::detail::fmt(__VA_ARGS__))
#define RCLCPP_ERROR(logger, ...) ::rclcpp::detail::log("ERROR", logger, ::rclcpp::detail::fmt(__VA_ARGS__))
#define RCLCPP_FATAL(logger, ...) ::rclcpp::detail::log("FATAL", logger, ::rclcpp::detail::fmt(__VA_ARGS__))
#define RCLCPP_DEBUG(logger, ...) do { (void)(logger); } while (0)
#define RCLCPP_INFO_STREAM(logger, x) do { std::ostringstream os_; os_ << x; ::rclcpp::detail::log("INFO", logger, os_.str()); } while (0)
#define RCLCPP_WARN_STREAM(logger, x) do { std::ostringstream os_; os_ << x; ::rclcpp::detail::log("WARN", logger, os_.str()); } while (0)
#define RCLCPP_ERROR_STREAM(logger, x) do { std::ostringstream os_; os_ << x; ::rclcpp::detail::log("ERROR", logger, os_.str()); } while (0)
#define RCLCPP_DEBUG_STREAM(logger, x) do { (void)(logger); } while (0)
