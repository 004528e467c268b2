// Leveled logger, stall detector and scoped trace for the host runtime.
//
// Parity: srcs/go/log/logger.go:14-150 (levels from KUNGFU_CONFIG_LOG_LEVEL,
// prefixes [D]/[I]/[W]/[E]/[F]); srcs/go/utils/stalldetector.go:9-46 (prints
// "<name> stalled for <t>" every 3 s); srcs/cpp/include/kungfu/utils/trace.hpp
// (TRACE_SCOPE; here it is always compiled and enabled by KUNGFU_CONFIG_ENABLE_TRACE,
// printing per-scope count/total/mean at exit).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>

namespace kungfu {

enum class LogLevel : int { DEBUG = 0, INFO = 1, WARN = 2, ERROR = 3 };

LogLevel log_level();
void set_log_level(LogLevel l);
void logf(LogLevel l, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
[[noreturn]] void fatalf(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

#define KF_DEBUG(...) ::kungfu::logf(::kungfu::LogLevel::DEBUG, __VA_ARGS__)
#define KF_INFO(...) ::kungfu::logf(::kungfu::LogLevel::INFO, __VA_ARGS__)
#define KF_WARN(...) ::kungfu::logf(::kungfu::LogLevel::WARN, __VA_ARGS__)
#define KF_ERROR(...) ::kungfu::logf(::kungfu::LogLevel::ERROR, __VA_ARGS__)

// Environment helpers shared by the runtime.
std::string env_str(const char *key, const std::string &def = "");
bool env_bool(const char *key, bool def = false);
double env_duration_sec(const char *key, double def);  // "5m", "1s", "200ms", "3"

bool stall_detection_enabled();

// Prints "<name> stalled for <t>s" every `period` until destroyed.
class StallDetector {
  public:
    explicit StallDetector(std::string name, double period_sec = 3.0);
    ~StallDetector();

  private:
    std::string name_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool done_ = false;
    std::thread th_;
};

// Host-op watchdog (parity: the reference's stall detector around every collective,
// srcs/go/libkungfu-comm/main.go:163-179, turned into a failure detector).  Every
// collective of the host runtime holds an OpWatch for its duration; one process-wide
// thread checks them and, when an op has run longer than KUNGFU_OP_TIMEOUT_S (a
// duration: "90", "2m"; unset or 0 = disabled), prints the op name and this peer's
// label and terminates the process with exit status 3 (a hung peer would otherwise
// block the whole job until an outer timeout, leaving nothing to diagnose).
class OpWatch {
  public:
    explicit OpWatch(const std::string &name);
    ~OpWatch();
    OpWatch(const OpWatch &) = delete;
    OpWatch &operator=(const OpWatch &) = delete;

  private:
    uint64_t id_ = 0;
};
void op_watchdog_set_label(const std::string &label);
double op_watchdog_timeout();  // seconds, 0 = disabled
void op_watchdog_set_timeout(double seconds);

// Scoped timer aggregated per name; report printed at process exit when
// KUNGFU_CONFIG_ENABLE_TRACE is set.
class TraceScope {
  public:
    explicit TraceScope(const char *name);
    ~TraceScope();

  private:
    const char *name_;
    std::chrono::steady_clock::time_point t0_;
};

bool trace_enabled();  // KUNGFU_CONFIG_ENABLE_TRACE
std::string trace_report();
// roctx range push/pop (no-ops unless tracing is enabled and libroctx64 is loadable)
void trace_push(const char *name);
void trace_pop();
void trace_record(const std::string &name, double seconds);

#define KF_TRACE_CAT2(a, b) a##b
#define KF_TRACE_CAT(a, b) KF_TRACE_CAT2(a, b)
// Compile-time switch (./configure --disable-trace => -DKUNGFU_DISABLE_TRACE): scopes
// compile to nothing, like the reference's stdtracer-less build (utils/trace.hpp:1-16).
// Otherwise they are runtime-gated by KUNGFU_CONFIG_ENABLE_TRACE.
#ifdef KUNGFU_DISABLE_TRACE
#define KF_TRACE_SCOPE(name) ((void)0)
#else
#define KF_TRACE_SCOPE(name) ::kungfu::TraceScope KF_TRACE_CAT(_kf_trace_, __LINE__)(name)
#endif

}  // namespace kungfu
