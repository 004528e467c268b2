#include <kungfu/log.hpp>

#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <sstream>

namespace kungfu {

namespace {

LogLevel parse_level(const std::string &s) {
    if (s == "DEBUG" || s == "debug") return LogLevel::DEBUG;
    if (s == "WARN" || s == "warn") return LogLevel::WARN;
    if (s == "ERROR" || s == "error") return LogLevel::ERROR;
    return LogLevel::INFO;
}

std::atomic<int> &level_ref() {
    static std::atomic<int> lvl{static_cast<int>(parse_level(env_str("KUNGFU_CONFIG_LOG_LEVEL", "INFO")))};
    return lvl;
}

const char *prefix(LogLevel l) {
    switch (l) {
    case LogLevel::DEBUG: return "[D]";
    case LogLevel::INFO: return "[I]";
    case LogLevel::WARN: return "[W]";
    case LogLevel::ERROR: return "[E]";
    }
    return "[?]";
}

struct TraceStat {
    uint64_t count = 0;
    double total = 0;
};

// Intentionally leaked: the at-exit reporter below runs during static destruction,
// after function-local statics constructed later than it would already be gone.
std::mutex &trace_mu() {
    static std::mutex *m = new std::mutex;
    return *m;
}

std::map<std::string, TraceStat> &trace_stats() {
    static auto *s = new std::map<std::string, TraceStat>;
    return *s;
}

struct TraceReporter {
    ~TraceReporter() {
        if (trace_enabled()) {
            auto r = trace_report();
            if (!r.empty()) std::fprintf(stderr, "%s", r.c_str());
        }
    }
} g_trace_reporter;

}  // namespace

std::string env_str(const char *key, const std::string &def) {
    const char *v = std::getenv(key);
    return v ? std::string(v) : def;
}

bool env_bool(const char *key, bool def) {
    const char *v = std::getenv(key);
    if (!v) return def;
    std::string s(v);
    return s == "1" || s == "true" || s == "TRUE" || s == "True" || s == "yes" || s == "on";
}

double env_duration_sec(const char *key, double def) {
    const char *v = std::getenv(key);
    if (!v || !*v) return def;
    std::string s(v);
    try {
        size_t pos = 0;
        double x = std::stod(s, &pos);
        std::string unit = s.substr(pos);
        if (unit.empty() || unit == "s") return x;
        if (unit == "ms") return x / 1000.0;
        if (unit == "us") return x / 1e6;
        if (unit == "m") return x * 60.0;
        if (unit == "h") return x * 3600.0;
    } catch (...) {
    }
    return def;
}

LogLevel log_level() { return static_cast<LogLevel>(level_ref().load()); }
void set_log_level(LogLevel l) { level_ref().store(static_cast<int>(l)); }

void logf(LogLevel l, const char *fmt, ...) {
    if (static_cast<int>(l) < level_ref().load()) return;
    char buf[4096];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    std::fprintf(stderr, "%s %s\n", prefix(l), buf);
}

void fatalf(const char *fmt, ...) {
    char buf[4096];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    std::fprintf(stderr, "[F] %s\n", buf);
    std::fflush(stderr);
    std::abort();
}

bool stall_detection_enabled() {
    static bool on = env_bool("KUNGFU_CONFIG_ENABLE_STALL_DETECTION", false);
    return on;
}

StallDetector::StallDetector(std::string name, double period_sec) : name_(std::move(name)) {
    if (!stall_detection_enabled()) return;
    th_ = std::thread([this, period_sec] {
        auto t0 = std::chrono::steady_clock::now();
        std::unique_lock<std::mutex> lk(mu_);
        while (!cv_.wait_for(lk, std::chrono::duration<double>(period_sec), [this] { return done_; })) {
            double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            std::fprintf(stderr, "[W] %s stalled for %.1fs\n", name_.c_str(), dt);
        }
    });
}

StallDetector::~StallDetector() {
    if (!th_.joinable()) return;
    {
        std::lock_guard<std::mutex> lk(mu_);
        done_ = true;
    }
    cv_.notify_all();
    th_.join();
}

namespace {
class OpWatchdog {
  public:
    static OpWatchdog &get() {
        static OpWatchdog *w = new OpWatchdog();  // never destroyed (used until _exit)
        return *w;
    }
    uint64_t begin(const std::string &name) {
        if (timeout_.load() <= 0) return 0;
        std::lock_guard<std::mutex> lk(mu_);
        const uint64_t id = ++next_;
        ops_.emplace(id, Op{name, std::chrono::steady_clock::now()});
        if (!started_) {
            started_ = true;
            std::thread([this] { loop(); }).detach();
        }
        return id;
    }
    void end(uint64_t id) {
        if (!id) return;
        std::lock_guard<std::mutex> lk(mu_);
        ops_.erase(id);
    }
    void set_label(const std::string &l) {
        std::lock_guard<std::mutex> lk(mu_);
        label_ = l;
    }
    double timeout() const { return timeout_.load(); }
    void set_timeout(double t) { timeout_.store(t); }

  private:
    struct Op {
        std::string name;
        std::chrono::steady_clock::time_point t0;
    };
    OpWatchdog() : timeout_(env_duration_sec("KUNGFU_OP_TIMEOUT_S", 0)) {}
    void loop() {
        for (;;) {
            const double t = timeout_.load();
            std::this_thread::sleep_for(std::chrono::duration<double>(t > 0 ? std::min(0.25, std::max(0.01, t / 20)) : 0.25));
            if (t <= 0) continue;
            std::lock_guard<std::mutex> lk(mu_);
            const auto now = std::chrono::steady_clock::now();
            for (const auto &kv : ops_) {
                const double age = std::chrono::duration<double>(now - kv.second.t0).count();
                if (age <= t) continue;
                std::fprintf(stderr,
                             "[F] kungfu op watchdog (%s): host op '%s' has not completed after %.1f s "
                             "(KUNGFU_OP_TIMEOUT_S=%g); %zu op(s) in flight; exiting with status 3\n",
                             label_.empty() ? "?" : label_.c_str(), kv.second.name.c_str(), age, t, ops_.size());
                std::fflush(stderr);
                std::fflush(stdout);
                ::_exit(3);
            }
        }
    }
    std::mutex mu_;
    std::map<uint64_t, Op> ops_;
    uint64_t next_ = 0;
    bool started_ = false;
    std::string label_;
    std::atomic<double> timeout_;
};
}  // namespace

OpWatch::OpWatch(const std::string &name) : id_(OpWatchdog::get().begin(name)) {}
OpWatch::~OpWatch() { OpWatchdog::get().end(id_); }
void op_watchdog_set_label(const std::string &label) { OpWatchdog::get().set_label(label); }
double op_watchdog_timeout() { return OpWatchdog::get().timeout(); }
void op_watchdog_set_timeout(double seconds) { OpWatchdog::get().set_timeout(seconds); }

bool trace_enabled() {
    static bool on = env_bool("KUNGFU_CONFIG_ENABLE_TRACE", false);
    return on;
}

namespace {
// roctx ranges (rocprofv3 --marker-trace shows them next to the kernels) loaded at run
// time, so the runtime has no link dependency on the ROCm profiler libraries.
struct Roctx {
    int (*push)(const char *) = nullptr;
    int (*pop)() = nullptr;
    Roctx() {
        if (!trace_enabled()) return;
        for (const char *lib : {"libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"}) {
            void *h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
            if (!h) continue;
            push = reinterpret_cast<int (*)(const char *)>(dlsym(h, "roctxRangePushA"));
            pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
            if (push && pop) return;
            push = nullptr;
            pop = nullptr;
        }
    }
};
Roctx &roctx() {
    static Roctx r;
    return r;
}
}  // namespace

void trace_push(const char *name) {
    if (trace_enabled() && roctx().push) roctx().push(name);
}

void trace_pop() {
    if (trace_enabled() && roctx().pop) roctx().pop();
}

void trace_record(const std::string &name, double seconds) {
    std::lock_guard<std::mutex> lk(trace_mu());
    auto &s = trace_stats()[name];
    s.count++;
    s.total += seconds;
}

TraceScope::TraceScope(const char *name) : name_(name) {
    if (trace_enabled()) {
        t0_ = std::chrono::steady_clock::now();
        trace_push(name);
    }
}

TraceScope::~TraceScope() {
    if (!trace_enabled()) return;
    trace_pop();
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0_).count();
    std::lock_guard<std::mutex> lk(trace_mu());
    auto &s = trace_stats()[name_];
    s.count++;
    s.total += dt;
}

std::string trace_report() {
    std::lock_guard<std::mutex> lk(trace_mu());
    std::ostringstream os;
    for (auto &kv : trace_stats()) {
        char buf[512];
        std::snprintf(buf, sizeof(buf), "[trace] %-40s count=%llu total=%.6fs mean=%.3fms\n", kv.first.c_str(),
                      static_cast<unsigned long long>(kv.second.count), kv.second.total,
                      kv.second.count ? 1e3 * kv.second.total / kv.second.count : 0.0);
        os << buf;
    }
    return os.str();
}

}  // namespace kungfu
