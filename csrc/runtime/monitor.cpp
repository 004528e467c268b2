#include <kungfu/log.hpp>
#include <kungfu/monitor.hpp>

#include <cstdio>
#include <sstream>

namespace kungfu {

Monitor &Monitor::get() {
    static Monitor m;
    return m;
}

Monitor::Monitor() {
    period_ = env_duration_sec("KUNGFU_CONFIG_MONITORING_PERIOD", 1.0);
    if (period_ <= 0) period_ = 1.0;
    set_enabled(env_bool("KUNGFU_CONFIG_ENABLE_MONITORING", false));
}

Monitor::~Monitor() { stop(); }

void Monitor::set_enabled(bool on) {
    std::lock_guard<std::mutex> lk(tmu_);
    if (on == enabled_) return;
    enabled_ = on;
    if (on && !th_.joinable()) {
        stop_ = false;
        th_ = std::thread([this] {
            std::unique_lock<std::mutex> lk2(tmu_);
            while (!tcv_.wait_for(lk2, std::chrono::duration<double>(period_), [this] { return stop_; })) {
                lk2.unlock();
                tick();
                lk2.lock();
            }
        });
    }
}

void Monitor::stop() {
    {
        std::lock_guard<std::mutex> lk(tmu_);
        stop_ = true;
    }
    tcv_.notify_all();
    if (th_.joinable()) th_.join();
}

Monitor::Counter *Monitor::counter(std::map<uint64_t, std::unique_ptr<Counter>> &m, const PeerID &p) {
    std::lock_guard<std::mutex> lk(mu_);
    auto &c = m[p.hash()];
    if (!c) {
        c.reset(new Counter);
        ids_[p.hash()] = p;
    }
    return c.get();
}

void Monitor::egress(const PeerID &p, uint64_t n) {
    if (!enabled_) return;
    counter(egress_, p)->total.fetch_add(n, std::memory_order_relaxed);
}

void Monitor::ingress(const PeerID &p, uint64_t n) {
    if (!enabled_) return;
    counter(ingress_, p)->total.fetch_add(n, std::memory_order_relaxed);
}

void Monitor::tick() {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto *m : {&egress_, &ingress_})
        for (auto &kv : *m) {
            uint64_t t = kv.second->total.load();
            kv.second->rate = static_cast<double>(t - kv.second->last_total) / period_;
            kv.second->last_total = t;
        }
}

std::vector<double> Monitor::egress_rates(const PeerList &peers) {
    std::vector<double> out;
    std::lock_guard<std::mutex> lk(mu_);
    for (auto &p : peers) {
        auto it = egress_.find(p.hash());
        out.push_back(it == egress_.end() ? 0.0 : it->second->rate);
    }
    return out;
}

std::vector<double> Monitor::ingress_rates(const PeerList &peers) {
    std::vector<double> out;
    std::lock_guard<std::mutex> lk(mu_);
    for (auto &p : peers) {
        auto it = ingress_.find(p.hash());
        out.push_back(it == ingress_.end() ? 0.0 : it->second->rate);
    }
    return out;
}

uint64_t Monitor::egress_total(const PeerID &p) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = egress_.find(p.hash());
    return it == egress_.end() ? 0 : it->second->total.load();
}

uint64_t Monitor::ingress_total(const PeerID &p) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = ingress_.find(p.hash());
    return it == ingress_.end() ? 0 : it->second->total.load();
}

std::string Monitor::metrics_text() {
    std::ostringstream os;
    std::lock_guard<std::mutex> lk(mu_);
    auto emit = [&](const char *what, std::map<uint64_t, std::unique_ptr<Counter>> &m) {
        for (auto &kv : m)
            os << what << "_total_bytes{peer=\"" << ids_[kv.first].str() << "\"} " << kv.second->total.load()
               << "\n";
        for (auto &kv : m)
            os << what << "_rate_bytes_per_sec{peer=\"" << ids_[kv.first].str() << "\"} " << kv.second->rate
               << "\n";
    };
    emit("egress", egress_);
    emit("ingress", ingress_);
    return os.str();
}

}  // namespace kungfu
