// Network monitor: per-peer egress/ingress byte counters and rates, exposed as
// Prometheus-style text (served over HTTP by the peer when monitoring is on).
//
// Parity: srcs/go/monitor/monitor.go:13-107, monitor/counters.go:13-164
// (egress_total_bytes{peer=".."}, egress_rate_bytes_per_sec{...}; rate window
// KUNGFU_CONFIG_MONITORING_PERIOD, default 1 s; enabled by
// KUNGFU_CONFIG_ENABLE_MONITORING).  Unlike the reference, ingress is recorded
// by the transport's reader.
#pragma once

#include <kungfu/plan.hpp>

#include <atomic>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace kungfu {

class Monitor {
  public:
    static Monitor &get();

    bool enabled() const { return enabled_; }
    void egress(const PeerID &p, uint64_t n);
    void ingress(const PeerID &p, uint64_t n);
    // Rates (bytes/s) over the last completed window, ordered like `peers`.
    std::vector<double> egress_rates(const PeerList &peers);
    std::vector<double> ingress_rates(const PeerList &peers);
    uint64_t egress_total(const PeerID &p);
    uint64_t ingress_total(const PeerID &p);
    std::string metrics_text();
    void set_enabled(bool on);
    void stop();
    ~Monitor();

  private:
    Monitor();
    struct Counter {
        std::atomic<uint64_t> total{0};
        uint64_t last_total = 0;
        double rate = 0;
    };
    Counter *counter(std::map<uint64_t, std::unique_ptr<Counter>> &m, const PeerID &p);
    void tick();

    bool enabled_ = false;
    double period_ = 1.0;
    std::mutex mu_;
    std::map<uint64_t, std::unique_ptr<Counter>> egress_, ingress_;
    std::map<uint64_t, PeerID> ids_;
    std::mutex tmu_;
    std::condition_variable tcv_;
    bool stop_ = false;
    std::thread th_;
};

}  // namespace kungfu
