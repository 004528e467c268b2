// kungfu-run main() and the standalone config-server main().
// Parity: srcs/go/cmd/kungfu-run/app/kungfu-run.go:18-112,
//         srcs/go/cmd/kungfu-config-server/kungfu-config-server.go:19-72.
#include "launcher.hpp"

#include <kungfu/log.hpp>

#include <cstdio>
#include <fstream>
#include <sstream>
#include <thread>

namespace kungfu {
namespace launcher {

int kungfu_run_main(int argc, char **argv) {
    Flags f;
    auto err = f.parse(argc, argv);
    if (!err.empty()) {
        std::fprintf(stderr, "%s\n%s", err.c_str(), err == Flags::usage() ? "" : Flags::usage().c_str());
        return err == Flags::usage() ? 0 : 2;
    }
    if (f.quiet) set_log_level(LogLevel::WARN);
    if (f.delay > 0) {
        KF_WARN("delay start for %.1fs", f.delay);
        std::this_thread::sleep_for(std::chrono::duration<double>(f.delay));
    }
    std::unique_ptr<ConfigServer> builtin;
    if (f.builtin_config_port > 0) {
        builtin.reset(new ConfigServer(static_cast<uint16_t>(f.builtin_config_port), "/config"));
        builtin->start();
        KF_INFO("running builtin config server listening :%d/config", f.builtin_config_port);
    }
    if (!f.logfile.empty()) {
        std::string lf = f.logdir.empty() ? f.logfile : f.logdir + "/" + f.logfile;
        if (!std::freopen(lf.c_str(), "w", stderr)) KF_WARN("cannot open logfile %s", lf.c_str());
    }
    uint32_t self_ip;
    try {
        self_ip = infer_self_ipv4(f.self, f.nic, f.hosts);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    PeerID self{self_ip, static_cast<uint16_t>(f.port)};
    PeerList runners = f.hosts.gen_runner_list(static_cast<uint16_t>(f.port));
    if (!runners.contains(self)) {
        std::fprintf(stderr, "%s not in %s\n", self.str().c_str(), runners.str().c_str());
        return 1;
    }
    PeerList peers;
    try {
        peers = f.hosts.gen_peer_list(f.np, f.port_range);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "failed to create peers: %s\n", e.what());
        return 1;
    }
    Job j;
    j.start_time = f.job_start_time;
    j.strategy = f.strategy;
    j.parent = self;
    j.hosts = f.hosts;
    j.port_range = f.port_range;
    j.prog = f.prog;
    j.args = f.args;
    j.logdir = f.logdir;
    j.allow_xgmi = f.allow_xgmi;
    std::atomic<bool> cancel{false};
    trap_signals(&cancel);
    std::atomic<bool> timed_out{false}, finished{false};
    std::thread timer;
    if (f.timeout > 0) {
        timer = std::thread([&] {
            auto t0 = std::chrono::steady_clock::now();
            while (!finished.load()) {
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > f.timeout) {
                    KF_ERROR("timeout after %.1fs, killing workers", f.timeout);
                    timed_out.store(true);
                    cancel.store(true);
                    return;
                }
                std::this_thread::sleep_for(std::chrono::milliseconds(50));
            }
        });
    }
    Cluster init{runners, peers};
    int rc;
    auto t0 = std::chrono::steady_clock::now();
    if (f.watch) {
        j.config_server = f.config_server;
        Stage st{f.init_version, init};
        rc = watch_run(self, runners, f.init_version < 0 ? nullptr : &st, j, f.keep, f.debug_port, &cancel);
    } else {
        rc = simple_run(self_ip, init, j, f.verbose, &cancel);
    }
    finished.store(true);
    if (timer.joinable()) timer.join();
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    KF_DEBUG("%s finished, took %.3fs", f.prog.c_str(), dt);
    if (builtin) builtin->stop();
    if (timed_out.load()) return 124;
    return rc;
}

int config_server_main(int argc, char **argv) {
    int port = 9100;
    std::string init_file;
    double ttl = 0;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : ""; };
        if (a == "-port" || a == "--port") port = std::stoi(next());
        else if (a == "-init" || a == "--init") init_file = next();
        else if (a == "-ttl" || a == "--ttl") ttl = std::stod(next());
        else {
            std::fprintf(stderr, "usage: kungfu-config-server [-port 9100] [-init cluster.json] [-ttl seconds]\n");
            return 2;
        }
    }
    ConfigServer s(static_cast<uint16_t>(port), "/config");
    if (!init_file.empty()) {
        std::ifstream in(init_file);
        std::stringstream ss;
        ss << in.rdbuf();
        s.set_cluster(Cluster::from_json(json::parse(ss.str())));
    }
    s.start();
    KF_INFO("config server listening on :%d/config", port);
    std::atomic<bool> cancel{false};
    trap_signals(&cancel);
    auto t0 = std::chrono::steady_clock::now();
    while (!s.stopped() && !cancel.load()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
        if (ttl > 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > ttl) break;
    }
    s.stop();
    return 0;
}

}  // namespace launcher
}  // namespace kungfu
