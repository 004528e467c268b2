// kungfu-run flag parsing and self-IP inference.  See launcher.hpp for parity.
#include "launcher.hpp"

#include <kungfu/log.hpp>

#include <arpa/inet.h>
#include <ifaddrs.h>
#include <netdb.h>
#include <netinet/in.h>

#include <cstdlib>
#include <ctime>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <thread>

namespace kungfu {
namespace launcher {

namespace {

double parse_duration(const std::string &s) {
    size_t pos = 0;
    double x = std::stod(s, &pos);
    std::string unit = s.substr(pos);
    if (unit.empty() || unit == "s") return x;
    if (unit == "ms") return x / 1000.0;
    if (unit == "m") return x * 60.0;
    if (unit == "h") return x * 3600.0;
    // Go-style composite like "1m30s"
    double total = 0;
    std::string cur;
    for (size_t i = 0; i < s.size(); ++i) {
        char c = s[i];
        if ((c >= '0' && c <= '9') || c == '.') {
            cur.push_back(c);
            continue;
        }
        std::string u(1, c);
        if (c == 'm' && i + 1 < s.size() && s[i + 1] == 's') {
            u = "ms";
            ++i;
        }
        double v = std::stod(cur);
        cur.clear();
        if (u == "h") total += v * 3600;
        else if (u == "m") total += v * 60;
        else if (u == "s") total += v;
        else if (u == "ms") total += v / 1000;
        else throw std::invalid_argument("bad duration " + s);
    }
    return total;
}

bool parse_bool(const std::string &v) { return v == "1" || v == "true" || v == "True" || v == "t" || v == "T"; }

}  // namespace

std::string Flags::usage() {
    return "usage: kungfu-run [flags] <prog> [args...]\n"
           "  -np N                  number of peers (1)\n"
           "  -H ip:slots[:pub],...  host list (127.0.0.1:<ncpu>)\n"
           "  -hostfile PATH         OpenMPI-style hostfile (overrides -H)\n"
           "  -u USER                ssh user (remote launch)\n"
           "  -port-range A-B        worker ports (10000-11000)\n"
           "  -self IPv4             this host's internal IPv4\n"
           "  -nic NAME              infer self IPv4 from this interface\n"
           "  -platform NAME         peer discovery from a platform's env (modelarts); or KUNGFU_PLATFORM\n"
           "  -timeout DUR           kill the job after DUR (e.g. 30s, 5m)\n"
           "  -v[=bool]              stream worker output (true)\n"
           "  -q                     quiet launcher logs\n"
           "  -allow-xgmi[=bool]     keep all GPUs visible to every worker (default; alias -allow-nvlink)\n"
           "  -isolate-gpus          one visible GPU per worker (HIP_VISIBLE_DEVICES=<slot>)\n"
           "  -strategy NAME         STAR|MULTI_STAR|RING|CLIQUE|TREE|BINARY_TREE|BINARY_TREE_STAR|"
           "MULTI_BINARY_TREE_STAR|AUTO\n"
           "  -port N                runner port (38080)\n"
           "  -debug-port N          runner HTTP debug server port\n"
           "  -w                     watch mode (elastic)\n"
           "  -k                     keep runner alive after workers finish (watch mode)\n"
           "  -init-version N        initial cluster version (-1: wait for a stage)\n"
           "  -config-server URL     config server URL\n"
           "  -builtin-config-port N run a config server in the launcher\n"
           "  -t0 UNIX               job start timestamp\n"
           "  -logfile PATH, -logdir DIR\n"
           "  -delay DUR             delay start (testing)\n";
}

std::string Flags::parse(int argc, char **argv) {
    job_start_time = static_cast<long>(std::time(nullptr));
    host_list_str = "127.0.0.1:" + std::to_string(std::max(1u, std::thread::hardware_concurrency()));
    int i = 1;
    auto need = [&](const std::string &name) -> std::string {
        if (i + 1 >= argc) throw std::invalid_argument("flag needs an argument: -" + name);
        return argv[++i];
    };
    try {
        for (; i < argc; ++i) {
            std::string a = argv[i];
            if (a == "--") {
                ++i;
                break;
            }
            if (a.size() < 2 || a[0] != '-') break;
            std::string name = a.substr(a[1] == '-' ? 2 : 1), val;
            bool has_val = false;
            auto eq = name.find('=');
            if (eq != std::string::npos) {
                val = name.substr(eq + 1);
                name = name.substr(0, eq);
                has_val = true;
            }
            auto get = [&]() { return has_val ? val : need(name); };
            auto getb = [&]() { return has_val ? parse_bool(val) : true; };
            if (name == "np") np = std::stoi(get());
            else if (name == "H") host_list_str = get();
            else if (name == "hostfile") hostfile = get();
            else if (name == "P") throw std::invalid_argument("-P is not supported (use -H)");
            else if (name == "u") user = get();
            else if (name == "port-range") port_range = PortRange::parse(get());
            else if (name == "self") self = get();
            else if (name == "timeout") timeout = parse_duration(get());
            else if (name == "v") verbose = getb();
            else if (name == "nic") nic = get();
            else if (name == "allow-xgmi" || name == "allow-nvlink") allow_xgmi = getb();
            else if (name == "isolate-gpus") allow_xgmi = !getb();
            else if (name == "strategy") {
                auto s = get();
                if (!parse_strategy(s, &strategy)) throw std::invalid_argument("invalid strategy " + s);
            } else if (name == "port") port = std::stoi(get());
            else if (name == "debug-port") debug_port = std::stoi(get());
            else if (name == "w") watch = getb();
            else if (name == "k") keep = getb();
            else if (name == "init-version") init_version = std::stoi(get());
            else if (name == "config-server") config_server = get();
            else if (name == "t0") job_start_time = std::stol(get());
            else if (name == "logfile") logfile = get();
            else if (name == "logdir") logdir = get();
            else if (name == "q") quiet = getb();
            else if (name == "delay") delay = parse_duration(get());
            else if (name == "builtin-config-port") builtin_config_port = std::stoi(get());
            else if (name == "platform") platform = get();
            else if (name == "h" || name == "help") return usage();
            else throw std::invalid_argument("unknown flag -" + name);
        }
        if (platform.empty()) {
            const char *e = std::getenv("KUNGFU_PLATFORM");
            if (e) platform = e;
        }
        if (platform == "modelarts") {
            // runner list, self and ports come from the platform's env (one runner per container)
            auto info = parse_modelarts_env();
            self = format_ipv4(info.self.ipv4);
            port = info.self.port;
            hosts.clear();
            const int n = static_cast<int>(info.runners.size());
            for (size_t k = 0; k < info.runners.size(); ++k) {
                HostSpec h;
                h.ipv4 = info.runners[k].ipv4;
                h.slots = (np + n - 1) / n;
                hosts.push_back(h);
            }
        } else if (!platform.empty()) {
            throw std::invalid_argument("unknown platform " + platform);
        } else if (!hostfile.empty()) {
            std::ifstream in(hostfile);
            if (!in) throw std::invalid_argument("cannot open hostfile " + hostfile);
            std::stringstream ss;
            ss << in.rdbuf();
            hosts = HostList::parse_hostfile(ss.str());
        } else hosts = HostList::parse(host_list_str);
    } catch (const std::exception &e) {
        return e.what();
    }
    if (i >= argc) return "missing program name";
    prog = argv[i++];
    for (; i < argc; ++i) args.push_back(argv[i]);
    return "";
}

// ModelArts (reference: srcs/go/platforms/modelarts/modelarts.go:14-115):
// DLS_TASK_INDEX / DLS_TASK_NUMBER select this container among the
// BATCH_CUSTOM<i>_HOSTS "host:port" entries (one runner per container); a
// single-container job runs on 127.0.0.1:38888.
ContainerInfo parse_modelarts_env() {
    auto req_int = [](const char *k) {
        const char *v = std::getenv(k);
        if (!v || !*v) throw std::invalid_argument(std::string(k) + " not set");
        return std::stoi(v);
    };
    int idx = req_int("DLS_TASK_INDEX");
    const int num = req_int("DLS_TASK_NUMBER");
    if (num < 1) throw std::invalid_argument("DLS_TASK_NUMBER must be >= 1");
    ContainerInfo info;
    if (num == 1) {
        info.runners.push_back(PeerID{parse_ipv4("127.0.0.1"), 38888});
    } else {
        for (int i = 0; i < num; ++i) {
            std::string key = "BATCH_CUSTOM" + std::to_string(i) + "_HOSTS";
            const char *v = std::getenv(key.c_str());
            if (!v || !*v) throw std::invalid_argument(key + " not set");
            std::string hp = v;
            auto colon = hp.rfind(':');
            if (colon == std::string::npos) throw std::invalid_argument(key + ": host:port expected");
            std::string host = hp.substr(0, colon);
            int port = std::stoi(hp.substr(colon + 1));
            addrinfo hints{}, *res = nullptr;
            hints.ai_family = AF_INET;
            if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res)
                throw std::invalid_argument("cannot resolve " + host);
            uint32_t ip = ntohl(reinterpret_cast<sockaddr_in *>(res->ai_addr)->sin_addr.s_addr);
            freeaddrinfo(res);
            info.runners.push_back(PeerID{ip, static_cast<uint16_t>(port)});
        }
    }
    if (num == 1 && idx == 1) idx = 0;  // tolerated by the platform
    if (idx < 0 || idx >= num) throw std::invalid_argument("DLS_TASK_INDEX out of range");
    info.self = info.runners[idx];
    return info;
}

std::vector<uint32_t> local_ipv4s() {
    std::vector<uint32_t> out;
    ifaddrs *ifa = nullptr;
    if (getifaddrs(&ifa) != 0) return out;
    for (auto *p = ifa; p; p = p->ifa_next)
        if (p->ifa_addr && p->ifa_addr->sa_family == AF_INET)
            out.push_back(ntohl(reinterpret_cast<sockaddr_in *>(p->ifa_addr)->sin_addr.s_addr));
    freeifaddrs(ifa);
    return out;
}

uint32_t infer_self_ipv4(const std::string &self, const std::string &nic, const HostList &hosts) {
    if (self.empty() && nic.empty()) {
        // no hint: the local address that appears in the host list (so `-H node1:8,node2:8`
        // works unchanged on every node), else loopback
        auto mine = local_ipv4s();
        for (auto &h : hosts)
            for (uint32_t ip : mine)
                if (h.ipv4 == ip) return ip;
    }
    return infer_self_ipv4(self, nic);
}

uint32_t infer_self_ipv4(const std::string &self, const std::string &nic) {
    if (!self.empty()) return resolve_ipv4(self);
    if (!nic.empty()) {
        ifaddrs *ifa = nullptr;
        if (getifaddrs(&ifa) != 0) throw std::runtime_error("getifaddrs failed");
        uint32_t ip = 0;
        for (auto *p = ifa; p; p = p->ifa_next) {
            if (!p->ifa_addr || p->ifa_addr->sa_family != AF_INET || nic != p->ifa_name) continue;
            ip = ntohl(reinterpret_cast<sockaddr_in *>(p->ifa_addr)->sin_addr.s_addr);
            break;
        }
        freeifaddrs(ifa);
        if (!ip) throw std::runtime_error("no ipv4 found on " + nic);
        return ip;
    }
    return parse_ipv4("127.0.0.1");
}

std::vector<int> parse_visible_devices(const std::string &val, bool *ok) {
    std::vector<int> ids;
    *ok = true;
    if (val.empty()) return ids;
    std::stringstream ss(val);
    std::string part;
    while (std::getline(ss, part, ',')) {
        try {
            int n = std::stoi(part);
            if (n < 0) continue;
            for (int x : ids)
                if (x == n) *ok = false;
            ids.push_back(n);
        } catch (...) {
            *ok = false;
        }
    }
    if (!*ok) ids.clear();
    return ids;
}

int gpu_index(int local_rank) {
    const char *keys[] = {"HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"};
    for (auto *k : keys) {
        const char *v = std::getenv(k);
        if (!v || !*v) continue;
        bool ok = true;
        auto ids = parse_visible_devices(v, &ok);
        if (!ok) {
            KF_WARN("invalid value of %s: %s", k, v);
            return -1;
        }
        if (static_cast<int>(ids.size()) <= local_rank) {
            KF_WARN("%s=%s is not enough for local rank %d", k, v, local_rank);
            return -1;
        }
        return ids[local_rank];
    }
    return local_rank;
}

int GPUPool::get() {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < mask_.size(); ++i)
        if (mask_[i]) {
            mask_[i] = false;
            return static_cast<int>(i);
        }
    return -1;
}

void GPUPool::put(int id) {
    std::lock_guard<std::mutex> lk(mu_);
    if (id < 0 || id >= static_cast<int>(mask_.size())) return;
    if (mask_[id]) fatalf("GPU %d not allocated", id);
    mask_[id] = true;
}

}  // namespace launcher
}  // namespace kungfu
