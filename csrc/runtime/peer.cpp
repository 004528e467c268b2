// Peer implementation: see peer.hpp for the parity map.
#include <kungfu/log.hpp>
#include <kungfu/monitor.hpp>
#include <kungfu/peer.hpp>

#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace kungfu {

const char *const kEnvSelfSpec = "KUNGFU_SELF_SPEC";
const char *const kEnvInitPeers = "KUNGFU_INIT_PEERS";
const char *const kEnvInitRunners = "KUNGFU_INIT_RUNNERS";
const char *const kEnvParentID = "KUNGFU_PARENT_ID";
const char *const kEnvStrategy = "KUNGFU_ALLREDUCE_STRATEGY";
const char *const kEnvConfigServer = "KUNGFU_CONFIG_SERVER";
const char *const kEnvInitClusterVersion = "KUNGFU_INIT_CLUSTER_VERSION";
const char *const kEnvJobStartTimestamp = "KUNGFU_JOB_START_TIMESTAMP";
const char *const kEnvProcStartTimestamp = "KUNGFU_PROC_START_TIMESTAMP";

PeerConfig PeerConfig::single_mode() {
    PeerConfig c;
    c.self = PeerID{parse_ipv4("127.0.0.1"), PortRange().begin};
    c.init_peers = {c.self};
    c.strategy = default_strategy();
    c.single = true;
    return c;
}

PeerConfig PeerConfig::from_env() {
    if (!std::getenv(kEnvSelfSpec)) return single_mode();
    PeerConfig c;
    c.self = PeerID::parse(env_str(kEnvSelfSpec));
    auto parent = env_str(kEnvParentID);
    if (!parent.empty()) c.parent = PeerID::parse(parent);
    c.init_runners = PeerList::parse(env_str(kEnvInitRunners));
    c.init_peers = PeerList::parse(env_str(kEnvInitPeers));
    auto s = env_str(kEnvStrategy);
    if (s.empty()) c.strategy = default_strategy();
    else if (!parse_strategy(s, &c.strategy)) throw std::invalid_argument("invalid strategy: " + s);
    c.config_server = env_str(kEnvConfigServer);
    auto v = env_str(kEnvInitClusterVersion);
    c.init_cluster_version = v.empty() ? 0 : std::stoi(v);
    return c;
}

std::string Stage::encode() const {
    auto v = json::Value::object();
    v.set("Version", json::Value::number(version));
    v.set("Cluster", cluster.to_json());
    return json::dump(v);
}

Stage Stage::decode(const std::string &s) {
    auto v = json::parse(s);
    Stage st;
    st.version = static_cast<int>(v.at("Version").as_int());
    st.cluster = Cluster::from_json(v.at("Cluster"));
    return st;
}

// ---- Peer -------------------------------------------------------------------------

Peer::Peer(const PeerConfig &cfg) : cfg_(cfg) {
    router_.reset(new Router(cfg_.self, env_bool("KUNGFU_CONFIG_USE_UNIX_SOCK", true)));
    server_.reset(new Server(cfg_.self, router_.get(), env_bool("KUNGFU_CONFIG_USE_UNIX_SOCK", true)));
    version_ = cfg_.init_cluster_version;
    cluster_.runners = cfg_.init_runners;
    cluster_.workers = cfg_.init_peers;
}

Peer::~Peer() { close(); }

uint64_t Peer::uid() const {
    uint64_t hi = cfg_.self.ipv4;
    uint64_t lo = (static_cast<uint64_t>(cfg_.self.port) << 16) | static_cast<uint16_t>(cfg_.init_cluster_version);
    return (hi << 32) | lo;
}

void Peer::start() {
    if (started_) return;
    started_ = true;
    op_watchdog_set_label("peer " + cfg_.self.str());
    if (!cfg_.single) {
        server_->start();
        if (Monitor::get().enabled()) {
            uint16_t mport = static_cast<uint16_t>(cfg_.self.port + 10000);
            monitor_http_.reset(new HttpServer(mport, [](const HttpRequest &r) {
                HttpResponse resp;
                if (r.path == "/metrics") resp.body = Monitor::get().metrics_text();
                else resp.status = 404;
                return resp;
            }));
            try {
                monitor_http_->start();
                KF_INFO("kungfu peer %s started, monitoring endpoint http://%s:%d/metrics", cfg_.self.str().c_str(),
                        format_ipv4(cfg_.self.ipv4).c_str(), mport);
            } catch (const std::exception &e) {
                KF_WARN("monitor http: %s", e.what());
                monitor_http_.reset();
            }
        }
    }
    std::lock_guard<std::mutex> lk(mu_);
    update_locked();
}

void Peer::close() {
    if (monitor_http_) monitor_http_->stop();
    if (server_) server_->stop();
    if (router_) router_->client().close_all();
}

int Peer::cluster_version() {
    std::lock_guard<std::mutex> lk(mu_);
    return version_;
}

Cluster Peer::current_cluster() {
    std::lock_guard<std::mutex> lk(mu_);
    return cluster_;
}

std::shared_ptr<Session> Peer::session() {
    std::lock_guard<std::mutex> lk(mu_);
    if (!session_ && !detached_) update_locked();
    return session_;
}

bool Peer::update_locked() {
    StallDetector sd("update_to(" + cluster_.workers.str() + ")");
    server_->set_token(static_cast<uint32_t>(version_));
    if (updated_) return true;
    const PeerList &pl = cluster_.workers;
    if (!pl.contains(cfg_.self)) return false;
    router_->client().reset(pl, static_cast<uint32_t>(version_));
    session_ = std::make_shared<Session>(cfg_.strategy, cfg_.self, pl, router_.get());
    if (!cfg_.single && pl.size() > 1) session_->barrier();
    updated_ = true;
    return true;
}

bool Peer::consensus(const std::string &bytes) {
    auto s = session();
    if (!s) return false;
    return s->bytes_consensus(bytes.data(), bytes.size(), "kungfu::peer");
}

bool Peer::get_cluster_config(Cluster *c) {
    std::string body;
    int st = http_request("GET", cfg_.config_server, "", &body);
    if (st != 200) return false;
    try {
        *c = Cluster::from_json(json::parse(body));
    } catch (const std::exception &e) {
        KF_ERROR("bad cluster config: %s", e.what());
        return false;
    }
    return true;
}

bool Peer::propose_new_size(int n) {
    if (cfg_.config_server.empty()) {
        KF_WARN("propose_new_size: no config server");
        return false;
    }
    Cluster c = current_cluster().resize(n);
    std::string body = json::dump(c.to_json());
    std::string resp;
    int st = http_request("PUT", cfg_.config_server, body, &resp);
    if (st != 200) {
        KF_WARN("propose_new_size: config server returned %d", st);
        return false;
    }
    return true;
}

std::pair<bool, bool> Peer::propose(const Cluster &c) {
    StallDetector sd("propose(" + c.debug_string() + ")");
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (cluster_ == c) return {false, false};
    }
    if (!consensus(c.bytes())) {
        KF_ERROR("diverged proposal detected among peers: %s", c.workers.str().c_str());
        return {false, false};
    }
    Stage stage;
    {
        std::lock_guard<std::mutex> lk(mu_);
        stage.version = version_ + 1;
    }
    stage.cluster = c;
    std::string enc = stage.encode();
    double timeout = env_duration_sec("KUNGFU_CONFIG_WAIT_RUNNER_TIMEOUT", 300.0);
    std::vector<std::function<void()>> fs;
    for (auto &r : c.runners) {
        fs.push_back([this, r, &enc, timeout] {
            auto t0 = now_sec();
            int n = 0;
            while (router_->ping().ping(r, 1.0) < 0) {
                if (now_sec() - t0 > timeout) throw std::runtime_error("runner " + r.str() + " unreachable");
                ++n;
                std::this_thread::sleep_for(std::chrono::milliseconds(200));
            }
            if (n > 0) KF_WARN("%s is up after pinged %d times", r.str().c_str(), n + 1);
            router_->client().send(r, ConnType::CONTROL, "update", enc.data(), enc.size(), kNoFlag);
        });
    }
    par_run(std::move(fs));
    std::lock_guard<std::mutex> lk(mu_);
    if (cluster_.workers.disjoint(c.workers))
        KF_ERROR("full update detected: %s -> %s, state will be lost", cluster_.debug_string().c_str(),
                 c.debug_string().c_str());
    else if (!c.workers.empty() && !cluster_.workers.contains(c.workers[0]))
        KF_ERROR("new root cannot be a new worker, state will be lost");
    cluster_ = c;
    version_++;
    updated_ = false;
    session_.reset();
    bool keep = c.workers.contains(cfg_.self);
    return {true, !keep};
}

std::pair<bool, bool> Peer::resize_to(const Cluster &c) {
    auto r = propose(c);
    if (r.second) detached_ = true;
    else {
        std::lock_guard<std::mutex> lk(mu_);
        update_locked();
    }
    return r;
}

std::pair<bool, bool> Peer::resize_cluster_from_url() {
    Cluster c;
    for (int i = 0;; ++i) {
        if (!get_cluster_config(&c)) {
            KF_ERROR("get cluster config failed, using current config");
            c = current_cluster();
        }
        if (consensus(c.bytes())) {
            if (i > 0) KF_INFO("new peer list is consistent after %d failed attempts", i);
            break;
        }
        KF_WARN("diverged proposal detected, retrying");
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    return resize_to(c);
}

std::pair<bool, bool> Peer::resize_cluster(int n) {
    auto s = session();
    if (s && s->rank() == 0) propose_new_size(n);
    return resize_cluster_from_url();
}

void Peer::save(const std::string &name, const void *data, size_t len) { router_->store().save(name, data, len); }

void Peer::save_version(const std::string &version, const std::string &name, const void *data, size_t len) {
    router_->vstore().save(version, name, data, len);
}

bool Peer::request(int rank, const std::string &version, const std::string &name, void *buf, size_t len) {
    auto s = session();
    if (!s || rank < 0 || rank >= s->size()) return false;
    PeerID target = s->peers()[rank];
    if (target == cfg_.self) {
        bool ok = false;
        auto copy = [&](const void *d, size_t n) {
            if (n == len) {
                std::memcpy(buf, d, n);
                ok = true;
            }
        };
        if (version.empty()) router_->store().read(name, copy);
        else router_->vstore().read(version, name, copy);
        return ok;
    }
    return router_->p2p().request(target, version, name, buf, len);
}

std::vector<double> Peer::egress_rates() {
    auto s = session();
    if (!s) return {};
    return Monitor::get().egress_rates(s->peers());
}

// ---- ConfigServer -------------------------------------------------------------------

ConfigServer::ConfigServer(uint16_t port, const std::string &path) : path_(path) {
    http_.reset(new HttpServer(port, [this](const HttpRequest &r) { return handle(r); }));
}

ConfigServer::~ConfigServer() { stop(); }

void ConfigServer::start() { http_->start(); }

void ConfigServer::stop() {
    stopped_.store(true);
    cv_.notify_all();
    if (http_) http_->stop();
}

void ConfigServer::set_cluster(const Cluster &c) {
    std::lock_guard<std::mutex> lk(mu_);
    cluster_ = c;
    has_cluster_ = true;
    version_++;
}

int ConfigServer::version() {
    std::lock_guard<std::mutex> lk(mu_);
    return version_;
}

bool ConfigServer::wait_stopped(double timeout_sec) {
    std::unique_lock<std::mutex> lk(mu_);
    return cv_.wait_for(lk, std::chrono::duration<double>(timeout_sec), [&] { return stopped_.load(); });
}

HttpResponse ConfigServer::handle(const HttpRequest &r) {
    HttpResponse resp;
    if (r.path == "/stop") {
        stopped_.store(true);
        cv_.notify_all();
        resp.body = "stopping\n";
        return resp;
    }
    if (r.path != path_) {
        resp.status = 404;
        return resp;
    }
    std::lock_guard<std::mutex> lk(mu_);
    if (r.method == "GET") {
        if (!has_cluster_) {
            resp.status = 404;
            resp.body = "No Config Found.\n";
            return resp;
        }
        resp.content_type = "application/json";
        resp.body = json::dump(cluster_.to_json());
        return resp;
    }
    if (r.method == "PUT") {
        Cluster c;
        try {
            c = Cluster::from_json(json::parse(r.body));
        } catch (const std::exception &e) {
            resp.status = 400;
            resp.body = std::string("bad json: ") + e.what();
            return resp;
        }
        auto err = c.validate();
        if (!err.empty()) {
            resp.status = 400;
            resp.body = "invalid cluster config: " + err;
            return resp;
        }
        if (!has_cluster_) {
            version_ = 1;
            KF_INFO("config server: init first config to %zu workers", c.workers.size());
        } else if (cluster_.workers.empty()) {
            resp.status = 403;
            resp.body = "config was cleared, update rejected\n";
            return resp;
        } else version_++;
        cluster_ = c;
        has_cluster_ = true;
        return resp;
    }
    if (r.method == "POST" || r.method == "DELETE") {
        has_cluster_ = false;
        cluster_ = Cluster();
        return resp;
    }
    resp.status = 405;
    return resp;
}

}  // namespace kungfu
