// Peer: membership, cluster version, elastic resize, P2P store, and the
// current Session.  Plus the env contract between launcher and workers, the
// runner Stage message and the config server.
//
// Parity (reference paths relative to /root/reference/srcs/go/kungfu):
//   env contract            env/envs.go:4-18, env/config.go:24-68 (single mode when
//                           KUNGFU_SELF_SPEC is absent)
//   Peer New/Start/Update   peer/peer.go:27-166 (monitor HTTP on port+10000; UID)
//   resize / propose        peer/peer.go:168-276, peer/legacy.go:18-39
//   P2P                     peer/p2p.go:15-34
//   Stage                   runner/handler.go (update/exit control messages)
//   ConfigServer            elastic/configserver/configserver.go:15-112
#pragma once

#include <kungfu/http.hpp>
#include <kungfu/plan.hpp>
#include <kungfu/session.hpp>
#include <kungfu/transport.hpp>

#include <memory>
#include <mutex>
#include <string>

namespace kungfu {

struct PeerConfig {
    std::string config_server;
    PeerID parent;
    PeerList init_runners;
    PeerID self;
    Strategy strategy = Strategy::BINARY_TREE_STAR;
    int init_cluster_version = 0;
    PeerList init_peers;
    bool single = false;

    static PeerConfig from_env();  // throws on malformed env
    static PeerConfig single_mode();
};

// Env keys (launcher -> worker contract).
extern const char *const kEnvSelfSpec;
extern const char *const kEnvInitPeers;
extern const char *const kEnvInitRunners;
extern const char *const kEnvParentID;
extern const char *const kEnvStrategy;
extern const char *const kEnvConfigServer;
extern const char *const kEnvInitClusterVersion;
extern const char *const kEnvJobStartTimestamp;
extern const char *const kEnvProcStartTimestamp;

struct Stage {
    int version = 0;
    Cluster cluster;
    std::string encode() const;
    static Stage decode(const std::string &s);
};

class Peer {
  public:
    explicit Peer(const PeerConfig &cfg);
    ~Peer();

    void start();
    void close();

    bool single() const { return cfg_.single; }
    bool detached() const { return detached_; }
    uint64_t uid() const;
    PeerID self() const { return cfg_.self; }
    int cluster_version();
    Cluster current_cluster();
    std::shared_ptr<Session> session();  // current session (updates lazily)
    Router &router() { return *router_; }

    // Elastic API: returns {changed, detached}.
    bool propose_new_size(int n);  // rank 0 -> PUT config server
    std::pair<bool, bool> resize_cluster(int n);
    std::pair<bool, bool> resize_cluster_from_url();
    // Apply an explicit cluster (no config server): consensus + notify runners.
    std::pair<bool, bool> resize_to(const Cluster &c);

    // P2P
    void save(const std::string &name, const void *data, size_t len);
    void save_version(const std::string &version, const std::string &name, const void *data, size_t len);
    bool request(int rank, const std::string &version, const std::string &name, void *buf, size_t len);

    std::vector<double> egress_rates();

  private:
    bool update_locked();
    bool consensus(const std::string &bytes);
    std::pair<bool, bool> propose(const Cluster &c);
    bool get_cluster_config(Cluster *c);

    PeerConfig cfg_;
    std::unique_ptr<Router> router_;
    std::unique_ptr<Server> server_;
    std::unique_ptr<HttpServer> monitor_http_;
    std::mutex mu_;
    int version_ = 0;
    Cluster cluster_;
    std::shared_ptr<Session> session_;
    bool updated_ = false;
    bool detached_ = false;
    bool started_ = false;
};

class ConfigServer {
  public:
    ConfigServer(uint16_t port, const std::string &path = "/config");
    ~ConfigServer();
    void start();
    void stop();
    bool stopped() const { return stopped_.load(); }
    uint16_t port() const { return http_->port(); }
    void set_cluster(const Cluster &c);
    int version();
    bool wait_stopped(double timeout_sec);

  private:
    HttpResponse handle(const HttpRequest &r);
    std::string path_;
    std::unique_ptr<HttpServer> http_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool has_cluster_ = false;
    Cluster cluster_;
    int version_ = 0;
    std::atomic<bool> stopped_{false};
};

}  // namespace kungfu
