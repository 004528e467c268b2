// Host transport ("rchannel" equivalent): framed named messages over TCP and
// Unix-domain sockets, per-(peer, type) simplex connections, a version token on
// collective connections, zero-copy receive into registered buffers, one-sided
// P2P pulls served from a (versioned) model store, control and ping channels.
//
// Parity (reference paths relative to /root/reference/srcs/go/rchannel):
//   wire format + flags       connection/message.go:12-17,42-81,143-163
//   connection / UDS / token  connection/connection.go:57-178 (dial retry 500x200ms,
//                             kungfu/config/config.go:15-18)
//   byte-slice pool           connection/byte_slice_pool.go:7-60
//   client + conn pool        client/client.go:13-88, client/connection_pool.go:15-51
//   server (TCP + UDS)        server/server.go:16-133, server/composed.go:14-95
//   CollectiveEndpoint        handler/collective.go:10-65
//   PeerToPeerEndpoint        handler/p2p.go:13-120 (version window 3)
//   control / ping            handler/control.go:10-23, handler/ping.go:7-19
//   Store / VersionedStore    srcs/go/store/{blob,store,versionedstore}.go
//   router                    srcs/go/kungfu/peer/router.go:14-73
//
// MI355X-era design notes: connections are C++ threads over blocking sockets
// (no Go runtime); a receive that has not been posted yet lands in a pooled
// buffer and is memcpy'd on post, so a slow consumer never blocks the socket
// reader (the reference's WaitRecvBuf reader blocks); blob writes take the
// blob's exclusive lock (fixes the reference's Blob.CopyFrom race).
#pragma once

#include <kungfu/plan.hpp>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

namespace kungfu {

enum class ConnType : uint16_t { PING = 0, CONTROL = 1, COLLECTIVE = 2, P2P = 3 };

enum MsgFlag : uint32_t {
    kNoFlag = 0,
    kWaitRecvBuf = 1,
    kIsResponse = 2,
    kRequestFailed = 4,
};

constexpr uint32_t kConnMagic = 0x4b464d49;  // "KFMI"

// Pooled byte buffers (size-bucketed free lists).
class BufferPool {
  public:
    static BufferPool &get();
    std::vector<char> take(size_t n);
    void put(std::vector<char> &&b);

  private:
    std::mutex mu_;
    std::map<size_t, std::vector<std::vector<char>>> free_;
    size_t held_ = 0;
};

// ---------------------------------------------------------------------------
// Store

class Blob {
  public:
    std::vector<char> data;
    mutable std::shared_mutex mu;
};

class Store {
  public:
    // Creates or overwrites (exclusive lock on the blob).
    void save(const std::string &name, const void *data, size_t len);
    // Calls f(ptr, len) under the blob's shared lock; false if missing.
    bool read(const std::string &name, const std::function<void(const void *, size_t)> &f) const;
    bool contains(const std::string &name) const;
    std::vector<std::string> names() const;

  private:
    mutable std::mutex mu_;
    std::map<std::string, std::shared_ptr<Blob>> blobs_;
};

class VersionedStore {
  public:
    explicit VersionedStore(size_t window = 3) : window_(window) {}
    void save(const std::string &version, const std::string &name, const void *data, size_t len);
    bool read(const std::string &version, const std::string &name,
              const std::function<void(const void *, size_t)> &f) const;
    std::vector<std::string> versions() const;

  private:
    size_t window_;
    mutable std::mutex mu_;
    std::deque<std::string> order_;
    std::map<std::string, std::shared_ptr<Store>> stores_;
};

// ---------------------------------------------------------------------------
// Client

class Client {
  public:
    Client(PeerID self, bool use_uds);
    ~Client();

    // Throws std::runtime_error when the peer cannot be reached.
    void send(const PeerID &dst, ConnType t, const std::string &name, const void *data, size_t len,
              uint32_t flags = kNoFlag);
    // Drop connections to peers not in `keeps`, and use `token` for new
    // collective connections.
    void reset(const PeerList &keeps, uint32_t token);
    void close_all();
    uint32_t token() const { return token_.load(); }

  private:
    struct Conn {
        int fd = -1;
        std::mutex mu;
    };
    std::shared_ptr<Conn> get(const PeerID &dst, ConnType t);
    int dial(const PeerID &dst, ConnType t);

    PeerID self_;
    bool use_uds_;
    std::atomic<uint32_t> token_{0};
    std::mutex mu_;
    std::map<std::pair<uint64_t, uint16_t>, std::shared_ptr<Conn>> conns_;
};

// ---------------------------------------------------------------------------
// Endpoints

// Reads a message payload of `len` bytes into `dst`.
using PayloadReader = std::function<void(void *dst, size_t len)>;

class CollectiveEndpoint {
  public:
    // Blocking receive of the next message (src, name); returns its bytes.
    std::vector<char> recv(const PeerID &src, const std::string &name);
    // Blocking receive straight into [buf, buf+len).
    void recv_into(const PeerID &src, const std::string &name, void *buf, size_t len);
    void on_message(const PeerID &src, const std::string &name, uint32_t flags, size_t len,
                    const PayloadReader &read);
    // Unblock every waiter with an error (used on shutdown).
    void abort();

  private:
    struct Slot {
        std::deque<std::vector<char>> queue;
        void *reg_buf = nullptr;
        size_t reg_len = 0;
        bool reg_busy = false, reg_done = false;
        int waiters = 0;
        std::condition_variable cv;
    };
    using Key = std::pair<uint64_t, std::string>;
    Slot &slot(const Key &k);
    void maybe_erase(const Key &k);

    std::mutex mu_;
    std::map<Key, std::unique_ptr<Slot>> slots_;
    bool aborted_ = false;
};

class P2PEndpoint {
  public:
    P2PEndpoint(Client *client, Store *store, VersionedStore *vstore)
        : client_(client), store_(store), vstore_(vstore) {}
    // Pull `name` (at `version`, "" = latest unversioned) from `target` into buf.
    // Returns false if the target does not have it (or size mismatch).
    bool request(const PeerID &target, const std::string &version, const std::string &name, void *buf,
                 size_t len);
    void on_message(const PeerID &src, const std::string &name, uint32_t flags, size_t len,
                    const PayloadReader &read);
    void abort();

  private:
    struct Pending {
        void *buf = nullptr;
        size_t len = 0;
        bool done = false, ok = false;
    };
    using Key = std::pair<uint64_t, std::string>;
    Client *client_;
    Store *store_;
    VersionedStore *vstore_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::map<Key, Pending *> pending_;
    bool aborted_ = false;
};

class PingEndpoint {
  public:
    explicit PingEndpoint(Client *client) : client_(client) {}
    // Round-trip latency in seconds, or -1 on failure.
    double ping(const PeerID &target, double timeout_sec = 5.0);
    void on_message(const PeerID &src, const std::string &name, uint32_t flags, size_t len,
                    const PayloadReader &read);

  private:
    Client *client_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::set<std::string> done_;
    std::atomic<uint64_t> seq_{0};
};

// Control messages: name -> handler(payload).  Default "exit" exits the process.
class ControlEndpoint {
  public:
    using Handler = std::function<void(const PeerID &src, const std::string &payload)>;
    void set_handler(const std::string &name, Handler h);
    void on_message(const PeerID &src, const std::string &name, uint32_t flags, size_t len,
                    const PayloadReader &read);

  private:
    std::mutex mu_;
    std::map<std::string, Handler> handlers_;
};

// ---------------------------------------------------------------------------
// Server

class Router {
  public:
    Router(PeerID self, bool use_uds);
    ~Router();

    PeerID self() const { return self_; }
    Client &client() { return client_; }
    CollectiveEndpoint &collective() { return collective_; }
    P2PEndpoint &p2p() { return p2p_; }
    PingEndpoint &ping() { return ping_; }
    ControlEndpoint &control() { return control_; }
    Store &store() { return store_; }
    VersionedStore &vstore() { return vstore_; }

    void dispatch(ConnType t, const PeerID &src, const std::string &name, uint32_t flags, size_t len,
                  const PayloadReader &read);

  private:
    PeerID self_;
    Client client_;
    Store store_;
    VersionedStore vstore_;
    CollectiveEndpoint collective_;
    P2PEndpoint p2p_;
    PingEndpoint ping_;
    ControlEndpoint control_;
};

class Server {
  public:
    // Listens on 0.0.0.0:self.port (TCP) and, if use_uds, on the UDS path of self.
    Server(PeerID self, Router *router, bool use_uds);
    ~Server();
    void start();  // throws if the port cannot be bound
    void stop();
    void set_token(uint32_t t) { token_.store(t); }
    uint32_t token() const { return token_.load(); }
    uint16_t port() const { return self_.port; }

  private:
    void accept_loop(int lfd);
    void serve(int fd);

    PeerID self_;
    Router *router_;
    bool use_uds_;
    std::atomic<uint32_t> token_{0};
    int tcp_fd_ = -1, uds_fd_ = -1;
    std::string uds_path_;
    std::atomic<bool> stopping_{false};
    std::vector<std::thread> acceptors_;
    std::mutex conns_mu_;
    std::set<int> conn_fds_;
    std::vector<std::thread> conn_threads_;
};

std::string uds_path_for(const PeerID &p);

// Socket helpers (also used by the HTTP layer).
bool write_full(int fd, const void *buf, size_t len);
bool read_full(int fd, void *buf, size_t len);

}  // namespace kungfu
