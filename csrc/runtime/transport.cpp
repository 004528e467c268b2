// Host transport implementation.  See transport.hpp for the parity map.
#include <kungfu/log.hpp>
#include <kungfu/monitor.hpp>
#include <kungfu/transport.hpp>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>

namespace kungfu {

namespace {

struct ConnHeader {
    uint32_t magic;
    uint16_t type;
    uint16_t src_port;
    uint32_t src_ipv4;
    uint32_t token;
};
static_assert(sizeof(ConnHeader) == 16, "ConnHeader layout");

enum : uint32_t { kAckOK = 0, kAckBadToken = 1, kAckBadMagic = 2 };

int retry_count() {
    static int n = [] {
        auto s = env_str("KUNGFU_CONFIG_CONN_RETRY_COUNT", "500");
        try { return std::max(1, std::stoi(s)); } catch (...) { return 500; }
    }();
    return n;
}

double retry_period() {
    static double p = env_duration_sec("KUNGFU_CONFIG_CONN_RETRY_PERIOD", 0.2);
    return p;
}

void set_sock_opts(int fd, bool tcp) {
    int one = 1;
    if (tcp) setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int buf = 4 << 20;
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

socklen_t make_uds_addr(const PeerID &p, sockaddr_un *addr) {
    std::memset(addr, 0, sizeof(*addr));
    addr->sun_family = AF_UNIX;
    std::string path = uds_path_for(p);
    // abstract namespace: leading NUL, no filesystem entry to clean up.
    addr->sun_path[0] = '\0';
    std::memcpy(addr->sun_path + 1, path.data(), std::min(path.size(), sizeof(addr->sun_path) - 2));
    return static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + 1 + path.size());
}

}  // namespace

std::string uds_path_for(const PeerID &p) { return "kungfu-amd-" + format_ipv4(p.ipv4) + "-" + std::to_string(p.port); }

bool write_full(int fd, const void *buf, size_t len) {
    const char *p = static_cast<const char *>(buf);
    while (len > 0) {
        ssize_t n = ::send(fd, p, len, MSG_NOSIGNAL);
        if (n < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        p += n;
        len -= static_cast<size_t>(n);
    }
    return true;
}

bool read_full(int fd, void *buf, size_t len) {
    char *p = static_cast<char *>(buf);
    while (len > 0) {
        ssize_t n = ::recv(fd, p, len, 0);
        if (n == 0) return false;
        if (n < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        p += n;
        len -= static_cast<size_t>(n);
    }
    return true;
}

// ---- BufferPool ----------------------------------------------------------------

BufferPool &BufferPool::get() {
    static BufferPool p;
    return p;
}

std::vector<char> BufferPool::take(size_t n) {
    if (n >= 512) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = free_.find(n);
        if (it != free_.end() && !it->second.empty()) {
            std::vector<char> b = std::move(it->second.back());
            it->second.pop_back();
            held_ -= n;
            return b;
        }
    }
    return std::vector<char>(n);
}

void BufferPool::put(std::vector<char> &&b) {
    size_t n = b.size();
    if (n < 512) return;
    std::lock_guard<std::mutex> lk(mu_);
    if (held_ + n > (size_t(1) << 30)) return;  // cap pooled bytes at 1 GiB
    held_ += n;
    free_[n].push_back(std::move(b));
}

// ---- Store ------------------------------------------------------------------------

void Store::save(const std::string &name, const void *data, size_t len) {
    std::shared_ptr<Blob> b;
    {
        std::lock_guard<std::mutex> lk(mu_);
        auto &slot = blobs_[name];
        if (!slot) slot = std::make_shared<Blob>();
        b = slot;
    }
    std::unique_lock<std::shared_mutex> wl(b->mu);
    b->data.resize(len);
    if (len) std::memcpy(b->data.data(), data, len);
}

bool Store::read(const std::string &name, const std::function<void(const void *, size_t)> &f) const {
    std::shared_ptr<Blob> b;
    {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = blobs_.find(name);
        if (it == blobs_.end()) return false;
        b = it->second;
    }
    std::shared_lock<std::shared_mutex> rl(b->mu);
    f(b->data.data(), b->data.size());
    return true;
}

bool Store::contains(const std::string &name) const {
    std::lock_guard<std::mutex> lk(mu_);
    return blobs_.count(name) > 0;
}

std::vector<std::string> Store::names() const {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<std::string> out;
    for (auto &kv : blobs_) out.push_back(kv.first);
    return out;
}

void VersionedStore::save(const std::string &version, const std::string &name, const void *data, size_t len) {
    std::shared_ptr<Store> s;
    {
        std::lock_guard<std::mutex> lk(mu_);
        auto &slot = stores_[version];
        if (!slot) {
            slot = std::make_shared<Store>();
            order_.push_back(version);
            while (order_.size() > window_) {
                stores_.erase(order_.front());
                order_.pop_front();
            }
        }
        s = stores_[version];
    }
    s->save(name, data, len);
}

bool VersionedStore::read(const std::string &version, const std::string &name,
                          const std::function<void(const void *, size_t)> &f) const {
    std::shared_ptr<Store> s;
    {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = stores_.find(version);
        if (it == stores_.end()) return false;
        s = it->second;
    }
    return s->read(name, f);
}

std::vector<std::string> VersionedStore::versions() const {
    std::lock_guard<std::mutex> lk(mu_);
    return std::vector<std::string>(order_.begin(), order_.end());
}

// ---- Client ------------------------------------------------------------------------

Client::Client(PeerID self, bool use_uds) : self_(self), use_uds_(use_uds) {}

Client::~Client() { close_all(); }

int Client::dial(const PeerID &dst, ConnType t) {
    const bool uds = use_uds_ && dst.ipv4 == self_.ipv4;
    const int tries = (t == ConnType::PING) ? 1 : retry_count();
    for (int attempt = 0; attempt < tries; ++attempt) {
        if (attempt) std::this_thread::sleep_for(std::chrono::duration<double>(retry_period()));
        int fd = -1;
        if (uds) {
            fd = ::socket(AF_UNIX, SOCK_STREAM, 0);
            sockaddr_un addr;
            socklen_t alen = make_uds_addr(dst, &addr);
            if (::connect(fd, reinterpret_cast<sockaddr *>(&addr), alen) != 0) {
                ::close(fd);
                continue;
            }
            set_sock_opts(fd, false);
        } else {
            fd = ::socket(AF_INET, SOCK_STREAM, 0);
            sockaddr_in addr{};
            addr.sin_family = AF_INET;
            addr.sin_port = htons(dst.port);
            addr.sin_addr.s_addr = htonl(dst.ipv4);
            if (::connect(fd, reinterpret_cast<sockaddr *>(&addr), sizeof(addr)) != 0) {
                ::close(fd);
                continue;
            }
            set_sock_opts(fd, true);
        }
        ConnHeader h{kConnMagic, static_cast<uint16_t>(t), self_.port, self_.ipv4, token_.load()};
        uint32_t ack = 0xffffffff;
        if (!write_full(fd, &h, sizeof(h)) || !read_full(fd, &ack, sizeof(ack)) || ack != kAckOK) {
            if (ack == kAckBadToken) KF_DEBUG("token rejected by %s, retrying", dst.str().c_str());
            ::close(fd);
            continue;
        }
        return fd;
    }
    return -1;
}

std::shared_ptr<Client::Conn> Client::get(const PeerID &dst, ConnType t) {
    std::shared_ptr<Conn> c;
    {
        std::lock_guard<std::mutex> lk(mu_);
        auto &slot = conns_[{dst.hash(), static_cast<uint16_t>(t)}];
        if (!slot) slot = std::make_shared<Conn>();
        c = slot;
    }
    return c;
}

void Client::send(const PeerID &dst, ConnType t, const std::string &name, const void *data, size_t len,
                  uint32_t flags) {
    auto c = get(dst, t);
    std::lock_guard<std::mutex> lk(c->mu);
    for (int attempt = 0; attempt < 2; ++attempt) {
        if (c->fd < 0) {
            c->fd = dial(dst, t);
            if (c->fd < 0)
                throw std::runtime_error("kungfu: cannot connect to " + dst.str() + " (" + uds_path_for(dst) + ")");
        }
        // header: u32 name_len | name | u32 flags | u64 len
        std::string hdr;
        uint32_t nl = static_cast<uint32_t>(name.size());
        uint64_t l64 = len;
        hdr.append(reinterpret_cast<const char *>(&nl), 4);
        hdr += name;
        hdr.append(reinterpret_cast<const char *>(&flags), 4);
        hdr.append(reinterpret_cast<const char *>(&l64), 8);
        iovec iov[2] = {{const_cast<char *>(hdr.data()), hdr.size()}, {const_cast<void *>(data), len}};
        size_t total = hdr.size() + len;
        size_t sent = 0;
        bool ok = true;
        int idx = 0;
        while (sent < total) {
            msghdr mh{};
            mh.msg_iov = iov + idx;
            mh.msg_iovlen = 2 - idx;
            ssize_t n = ::sendmsg(c->fd, &mh, MSG_NOSIGNAL);
            if (n < 0) {
                if (errno == EINTR) continue;
                ok = false;
                break;
            }
            sent += static_cast<size_t>(n);
            size_t adv = static_cast<size_t>(n);
            while (adv > 0 && idx < 2) {
                if (adv >= iov[idx].iov_len) {
                    adv -= iov[idx].iov_len;
                    iov[idx].iov_len = 0;
                    ++idx;
                } else {
                    iov[idx].iov_base = static_cast<char *>(iov[idx].iov_base) + adv;
                    iov[idx].iov_len -= adv;
                    adv = 0;
                }
            }
            while (idx < 2 && iov[idx].iov_len == 0) ++idx;
        }
        if (ok) {
            Monitor::get().egress(dst, total);
            return;
        }
        ::close(c->fd);
        c->fd = -1;
        if (sent > 0) break;  // partial message: cannot resend safely
    }
    throw std::runtime_error("kungfu: send to " + dst.str() + " failed");
}

void Client::reset(const PeerList &keeps, uint32_t token) {
    token_.store(token);
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = conns_.begin(); it != conns_.end();) {
        bool keep = false;
        for (auto &p : keeps)
            if (p.hash() == it->first.first) keep = true;
        // collective connections carry the token: re-dial them all.
        if (!keep || it->first.second == static_cast<uint16_t>(ConnType::COLLECTIVE)) {
            std::lock_guard<std::mutex> cl(it->second->mu);
            if (it->second->fd >= 0) ::close(it->second->fd);
            it->second->fd = -1;
            it = conns_.erase(it);
        } else ++it;
    }
}

void Client::close_all() {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto &kv : conns_) {
        std::lock_guard<std::mutex> cl(kv.second->mu);
        if (kv.second->fd >= 0) ::close(kv.second->fd);
        kv.second->fd = -1;
    }
    conns_.clear();
}

// ---- CollectiveEndpoint --------------------------------------------------------------

CollectiveEndpoint::Slot &CollectiveEndpoint::slot(const Key &k) {
    auto &s = slots_[k];
    if (!s) s.reset(new Slot);
    return *s;
}

void CollectiveEndpoint::maybe_erase(const Key &k) {
    auto it = slots_.find(k);
    if (it == slots_.end()) return;
    Slot &s = *it->second;
    if (s.queue.empty() && s.reg_buf == nullptr && s.waiters == 0) slots_.erase(it);
}

std::vector<char> CollectiveEndpoint::recv(const PeerID &src, const std::string &name) {
    Key k{src.hash(), name};
    std::unique_lock<std::mutex> lk(mu_);
    Slot &s = slot(k);
    s.waiters++;
    s.cv.wait(lk, [&] { return !s.queue.empty() || aborted_; });
    s.waiters--;
    if (aborted_) throw std::runtime_error("kungfu: collective endpoint aborted");
    std::vector<char> b = std::move(s.queue.front());
    s.queue.pop_front();
    maybe_erase(k);
    return b;
}

void CollectiveEndpoint::recv_into(const PeerID &src, const std::string &name, void *buf, size_t len) {
    Key k{src.hash(), name};
    std::unique_lock<std::mutex> lk(mu_);
    Slot &s = slot(k);
    if (!s.queue.empty()) {
        std::vector<char> b = std::move(s.queue.front());
        s.queue.pop_front();
        maybe_erase(k);
        lk.unlock();
        if (b.size() != len) throw std::runtime_error("kungfu: recv_into size mismatch for " + name);
        std::memcpy(buf, b.data(), len);
        BufferPool::get().put(std::move(b));
        return;
    }
    s.reg_buf = buf;
    s.reg_len = len;
    s.reg_done = false;
    s.waiters++;
    s.cv.wait(lk, [&] { return s.reg_done || !s.queue.empty() || aborted_; });
    s.waiters--;
    if (aborted_) throw std::runtime_error("kungfu: collective endpoint aborted");
    if (!s.reg_done) {
        // a message arrived into the queue (size mismatch path) — copy it.
        s.reg_buf = nullptr;
        std::vector<char> b = std::move(s.queue.front());
        s.queue.pop_front();
        maybe_erase(k);
        lk.unlock();
        if (b.size() != len) throw std::runtime_error("kungfu: recv_into size mismatch for " + name);
        std::memcpy(buf, b.data(), len);
        return;
    }
    s.reg_buf = nullptr;
    s.reg_done = false;
    maybe_erase(k);
}

void CollectiveEndpoint::on_message(const PeerID &src, const std::string &name, uint32_t, size_t len,
                                    const PayloadReader &read) {
    Key k{src.hash(), name};
    std::unique_lock<std::mutex> lk(mu_);
    Slot &s = slot(k);
    if (s.reg_buf && !s.reg_busy && !s.reg_done && s.queue.empty() && s.reg_len == len) {
        s.reg_busy = true;
        void *dst = s.reg_buf;
        lk.unlock();
        read(dst, len);  // zero-copy straight into the posted buffer
        lk.lock();
        s.reg_busy = false;
        s.reg_done = true;
        s.cv.notify_all();
        return;
    }
    lk.unlock();
    std::vector<char> b = BufferPool::get().take(len);
    read(b.data(), len);
    lk.lock();
    Slot &s2 = slot(k);
    s2.queue.push_back(std::move(b));
    s2.cv.notify_all();
}

void CollectiveEndpoint::abort() {
    std::lock_guard<std::mutex> lk(mu_);
    aborted_ = true;
    for (auto &kv : slots_) kv.second->cv.notify_all();
}

// ---- P2PEndpoint ------------------------------------------------------------------------

bool P2PEndpoint::request(const PeerID &target, const std::string &version, const std::string &name, void *buf,
                          size_t len) {
    Key k{target.hash(), name};
    Pending p;
    p.buf = buf;
    p.len = len;
    {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return pending_.count(k) == 0 || aborted_; });
        if (aborted_) return false;
        pending_[k] = &p;
    }
    try {
        client_->send(target, ConnType::P2P, name, version.data(), version.size(), kNoFlag);
    } catch (...) {
        std::lock_guard<std::mutex> lk(mu_);
        pending_.erase(k);
        cv_.notify_all();
        throw;
    }
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return p.done || aborted_; });
    pending_.erase(k);
    cv_.notify_all();
    return p.done && p.ok;
}

void P2PEndpoint::on_message(const PeerID &src, const std::string &name, uint32_t flags, size_t len,
                             const PayloadReader &read) {
    if (flags & kIsResponse) {
        Key k{src.hash(), name};
        Pending *p = nullptr;
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = pending_.find(k);
            if (it != pending_.end()) p = it->second;
        }
        bool ok = p && !(flags & kRequestFailed) && p->len == len;
        if (ok) read(p->buf, len);
        else {
            std::vector<char> sink(len);
            read(sink.data(), len);
        }
        if (p) {
            std::lock_guard<std::mutex> lk(mu_);
            p->ok = ok;
            p->done = true;
            cv_.notify_all();
        }
        return;
    }
    // request: payload = version string
    std::string version(len, '\0');
    read(&version[0], len);
    bool found = false;
    auto reply = [&](const void *data, size_t n) {
        found = true;
        client_->send(src, ConnType::P2P, name, data, n, kIsResponse);
    };
    try {
        if (version.empty()) store_->read(name, reply);
        else vstore_->read(version, name, reply);
        if (!found) client_->send(src, ConnType::P2P, name, nullptr, 0, kIsResponse | kRequestFailed);
    } catch (const std::exception &e) {
        KF_WARN("p2p response to %s failed: %s", src.str().c_str(), e.what());
    }
}

void P2PEndpoint::abort() {
    std::lock_guard<std::mutex> lk(mu_);
    aborted_ = true;
    cv_.notify_all();
}

// ---- PingEndpoint --------------------------------------------------------------------

double PingEndpoint::ping(const PeerID &target, double timeout_sec) {
    std::string name = "ping:" + std::to_string(seq_.fetch_add(1));
    auto t0 = std::chrono::steady_clock::now();
    try {
        client_->send(target, ConnType::PING, name, nullptr, 0, kNoFlag);
    } catch (...) {
        return -1;
    }
    std::unique_lock<std::mutex> lk(mu_);
    bool ok = cv_.wait_for(lk, std::chrono::duration<double>(timeout_sec), [&] { return done_.count(name) > 0; });
    done_.erase(name);
    if (!ok) return -1;
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void PingEndpoint::on_message(const PeerID &src, const std::string &name, uint32_t flags, size_t len,
                              const PayloadReader &read) {
    std::vector<char> sink(len);
    read(sink.data(), len);
    if (flags & kIsResponse) {
        std::lock_guard<std::mutex> lk(mu_);
        done_.insert(name);
        cv_.notify_all();
        return;
    }
    try {
        client_->send(src, ConnType::PING, name, nullptr, 0, kIsResponse);
    } catch (...) {
    }
}

// ---- ControlEndpoint -----------------------------------------------------------------

void ControlEndpoint::set_handler(const std::string &name, Handler h) {
    std::lock_guard<std::mutex> lk(mu_);
    handlers_[name] = std::move(h);
}

void ControlEndpoint::on_message(const PeerID &src, const std::string &name, uint32_t, size_t len,
                                 const PayloadReader &read) {
    std::string payload(len, '\0');
    if (len) read(&payload[0], len);
    else read(nullptr, 0);
    Handler h;
    {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = handlers_.find(name);
        if (it != handlers_.end()) h = it->second;
    }
    if (h) {
        h(src, payload);
        return;
    }
    if (name == "exit") {
        KF_INFO("exit control message from %s", src.str().c_str());
        std::fflush(stdout);
        std::fflush(stderr);
        std::_Exit(0);
    }
    KF_WARN("unhandled control message %s from %s", name.c_str(), src.str().c_str());
}

// ---- Router ----------------------------------------------------------------------------

Router::Router(PeerID self, bool use_uds)
    : self_(self), client_(self, use_uds), p2p_(&client_, &store_, &vstore_), ping_(&client_) {}

Router::~Router() {
    collective_.abort();
    p2p_.abort();
}

void Router::dispatch(ConnType t, const PeerID &src, const std::string &name, uint32_t flags, size_t len,
                      const PayloadReader &read) {
    switch (t) {
    case ConnType::COLLECTIVE: collective_.on_message(src, name, flags, len, read); break;
    case ConnType::P2P: p2p_.on_message(src, name, flags, len, read); break;
    case ConnType::PING: ping_.on_message(src, name, flags, len, read); break;
    case ConnType::CONTROL: control_.on_message(src, name, flags, len, read); break;
    }
}

// ---- Server -------------------------------------------------------------------------------

Server::Server(PeerID self, Router *router, bool use_uds) : self_(self), router_(router), use_uds_(use_uds) {}

Server::~Server() { stop(); }

void Server::start() {
    tcp_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(tcp_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_port = htons(self_.port);
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
    if (::bind(tcp_fd_, reinterpret_cast<sockaddr *>(&addr), sizeof(addr)) != 0 || ::listen(tcp_fd_, 256) != 0) {
        int e = errno;
        ::close(tcp_fd_);
        tcp_fd_ = -1;
        throw std::runtime_error("kungfu: cannot listen on port " + std::to_string(self_.port) + ": " +
                                 std::strerror(e));
    }
    acceptors_.emplace_back([this] { accept_loop(tcp_fd_); });
    if (use_uds_) {
        uds_fd_ = ::socket(AF_UNIX, SOCK_STREAM, 0);
        sockaddr_un ua;
        socklen_t alen = make_uds_addr(self_, &ua);
        if (::bind(uds_fd_, reinterpret_cast<sockaddr *>(&ua), alen) != 0 || ::listen(uds_fd_, 256) != 0) {
            KF_WARN("cannot listen on UDS %s: %s", uds_path_for(self_).c_str(), std::strerror(errno));
            ::close(uds_fd_);
            uds_fd_ = -1;
        } else acceptors_.emplace_back([this] { accept_loop(uds_fd_); });
    }
}

void Server::accept_loop(int lfd) {
    for (;;) {
        pollfd pfd{lfd, POLLIN, 0};
        int r = ::poll(&pfd, 1, 200);
        if (stopping_.load()) return;
        if (r <= 0) continue;
        int fd = ::accept(lfd, nullptr, nullptr);
        if (fd < 0) {
            if (stopping_.load()) return;
            continue;
        }
        std::lock_guard<std::mutex> lk(conns_mu_);
        if (stopping_.load()) {
            ::close(fd);
            return;
        }
        conn_fds_.insert(fd);
        conn_threads_.emplace_back([this, fd] { serve(fd); });
    }
}

void Server::serve(int fd) {
    ConnHeader h;
    auto done = [&] {
        std::lock_guard<std::mutex> lk(conns_mu_);
        if (conn_fds_.erase(fd)) ::close(fd);
    };
    if (!read_full(fd, &h, sizeof(h))) return done();
    uint32_t ack = kAckOK;
    if (h.magic != kConnMagic) ack = kAckBadMagic;
    else if (h.type == static_cast<uint16_t>(ConnType::COLLECTIVE) && h.token != token_.load()) ack = kAckBadToken;
    write_full(fd, &ack, sizeof(ack));
    if (ack != kAckOK) return done();
    PeerID src{h.src_ipv4, h.src_port};
    ConnType t = static_cast<ConnType>(h.type);
    std::string name;
    for (;;) {
        uint32_t nl = 0, flags = 0;
        uint64_t len = 0;
        if (!read_full(fd, &nl, 4)) break;
        if (nl > (1u << 20)) break;
        name.resize(nl);
        if (nl && !read_full(fd, &name[0], nl)) break;
        if (!read_full(fd, &flags, 4) || !read_full(fd, &len, 8)) break;
        bool consumed = false, ok = true;
        PayloadReader reader = [&](void *dst, size_t n) {
            consumed = true;
            if (n == 0) return;
            if (dst == nullptr) {
                std::vector<char> sink(n);
                ok = read_full(fd, sink.data(), n);
            } else ok = read_full(fd, dst, n);
        };
        try {
            router_->dispatch(t, src, name, flags, static_cast<size_t>(len), reader);
        } catch (const std::exception &e) {
            KF_WARN("dispatch error from %s: %s", src.str().c_str(), e.what());
        }
        if (!consumed && len > 0) {
            std::vector<char> sink(len);
            ok = read_full(fd, sink.data(), len);
        }
        if (!ok) break;
        Monitor::get().ingress(src, len + nl + 16);
    }
    done();
}

void Server::stop() {
    if (stopping_.exchange(true)) return;
    for (auto &t : acceptors_)
        if (t.joinable()) t.join();
    acceptors_.clear();
    if (tcp_fd_ >= 0) ::close(tcp_fd_);
    if (uds_fd_ >= 0) ::close(uds_fd_);
    tcp_fd_ = uds_fd_ = -1;
    std::vector<std::thread> threads;
    {
        std::lock_guard<std::mutex> lk(conns_mu_);
        for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
        threads.swap(conn_threads_);
    }
    for (auto &t : threads)
        if (t.joinable()) t.join();
}

}  // namespace kungfu
