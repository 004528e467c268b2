// extern "C" ABI over the global kungfu::Peer.  See capi.h.
#include <kungfu/capi.h>
#include <kungfu/log.hpp>
#include <kungfu/peer.hpp>
#include <kungfu/runtime.hpp>

#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

namespace kungfu {

namespace {
std::mutex g_mu;
std::unique_ptr<Peer> g_peer;
thread_local std::string g_err;
}  // namespace

Peer *global_peer() {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_peer.get();
}

Peer &require_peer() {
    Peer *p = global_peer();
    if (!p) throw std::runtime_error("kungfu: not initialised (call init first)");
    return *p;
}

std::shared_ptr<Session> require_session() {
    auto s = require_peer().session();
    if (!s) throw std::runtime_error("kungfu: no session (peer detached?)");
    return s;
}

void init_global_peer(const PeerConfig &cfg) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_peer) return;
    std::unique_ptr<Peer> p(new Peer(cfg));
    p->start();
    g_peer = std::move(p);
}

void finalize_global_peer() {
    std::unique_ptr<Peer> p;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        p = std::move(g_peer);
    }
    if (p) p->close();
}

void set_last_error(const std::string &e) { g_err = e; }

}  // namespace kungfu

using namespace kungfu;

#define KF_CAPI_TRY(body)                   \
    try {                                   \
        body;                               \
        return 0;                           \
    } catch (const std::exception &e) {     \
        set_last_error(e.what());           \
        return 1;                           \
    } catch (...) {                         \
        set_last_error("unknown error");    \
        return 1;                           \
    }

static Workspace ws(const void *s, void *r, size_t n, int dt, int op, const char *name) {
    return Workspace{s, r, n, static_cast<DType>(dt), static_cast<ReduceOp>(op), name ? name : ""};
}

extern "C" {

int kungfu_init(void) { KF_CAPI_TRY(init_global_peer(PeerConfig::from_env())) }

int kungfu_init_explicit(const char *self, const char *peers, const char *strategy, int version) {
    KF_CAPI_TRY({
        PeerConfig c;
        c.self = PeerID::parse(self);
        c.init_peers = PeerList::parse(peers);
        if (!strategy || !*strategy) c.strategy = default_strategy();
        else if (!parse_strategy(strategy, &c.strategy)) throw std::invalid_argument("bad strategy");
        c.init_cluster_version = version;
        c.single = c.init_peers.size() <= 1;
        init_global_peer(c);
    })
}

int kungfu_finalize(void) { KF_CAPI_TRY(finalize_global_peer()) }

const char *kungfu_last_error(void) { return g_err.c_str(); }

uint64_t kungfu_uid(void) {
    Peer *p = global_peer();
    return p ? p->uid() : 0;
}

int kungfu_detached(void) {
    Peer *p = global_peer();
    return p ? p->detached() : 0;
}

#define KF_SESSION_INT(fn, expr)                 \
    int fn(void) {                               \
        try {                                    \
            auto s = require_session();          \
            return expr;                         \
        } catch (...) {                          \
            return -1;                           \
        }                                        \
    }

KF_SESSION_INT(kungfu_rank, s->rank())
KF_SESSION_INT(kungfu_size, s->size())
KF_SESSION_INT(kungfu_local_rank, s->local_rank())
KF_SESSION_INT(kungfu_local_size, s->local_size())
KF_SESSION_INT(kungfu_host_count, s->host_count())

int kungfu_cluster_version(void) {
    Peer *p = global_peer();
    return p ? p->cluster_version() : -1;
}

int kungfu_barrier(void) { KF_CAPI_TRY(require_session()->barrier()) }

int kungfu_consensus(const void *data, size_t len, const char *name, int *ok) {
    KF_CAPI_TRY(*ok = require_session()->bytes_consensus(data, len, name ? name : ""))
}

int kungfu_all_reduce(const void *send, void *recv, size_t count, int dtype, int op, const char *name) {
    KF_CAPI_TRY(require_session()->all_reduce(ws(send, recv, count, dtype, op, name)))
}

int kungfu_all_reduce_async(const void *send, void *recv, size_t count, int dtype, int op, const char *name,
                            kungfu_callback_t cb, void *arg) {
    KF_CAPI_TRY({
        auto s = require_session();
        Workspace w = ws(send, recv, count, dtype, op, name);
        TaskPool::get().run([s, w, cb, arg] {
            int st = 0;
            try {
                s->all_reduce(w);
            } catch (const std::exception &e) {
                KF_ERROR("async all_reduce %s failed: %s", w.name.c_str(), e.what());
                st = 1;
            }
            if (cb) cb(st, arg);
        });
    })
}

int kungfu_cross_all_reduce(const void *send, void *recv, size_t count, int dtype, int op, const char *name) {
    KF_CAPI_TRY(require_session()->cross_all_reduce(ws(send, recv, count, dtype, op, name)))
}

int kungfu_monitored_all_reduce(const void *send, void *recv, size_t count, int dtype, int op, const char *name,
                                const int32_t *tree, int tree_len) {
    KF_CAPI_TRY({
        std::vector<int> t(tree, tree + (tree ? tree_len : 0));
        require_session()->monitored_all_reduce(ws(send, recv, count, dtype, op, name), &t);
    })
}

int kungfu_reduce(const void *send, void *recv, size_t count, int dtype, int op, const char *name) {
    KF_CAPI_TRY(require_session()->reduce(ws(send, recv, count, dtype, op, name)))
}

int kungfu_broadcast(const void *send, void *recv, size_t count, int dtype, const char *name) {
    KF_CAPI_TRY(require_session()->broadcast(ws(send, recv, count, dtype, 0, name)))
}

int kungfu_local_reduce(const void *send, void *recv, size_t count, int dtype, int op, const char *name) {
    KF_CAPI_TRY(require_session()->local_reduce(ws(send, recv, count, dtype, op, name)))
}

int kungfu_local_broadcast(const void *send, void *recv, size_t count, int dtype, const char *name) {
    KF_CAPI_TRY(require_session()->local_broadcast(ws(send, recv, count, dtype, 0, name)))
}

int kungfu_gather(const void *send, size_t count, int dtype, void *recv, const char *name) {
    KF_CAPI_TRY(require_session()->gather(ws(send, recv, count, dtype, 0, name)))
}

int kungfu_all_gather(const void *send, size_t count, int dtype, void *recv, const char *name) {
    KF_CAPI_TRY(require_session()->all_gather(ws(send, recv, count, dtype, 0, name)))
}

int kungfu_all_gather_transform(const void *send, size_t count, int dtype, void *out, size_t out_bytes,
                                kungfu_transform_t transform, void *arg, const char *name) {
    KF_CAPI_TRY(require_session()->all_gather_transform(
        send, count, static_cast<DType>(dtype), out, out_bytes,
        [&](const void *g, void *o) { transform(g, o, arg); }, name))
}

int kungfu_save(const char *name, const void *data, size_t len) { KF_CAPI_TRY(require_peer().save(name, data, len)) }

int kungfu_save_version(const char *version, const char *name, const void *data, size_t len) {
    KF_CAPI_TRY(require_peer().save_version(version, name, data, len))
}

int kungfu_request(int rank, const char *version, const char *name, void *buf, size_t len, int *found) {
    KF_CAPI_TRY(*found = require_peer().request(rank, version ? version : "", name, buf, len))
}

int kungfu_propose_new_size(int n) { KF_CAPI_TRY(require_peer().propose_new_size(n)) }

int kungfu_resize_cluster(int n, int *changed, int *detached) {
    KF_CAPI_TRY({
        auto r = require_peer().resize_cluster(n);
        *changed = r.first;
        *detached = r.second;
    })
}

int kungfu_resize_cluster_from_url(int *changed, int *detached) {
    KF_CAPI_TRY({
        auto r = require_peer().resize_cluster_from_url();
        *changed = r.first;
        *detached = r.second;
    })
}

int kungfu_set_tree(const int32_t *tree, int n) {
    KF_CAPI_TRY({
        std::vector<int> t(tree, tree + n);
        if (!require_session()->set_tree(t)) throw std::runtime_error("set_tree: no consensus");
    })
}

int kungfu_calc_stats(void) { KF_CAPI_TRY(require_session()->calc_stats()) }
int kungfu_log_stats(void) { KF_CAPI_TRY(require_session()->log_stats()) }

int kungfu_check_interference(int *switch_strategy) {
    KF_CAPI_TRY(*switch_strategy = require_session()->check_interference())
}

int kungfu_get_egress_rates(float *rates, int n) {
    KF_CAPI_TRY({
        auto r = require_peer().egress_rates();
        for (int i = 0; i < n && i < static_cast<int>(r.size()); ++i) rates[i] = static_cast<float>(r[i]);
    })
}

int kungfu_get_peer_latencies(float *lat, int n) {
    KF_CAPI_TRY({
        auto r = require_session()->peer_latencies();
        for (int i = 0; i < n && i < static_cast<int>(r.size()); ++i) lat[i] = static_cast<float>(r[i]);
    })
}

int kungfu_transform2(void *z, const void *x, const void *y, size_t n, int dtype, int op) {
    KF_CAPI_TRY(transform2(z, x, y, n, static_cast<DType>(dtype), static_cast<ReduceOp>(op)))
}

}  // extern "C"
