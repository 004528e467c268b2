// Session implementation (graph-executed collectives).  See session.hpp.
#include <kungfu/log.hpp>
#include <kungfu/monitor.hpp>
#include <kungfu/session.hpp>

#include <algorithm>
#include <cstring>
#include <exception>
#include <stdexcept>

namespace kungfu {

double now_sec() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---- TaskPool ------------------------------------------------------------------------

TaskPool &TaskPool::get() {
    static TaskPool *p = new TaskPool();  // intentionally leaked: outlives static dtors
    return *p;
}

TaskPool::~TaskPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : threads_) t.join();
}

void TaskPool::worker() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
        ++idle_;
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        --idle_;
        if (stop_ && q_.empty()) return;
        auto f = std::move(q_.front());
        q_.pop_front();
        lk.unlock();
        f();
        lk.lock();
    }
}

void TaskPool::run(std::function<void()> f) {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(std::move(f));
    if (idle_ < static_cast<int>(q_.size())) {
        threads_.emplace_back([this] { worker(); });
    } else cv_.notify_one();
}

void par_run(std::vector<std::function<void()>> fs) {
    if (fs.empty()) return;
    if (fs.size() == 1) {
        fs[0]();
        return;
    }
    std::mutex mu;
    std::condition_variable cv;
    size_t remaining = fs.size() - 1;
    std::exception_ptr err;
    for (size_t i = 1; i < fs.size(); ++i) {
        auto *f = &fs[i];
        TaskPool::get().run([&, f] {
            std::exception_ptr e;
            try {
                (*f)();
            } catch (...) {
                e = std::current_exception();
            }
            std::lock_guard<std::mutex> lk(mu);
            if (e && !err) err = e;
            if (--remaining == 0) cv.notify_all();
        });
    }
    std::exception_ptr e0;
    try {
        fs[0]();
    } catch (...) {
        e0 = std::current_exception();
    }
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return remaining == 0; });
    if (e0) std::rethrow_exception(e0);
    if (err) std::rethrow_exception(err);
}

// ---- StrategyStat -----------------------------------------------------------------------

void StrategyStat::update(double begin, double end, uint64_t bytes) {
    std::lock_guard<std::mutex> lk(mu);
    if (first_begin < 0 || begin < first_begin) first_begin = begin;
    if (end > last_end) last_end = end;
    acc_bytes += bytes;
}

void StrategyStat::reset() {
    acc_bytes = 0;
    first_begin = -1;
    last_end = 0;
}

// ---- strategies ---------------------------------------------------------------------------

static GraphPair simple_pair(const Graph &bcast) {
    GraphPair p;
    p.bcast = bcast;
    p.reduce = gen_default_reduce(bcast);
    return p;
}

Strategy auto_select(const PeerList &peers) {
    return peers.host_count() == 1 ? Strategy::STAR : Strategy::BINARY_TREE_STAR;
}

StrategyList make_strategies(const PeerList &peers, Strategy s) {
    int k = static_cast<int>(peers.size());
    StrategyList sl;
    if (s == Strategy::AUTO) s = auto_select(peers);
    switch (s) {
    case Strategy::STAR: sl.push_back(simple_pair(gen_star_bcast(k, 0))); break;
    case Strategy::MULTI_STAR:
        for (auto &g : gen_multi_star_all(peers)) sl.push_back(simple_pair(g));
        break;
    case Strategy::CLIQUE:
        for (int r = 0; r < k; ++r) sl.push_back(simple_pair(gen_star_bcast(k, r)));
        break;
    case Strategy::RING:
        for (int r = 0; r < k; ++r) {
            GraphPair p;
            gen_circular_pair(k, r, &p.reduce, &p.bcast);
            sl.push_back(p);
        }
        break;
    case Strategy::TREE: sl.push_back(simple_pair(gen_tree(peers))); break;
    case Strategy::BINARY_TREE: sl.push_back(simple_pair(gen_binary_tree(k))); break;
    case Strategy::BINARY_TREE_STAR: sl.push_back(simple_pair(gen_binary_tree_star(peers, 0))); break;
    case Strategy::MULTI_BINARY_TREE_STAR:
        for (auto &g : gen_multi_binary_tree_star(peers)) sl.push_back(simple_pair(g));
        break;
    case Strategy::AUTO: break;
    }
    if (sl.empty()) sl.push_back(simple_pair(gen_star_bcast(k, 0)));
    return sl;
}

StrategyList make_local_strategies(const PeerList &peers) {
    std::vector<int> masters, master_of;
    peers.partition_by_host(&masters, &master_of);
    Graph g;
    int roots = 0;
    if (!Graph::from_forest(master_of, &g, &roots)) throw std::logic_error("bad local forest");
    return {simple_pair(g)};
}

StrategyList make_cross_strategies(const PeerList &peers, Strategy s) {
    std::vector<int> masters, master_of;
    peers.partition_by_host(&masters, &master_of);
    int n = static_cast<int>(peers.size());
    StrategyList sl;
    if (s == Strategy::RING) {
        for (size_t r = 0; r < masters.size(); ++r) {
            GraphPair p;
            gen_sub_circular_pair(n, masters, static_cast<int>(r), &p.reduce, &p.bcast);
            sl.push_back(p);
        }
    } else sl.push_back(simple_pair(gen_sub_binary_tree(n, masters)));
    return sl;
}

std::string strategy_list_digest(const StrategyList &sl) {
    std::string d;
    for (auto &p : sl) d += p.reduce.digest() + p.bcast.digest();
    return d;
}

// ---- Session -------------------------------------------------------------------------------

Session::Session(Strategy strategy, PeerID self, PeerList peers, Router *router)
    : strategy_(strategy == Strategy::AUTO ? auto_select(peers) : strategy),
      self_(self),
      peers_(std::move(peers)),
      router_(router) {
    rank_ = peers_.rank(self_);
    if (rank_ < 0) throw std::invalid_argument("self " + self_.str() + " not in peer list " + peers_.str());
    local_rank_ = peers_.local_rank(self_);
    local_size_ = peers_.local_size(self_);
    host_count_ = peers_.host_count();
    local_ = make_local_strategies(peers_);
    global_ = make_strategies(peers_, strategy_);
    cross_ = make_cross_strategies(peers_, strategy_);
    hash_by_name_ = env_str("KUNGFU_CONFIG_STRATEGY_HASH_METHOD", "NAME") == "NAME";
    double mib = 1.0;
    try {
        mib = std::stod(env_str("KUNGFU_CONFIG_CHUNK_SIZE_MIB", "1"));
    } catch (...) {
    }
    chunk_bytes_ = std::max<size_t>(4096, static_cast<size_t>(mib * (1 << 20)));
}

uint64_t Session::chunk_hash(size_t i, const std::string &name) const {
    if (!hash_by_name_) return i;
    uint64_t h = 0;
    for (unsigned char c : name) h += static_cast<uint64_t>(c) * c;
    return h;
}

void Session::run_graphs(const Workspace &w, const std::vector<const Graph *> &graphs) {
    if (w.empty()) return;
    bool iso = true;
    for (auto *g : graphs)
        if (!g->isolated(rank_)) iso = false;
    if (iso) {
        w.forward();
        return;
    }
    std::mutex lock;
    int recv_count = 0;
    auto effective = [&]() -> const void * { return (recv_count > 0 || w.inplace()) ? w.recv : w.send; };
    Client &client = router_->client();
    CollectiveEndpoint &ep = router_->collective();
    const size_t nbytes = w.bytes();

    for (auto *g : graphs) {
        const auto &prevs = g->prevs(rank_);
        const auto &nexts = g->nexts(rank_);
        if (g->self_loop(rank_)) {
            std::vector<std::function<void()>> fs;
            for (int p : prevs) {
                PeerID src = peers_[p];
                fs.push_back([&, src] {
                    std::vector<char> b = ep.recv(src, w.name);
                    if (b.size() != nbytes) throw std::runtime_error("kungfu: size mismatch in " + w.name);
                    std::lock_guard<std::mutex> lk(lock);
                    transform2(w.recv, effective(), b.data(), w.count, w.dtype, w.op);
                    ++recv_count;
                    BufferPool::get().put(std::move(b));
                });
            }
            par_run(std::move(fs));
            std::vector<std::function<void()>> ss;
            for (int q : nexts) {
                PeerID dst = peers_[q];
                ss.push_back([&, dst] { client.send(dst, ConnType::COLLECTIVE, w.name, effective(), nbytes, kNoFlag); });
            }
            par_run(std::move(ss));
        } else {
            if (prevs.size() > 1) KF_ERROR("more than one recv_into at node %d", rank_);
            if (prevs.empty() && recv_count == 0) w.forward();
            else
                for (int p : prevs) {
                    ep.recv_into(peers_[p], w.name, w.recv, nbytes);
                    ++recv_count;
                }
            std::vector<std::function<void()>> ss;
            for (int q : nexts) {
                PeerID dst = peers_[q];
                ss.push_back(
                    [&, dst] { client.send(dst, ConnType::COLLECTIVE, w.name, effective(), nbytes, kWaitRecvBuf); });
            }
            par_run(std::move(ss));
        }
    }
}

void Session::run_strategies(const Workspace &w, StrategyList &sl, bool monitored) {
    if (w.empty()) return;
    size_t k = (w.bytes() + chunk_bytes_ - 1) / chunk_bytes_;
    if (k == 0) k = 1;
    auto parts = w.split(k);
    std::vector<std::function<void()>> fs;
    for (size_t i = 0; i < parts.size(); ++i) {
        GraphPair *s = &sl[chunk_hash(i, parts[i].name) % sl.size()];
        Workspace *wp = &parts[i];
        fs.push_back([this, s, wp, monitored] {
            double t0 = monitored ? now_sec() : 0;
            run_graphs(*wp, {&s->reduce, &s->bcast});
            if (monitored) s->stat->update(t0, now_sec(), wp->bytes());
        });
    }
    par_run(std::move(fs));
}

void Session::barrier() {
    KF_TRACE_SCOPE("session::barrier");
    OpWatch watch("barrier");
    std::vector<uint8_t> x(peers_.size(), 0), y(peers_.size(), 0);
    Workspace w{x.data(), y.data(), x.size(), DType::U8, ReduceOp::SUM, "kungfu::barrier"};
    StrategyList sl;
    {
        std::lock_guard<std::mutex> lk(strat_mu_);
        sl = global_;
    }
    run_strategies(w, sl, false);
}

bool Session::bytes_consensus(const void *data, size_t len, const std::string &name) {
    int32_t n = static_cast<int32_t>(len), lo = 0, hi = 0;
    all_reduce({&n, &lo, 1, DType::I32, ReduceOp::MIN, ":consensus:len:min:" + name});
    all_reduce({&n, &hi, 1, DType::I32, ReduceOp::MAX, ":consensus:len:max:" + name});
    if (lo != hi) return false;
    if (len == 0) return true;
    std::vector<uint8_t> a(len), b(len);
    all_reduce({data, a.data(), len, DType::U8, ReduceOp::MIN, ":consensus:min:" + name});
    all_reduce({data, b.data(), len, DType::U8, ReduceOp::MAX, ":consensus:max:" + name});
    return a == b;
}

void Session::all_reduce(const Workspace &w) {
    KF_TRACE_SCOPE("session::all_reduce");
    OpWatch watch("all_reduce(" + w.name + ")");
    StrategyList sl;
    {
        std::lock_guard<std::mutex> lk(strat_mu_);
        sl = global_;
    }
    run_strategies(w, sl, false);
}

void Session::monitored_all_reduce(const Workspace &w, const std::vector<int> *tree) {
    OpWatch watch("monitored_all_reduce(" + w.name + ")");
    StrategyList sl;
    if (tree && !tree->empty()) {
        Graph g;
        int roots = 0;
        if (!Graph::from_forest(*tree, &g, &roots) || roots != 1)
            throw std::invalid_argument("monitored_all_reduce: invalid tree");
        sl.push_back(simple_pair(g));
    } else {
        std::lock_guard<std::mutex> lk(strat_mu_);
        sl = global_;
    }
    run_strategies(w, sl, true);
}

void Session::all_reduce_with(const std::vector<int> &forest, const Workspace &w) { monitored_all_reduce(w, &forest); }

void Session::cross_all_reduce(const Workspace &w) {
    OpWatch watch("cross_all_reduce(" + w.name + ")");
    run_strategies(w, cross_, false);
}

void Session::reduce(const Workspace &w) {
    OpWatch watch("reduce(" + w.name + ")");
    GraphPair s;
    {
        std::lock_guard<std::mutex> lk(strat_mu_);
        s = global_[0];
    }
    run_graphs(w, {&s.reduce});
}

void Session::broadcast(const Workspace &w) {
    OpWatch watch("broadcast(" + w.name + ")");
    GraphPair s;
    {
        std::lock_guard<std::mutex> lk(strat_mu_);
        s = global_[0];
    }
    run_graphs(w, {&s.bcast});
}

void Session::local_reduce(const Workspace &w) {
    OpWatch watch("local_reduce(" + w.name + ")");
    run_graphs(w, {&local_[0].reduce});
}
void Session::local_broadcast(const Workspace &w) {
    OpWatch watch("local_broadcast(" + w.name + ")");
    run_graphs(w, {&local_[0].bcast});
}

void Session::gather(const Workspace &w) {
    OpWatch watch("gather(" + w.name + ")");
    const size_t nbytes = w.bytes();
    if (rank_ != 0) {
        router_->client().send(peers_[0], ConnType::COLLECTIVE, w.name, w.send, nbytes, kWaitRecvBuf);
        return;
    }
    std::vector<std::function<void()>> fs;
    for (int r = 0; r < size(); ++r) {
        char *dst = static_cast<char *>(w.recv) + nbytes * r;
        if (r == rank_) {
            std::memmove(dst, w.send, nbytes);
            continue;
        }
        PeerID src = peers_[r];
        fs.push_back([this, src, dst, nbytes, &w] { router_->collective().recv_into(src, w.name, dst, nbytes); });
    }
    par_run(std::move(fs));
}

void Session::all_gather(const Workspace &w) {
    OpWatch watch("all_gather(" + w.name + ")");
    const size_t nbytes = w.bytes();
    std::vector<std::function<void()>> fs;
    for (int r = 0; r < size(); ++r) {
        if (r == rank_) continue;
        PeerID p = peers_[r];
        char *dst = static_cast<char *>(w.recv) + nbytes * r;
        fs.push_back([this, p, &w, nbytes] {
            router_->client().send(p, ConnType::COLLECTIVE, w.name, w.send, nbytes, kWaitRecvBuf);
        });
        fs.push_back([this, p, dst, &w, nbytes] { router_->collective().recv_into(p, w.name, dst, nbytes); });
    }
    std::memmove(static_cast<char *>(w.recv) + nbytes * rank_, w.send, nbytes);
    par_run(std::move(fs));
}

bool Session::set_global_strategy(const StrategyList &sl) {
    barrier();
    std::string d = strategy_list_digest(sl);
    bool ok = bytes_consensus(d.data(), d.size(), "kungfu::SetStrategy");
    if (ok) {
        std::lock_guard<std::mutex> lk(strat_mu_);
        global_ = sl;
    }
    barrier();
    return ok;
}

void Session::simple_set_global_strategy(const std::vector<int> &forest) {
    if (!set_tree(forest)) throw std::runtime_error("set_tree: no consensus on the new tree");
}

bool Session::set_tree(const std::vector<int> &forest) {
    if (static_cast<int>(forest.size()) != size()) throw std::invalid_argument("set_tree: forest size != cluster size");
    Graph g;
    int roots = 0;
    if (!Graph::from_forest(forest, &g, &roots) || roots != 1) throw std::invalid_argument("set_tree: invalid tree");
    return set_global_strategy({simple_pair(g)});
}

std::vector<double> Session::strategy_throughputs() {
    std::lock_guard<std::mutex> lk(strat_mu_);
    std::vector<double> out;
    for (auto &s : global_) out.push_back(s.stat->throughput);
    return out;
}

void Session::calc_stats() {
    std::lock_guard<std::mutex> lk(strat_mu_);
    if (global_.size() != 1) {
        KF_ERROR("calc_stats should only be called with one active strategy");
        return;
    }
    auto &st = *global_[0].stat;
    std::lock_guard<std::mutex> sl(st.mu);
    if (st.acc_bytes == 0) return;
    double dt = st.last_end - st.first_begin;
    st.throughput = dt > 0 ? static_cast<double>(st.acc_bytes) / dt : 0;
    st.reset();
}

void Session::log_stats() {
    auto t = strategy_throughputs();
    for (size_t i = 0; i < t.size(); ++i) KF_INFO("strategy #%zu throughput=%.3f MiB/s", i, t[i] / (1 << 20));
}

bool Session::check_interference() {
    std::shared_ptr<StrategyStat> st;
    {
        std::lock_guard<std::mutex> lk(strat_mu_);
        if (global_.size() != 1) {
            KF_ERROR("check_interference should only be called with one active strategy");
            return false;
        }
        st = global_[0].stat;
    }
    if (st->ref_throughput == 0) {
        st->ref_throughput = st->throughput;
        return false;
    }
    int8_t vote = st->throughput < 0.8 * st->ref_throughput ? 1 : 0, total = 0;
    all_reduce({&vote, &total, 1, DType::I8, ReduceOp::SUM, "kungfu::StratMon"});
    return total > size() / 2;
}

void Session::all_gather_transform(const void *send, size_t count, DType dtype, void *out, size_t out_bytes,
                                   const std::function<void(const void *, void *)> &f, const std::string &name) {
    const size_t esz = dtype_size(dtype);
    std::vector<char> gathered(rank_ == 0 ? count * esz * size() : 0);
    gather(Workspace{send, gathered.data(), count, dtype, ReduceOp::SUM, name + ":gather"});
    // A transform that throws on the root must not leave the other peers blocked in the
    // broadcast: the root always broadcasts a status byte first, then everyone raises.
    std::exception_ptr err;
    uint8_t failed = 0;
    if (rank_ == 0) {
        try {
            f(gathered.data(), out);
        } catch (...) {
            err = std::current_exception();
            failed = 1;
        }
    }
    broadcast(Workspace{&failed, &failed, 1, DType::U8, ReduceOp::SUM, name + ":status"});
    if (failed) {
        if (err) std::rethrow_exception(err);
        throw std::runtime_error("all_gather_transform(" + name + "): the transform failed on rank 0");
    }
    broadcast(Workspace{out, out, out_bytes, DType::U8, ReduceOp::SUM, name + ":bcast"});
}

void Session::send_to(int rank, const std::string &name, const void *data, size_t len) {
    if (rank < 0 || rank >= size() || rank == rank_) throw std::invalid_argument("send_to: bad rank");
    OpWatch watch("send_to(" + std::to_string(rank) + ", " + name + ")");
    router_->client().send(peers_[rank], ConnType::COLLECTIVE, name, data, len, kNoFlag);
}

void Session::recv_from(int rank, const std::string &name, void *buf, size_t len) {
    if (rank < 0 || rank >= size() || rank == rank_) throw std::invalid_argument("recv_from: bad rank");
    OpWatch watch("recv_from(" + std::to_string(rank) + ", " + name + ")");
    std::vector<char> b = router_->collective().recv(peers_[rank], name);
    if (b.size() != len) throw std::runtime_error("kungfu: size mismatch in " + name);
    if (len) std::memcpy(buf, b.data(), len);
    BufferPool::get().put(std::move(b));
}

void Session::record_strategy_stat(double begin, double end, uint64_t bytes) {
    std::vector<std::shared_ptr<StrategyStat>> sts;
    {
        std::lock_guard<std::mutex> lk(strat_mu_);
        for (auto &p : global_) sts.push_back(p.stat);
    }
    if (sts.empty()) return;
    // every strategy of the list carried an equal share of the chunks
    for (auto &st : sts) st->update(begin, end, bytes / sts.size());
}

std::vector<double> Session::peer_latencies() {
    std::vector<double> out(peers_.size(), 0.0);
    std::vector<std::function<void()>> fs;
    for (int r = 0; r < size(); ++r) {
        if (r == rank_) continue;
        fs.push_back([this, r, &out] { out[r] = router_->ping().ping(peers_[r]); });
    }
    par_run(std::move(fs));
    return out;
}

std::vector<std::pair<std::vector<int>, std::vector<int>>> Session::global_strategy_pairs() {
    std::lock_guard<std::mutex> lk(strat_mu_);
    std::vector<std::pair<std::vector<int>, std::vector<int>>> out;
    for (auto &p : global_) out.push_back(graph_pair_fathers(p.reduce, p.bcast));
    return out;
}

}  // namespace kungfu
