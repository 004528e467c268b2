// Python binding of the host runtime: kungfu_amd._kungfu
//
// Tensors cross the boundary as (data_ptr, count, dtype-code) so this module
// has no torch dependency; kungfu_amd.ops wraps it for torch tensors.  Every
// blocking call releases the GIL.  Async ops return integer handles backed by
// the runtime's task pool (parity: HandleManager + wait_handle,
// srcs/cpp/include/kungfu/utils/handler_manager.hpp:9-84 — but waits block on
// a condition variable instead of spinning).
#include <kungfu/log.hpp>
#include <kungfu/model_avg.hpp>
#include <kungfu/scheduler.hpp>
#include <kungfu/peer.hpp>
#include <kungfu/runtime.hpp>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <kungfu/monitor.hpp>
#include <set>

#include <condition_variable>
#include <map>
#include <mutex>

namespace py = pybind11;
using namespace kungfu;

namespace {

struct HandleTable {
    std::mutex mu;
    std::condition_variable cv;
    std::map<int64_t, int> done;  // handle -> status (0 ok, 1 error); absent = pending
    std::map<int64_t, std::string> errors;
    std::set<int64_t> pending;
    int64_t next = 1;

    int64_t create() {
        std::lock_guard<std::mutex> lk(mu);
        int64_t h = next++;
        pending.insert(h);
        return h;
    }
    void finish(int64_t h, int st, const std::string &err) {
        std::lock_guard<std::mutex> lk(mu);
        pending.erase(h);
        done[h] = st;
        if (st) errors[h] = err;
        cv.notify_all();
    }
    void wait(int64_t h) {
        std::string err;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return done.count(h) > 0; });
            if (done[h]) err = errors[h];
            done.erase(h);
            errors.erase(h);
        }
        if (!err.empty()) throw std::runtime_error(err);
    }
};

HandleTable &handles() {
    static HandleTable t;
    return t;
}

template <typename F>
int64_t submit(F f) {
    int64_t h = handles().create();
    auto s = require_session();
    TaskPool::get().run([h, f, s] {
        try {
            f(*s);
            handles().finish(h, 0, "");
        } catch (const std::exception &e) {
            handles().finish(h, 1, e.what());
        }
    });
    return h;
}

Workspace W(uintptr_t send, uintptr_t recv, size_t count, int dt, int op, const std::string &name) {
    return Workspace{reinterpret_cast<const void *>(send), reinterpret_cast<void *>(recv), count,
                     static_cast<DType>(dt), static_cast<ReduceOp>(op), name};
}

py::dict graph_to_dict(const Graph &g) {
    py::dict d;
    py::list nodes;
    for (int i = 0; i < g.size(); ++i) {
        py::dict n;
        n["self_loop"] = g.self_loop(i);
        n["prevs"] = g.prevs(i);
        n["nexts"] = g.nexts(i);
        nodes.append(n);
    }
    d["nodes"] = nodes;
    d["debug"] = g.debug_string();
    return d;
}

}  // namespace

PYBIND11_MODULE(_kungfu, m) {
    m.doc() = "kungfu-amd host runtime (C++): peers, sessions, graph collectives, P2P store, elastic resize";

    // ---- lifecycle -------------------------------------------------------
    m.def("init", [] {
        py::gil_scoped_release r;
        init_global_peer(PeerConfig::from_env());
    });
    m.def(
        "init_explicit",
        [](const std::string &self, const std::string &peers, const std::string &strategy, int version,
           const std::string &runners, const std::string &config_server) {
            PeerConfig c;
            c.self = PeerID::parse(self);
            c.init_peers = PeerList::parse(peers);
            c.init_runners = PeerList::parse(runners);
            c.config_server = config_server;
            if (strategy.empty()) c.strategy = default_strategy();
            else if (!parse_strategy(strategy, &c.strategy)) throw std::invalid_argument("bad strategy " + strategy);
            c.init_cluster_version = version;
            c.single = false;
            py::gil_scoped_release r;
            init_global_peer(c);
        },
        py::arg("self"), py::arg("peers"), py::arg("strategy") = "", py::arg("version") = 0,
        py::arg("runners") = "", py::arg("config_server") = "");
    m.def("finalize", [] {
        py::gil_scoped_release r;
        finalize_global_peer();
    });
    m.def("initialized", [] { return global_peer() != nullptr; });
    m.def("single", [] { return require_peer().single(); });
    m.def("uid", [] { return require_peer().uid(); });
    m.def("detached", [] { return require_peer().detached(); });
    m.def("self_spec", [] { return require_peer().self().str(); });
    m.def("cluster_version", [] { return require_peer().cluster_version(); });
    m.def("rank", [] { return require_session()->rank(); });
    m.def("size", [] { return require_session()->size(); });
    m.def("local_rank", [] { return require_session()->local_rank(); });
    m.def("local_size", [] { return require_session()->local_size(); });
    m.def("host_count", [] { return require_session()->host_count(); });
    m.def("peers", [] { return require_session()->peers().str(); });
    m.def("strategy", [] { return std::string(strategy_name(require_session()->strategy())); });

    // ---- collectives ----------------------------------------------------
    m.def("barrier", [] {
        auto s = require_session();
        py::gil_scoped_release r;
        s->barrier();
    });
    m.def("consensus", [](py::bytes data, const std::string &name) {
        std::string b = data;
        auto s = require_session();
        py::gil_scoped_release r;
        return s->bytes_consensus(b.data(), b.size(), name);
    });
    m.def("all_reduce", [](uintptr_t send, uintptr_t recv, size_t count, int dt, int op, const std::string &name) {
        auto s = require_session();
        py::gil_scoped_release r;
        s->all_reduce(W(send, recv, count, dt, op, name));
    });
    m.def("all_reduce_async",
          [](uintptr_t send, uintptr_t recv, size_t count, int dt, int op, const std::string &name) {
              auto w = W(send, recv, count, dt, op, name);
              return submit([w](Session &s) { s.all_reduce(w); });
          });
    m.def("broadcast_async", [](uintptr_t send, uintptr_t recv, size_t count, int dt, const std::string &name) {
        auto w = W(send, recv, count, dt, 0, name);
        return submit([w](Session &s) { s.broadcast(w); });
    });
    m.def("wait", [](int64_t h) {
        py::gil_scoped_release r;
        handles().wait(h);
    });
    m.def("wait_all", [](const std::vector<int64_t> &hs) {
        py::gil_scoped_release r;
        std::string first;
        for (auto h : hs) {
            try {
                handles().wait(h);
            } catch (const std::exception &e) {
                if (first.empty()) first = e.what();
            }
        }
        if (!first.empty()) throw std::runtime_error(first);
    });
    m.def("cross_all_reduce",
          [](uintptr_t send, uintptr_t recv, size_t count, int dt, int op, const std::string &name) {
              auto s = require_session();
              py::gil_scoped_release r;
              s->cross_all_reduce(W(send, recv, count, dt, op, name));
          });
    m.def(
        "monitored_all_reduce",
        [](uintptr_t send, uintptr_t recv, size_t count, int dt, int op, const std::string &name,
           std::vector<int> tree) {
            auto s = require_session();
            py::gil_scoped_release r;
            s->monitored_all_reduce(W(send, recv, count, dt, op, name), &tree);
        },
        py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"), py::arg("op"), py::arg("name"),
        py::arg("tree") = std::vector<int>{});
    m.def("reduce", [](uintptr_t send, uintptr_t recv, size_t count, int dt, int op, const std::string &name) {
        auto s = require_session();
        py::gil_scoped_release r;
        s->reduce(W(send, recv, count, dt, op, name));
    });
    m.def("broadcast", [](uintptr_t send, uintptr_t recv, size_t count, int dt, const std::string &name) {
        auto s = require_session();
        py::gil_scoped_release r;
        s->broadcast(W(send, recv, count, dt, 0, name));
    });
    m.def("local_reduce",
          [](uintptr_t send, uintptr_t recv, size_t count, int dt, int op, const std::string &name) {
              auto s = require_session();
              py::gil_scoped_release r;
              s->local_reduce(W(send, recv, count, dt, op, name));
          });
    m.def("local_broadcast", [](uintptr_t send, uintptr_t recv, size_t count, int dt, const std::string &name) {
        auto s = require_session();
        py::gil_scoped_release r;
        s->local_broadcast(W(send, recv, count, dt, 0, name));
    });
    m.def("gather", [](uintptr_t send, uintptr_t recv, size_t count, int dt, const std::string &name) {
        auto s = require_session();
        py::gil_scoped_release r;
        s->gather(W(send, recv, count, dt, 0, name));
    });
    m.def("all_gather", [](uintptr_t send, uintptr_t recv, size_t count, int dt, const std::string &name) {
        auto s = require_session();
        py::gil_scoped_release r;
        s->all_gather(W(send, recv, count, dt, 0, name));
    });

    // ---- p2p ----------------------------------------------------------------
    m.def("save", [](const std::string &name, uintptr_t data, size_t nbytes) {
        py::gil_scoped_release r;
        require_peer().save(name, reinterpret_cast<const void *>(data), nbytes);
    });
    m.def("save_version", [](const std::string &version, const std::string &name, uintptr_t data, size_t nbytes) {
        py::gil_scoped_release r;
        require_peer().save_version(version, name, reinterpret_cast<const void *>(data), nbytes);
    });
    m.def("request", [](int rank, const std::string &version, const std::string &name, uintptr_t buf,
                        size_t nbytes) {
        py::gil_scoped_release r;
        return require_peer().request(rank, version, name, reinterpret_cast<void *>(buf), nbytes);
    });

    // ---- ordered collective scheduler -----------------------------------------
    py::class_<OrderedScheduler>(m, "OrderedScheduler")
        .def(py::init<int>())
        .def("reset", &OrderedScheduler::reset)
        .def("ready", &OrderedScheduler::ready)
        .def("flush", &OrderedScheduler::flush)
        .def("set_order", &OrderedScheduler::set_order)
        .def("auto_order", [](OrderedScheduler &o) {
            auto s = require_session();
            py::gil_scoped_release r;
            o.auto_order(*s);
        })
        .def("order", &OrderedScheduler::order)
        .def("arrivals", &OrderedScheduler::arrivals)
        .def("size", &OrderedScheduler::size);
    py::class_<BucketTracker>(m, "BucketTracker")
        .def(py::init<int, const std::vector<int> &>())
        .def("mark", &BucketTracker::mark)
        .def("flush", &BucketTracker::flush)
        .def("reset", &BucketTracker::reset)
        .def("learn", &BucketTracker::learn)
        .def("learned", &BucketTracker::learned)
        .def("launched", &BucketTracker::launched)
        .def("fires", &BucketTracker::fires)
        .def("expected", &BucketTracker::expected)
        .def("auto_order", [](BucketTracker &t) {
            auto s = require_session();
            py::gil_scoped_release r;
            t.scheduler().auto_order(*s);
        })
        .def("set_order", [](BucketTracker &t, const std::vector<int> &o) { t.scheduler().set_order(o); })
        .def("order", [](BucketTracker &t) { return t.scheduler().order(); })
        .def("arrivals", [](BucketTracker &t) { return t.scheduler().arrivals(); })
        .def_property_readonly_static("LATE", [](py::object) { return BucketTracker::kLate; });

    // ---- model averaging (legacy pair-averaging ops) --------------------------
    py::class_<ModelAverager>(m, "ModelAverager")
        .def(py::init([](size_t count, const std::string &name, const std::string &selection) {
                 return new ModelAverager(&require_peer(), count, name, selection);
             }),
             py::arg("count"), py::arg("name") = "kungfu-model", py::arg("selection") = "random")
        .def("save", [](ModelAverager &a, uintptr_t p) {
            py::gil_scoped_release r;
            a.save(reinterpret_cast<const float *>(p));
        })
        .def("request", [](ModelAverager &a, uintptr_t p) {
            py::gil_scoped_release r;
            return a.request(reinterpret_cast<float *>(p));
        })
        .def("average", [](ModelAverager &a, uintptr_t p) {
            py::gil_scoped_release r;
            return a.average(reinterpret_cast<float *>(p));
        })
        .def("async_average", [](ModelAverager &a, uintptr_t p) {
            py::gil_scoped_release r;
            return a.async_average(reinterpret_cast<float *>(p));
        })
        .def("wait", &ModelAverager::wait, py::call_guard<py::gil_scoped_release>())
        .def("count", &ModelAverager::count)
        .def("pulls", &ModelAverager::pulls);
    m.def("peer_selector_sequence", [](const std::string &kind, const std::vector<int> &ranks, uint64_t seed,
                                       int n) {
        PeerSelector s(kind, ranks, seed);
        std::vector<int> out;
        for (int i = 0; i < n; ++i) out.push_back(s.next());
        return out;
    });

    // ---- elastic / adaptation ------------------------------------------------
    m.def("propose_new_size", [](int n) {
        py::gil_scoped_release r;
        return require_peer().propose_new_size(n);
    });
    m.def("resize_cluster", [](int n) {
        py::gil_scoped_release r;
        return require_peer().resize_cluster(n);
    });
    m.def("resize_cluster_from_url", [] {
        py::gil_scoped_release r;
        return require_peer().resize_cluster_from_url();
    });
    m.def("current_cluster", [] { return json::dump(require_peer().current_cluster().to_json()); });
    m.def("set_tree", [](const std::vector<int> &tree) {
        auto s = require_session();
        py::gil_scoped_release r;
        return s->set_tree(tree);
    });
    m.def("set_strategy", [](const std::string &name) {
        Strategy st;
        if (!parse_strategy(name, &st)) throw std::invalid_argument("bad strategy " + name);
        auto s = require_session();
        auto sl = make_strategies(s->peers(), st);
        py::gil_scoped_release r;
        return s->set_global_strategy(sl);
    });
    m.def("all_gather_transform", [](uintptr_t send, size_t count, int dt, uintptr_t out, size_t out_bytes,
                                     py::function f, const std::string &name) {
        auto s = require_session();
        const size_t esz = dtype_size(static_cast<DType>(dt));
        const int np = s->size();
        py::gil_scoped_release r;
        s->all_gather_transform(reinterpret_cast<const void *>(send), count, static_cast<DType>(dt),
                                reinterpret_cast<void *>(out), out_bytes,
                                [&](const void *g, void *o) {
                                    py::gil_scoped_acquire a;
                                    // f(gathered_ptr, gathered_bytes, out_ptr, out_bytes) on rank 0
                                    f(reinterpret_cast<uintptr_t>(g), count * esz * np, reinterpret_cast<uintptr_t>(o),
                                      out_bytes);
                                },
                                name);
    }, "gather to rank 0, transform there with f(gathered_ptr, nbytes, out_ptr, out_bytes), broadcast out");
    m.def("send_to", [](int rank, const std::string &name, uintptr_t data, size_t nbytes) {
        auto s = require_session();
        py::gil_scoped_release r;
        s->send_to(rank, name, reinterpret_cast<const void *>(data), nbytes);
    }, "named point-to-point send on the collective channel");
    m.def("recv_from", [](int rank, const std::string &name, uintptr_t buf, size_t nbytes) {
        auto s = require_session();
        py::gil_scoped_release r;
        s->recv_from(rank, name, reinterpret_cast<void *>(buf), nbytes);
    }, "named point-to-point receive (exact size)");
    m.def("now", [] { return now_sec(); }, "the steady clock the strategy statistics use (seconds)");
    m.def("record_strategy_stat", [](double begin, double end, uint64_t bytes) {
        require_session()->record_strategy_stat(begin, end, bytes);
    }, "account a monitored collective of a device plane to the current global strategy");
    m.def("calc_stats", [] { require_session()->calc_stats(); });
    m.def("log_stats", [] { require_session()->log_stats(); });
    m.def("strategy_throughputs", [] { return require_session()->strategy_throughputs(); });
    m.def("check_interference", [] {
        auto s = require_session();
        py::gil_scoped_release r;
        return s->check_interference();
    });
    m.def("peer_latencies", [] {
        auto s = require_session();
        py::gil_scoped_release r;
        return s->peer_latencies();
    });
    m.def("egress_rates", [] { return require_peer().egress_rates(); });
    m.def("monitor_enable", [](bool on) { Monitor::get().set_enabled(on); });
    m.def("metrics_text", [] { return Monitor::get().metrics_text(); });
    m.def("trace_report", [] { return trace_report(); });
    m.def("trace_enabled", [] { return trace_enabled(); });
    m.def("op_watchdog_timeout", [] { return op_watchdog_timeout(); });
    m.def("op_watchdog_set_timeout", [](double t) { op_watchdog_set_timeout(t); });
    m.def("op_watchdog_set_label", [](const std::string &l) { op_watchdog_set_label(l); });
    m.def("trace_push", [](const std::string &name) { trace_push(name.c_str()); });
    m.def("trace_pop", [] { trace_pop(); });
    m.def("trace_record", [](const std::string &name, double seconds) { trace_record(name, seconds); });

    // ---- host kernels ------------------------------------------------------------
    m.def("transform2", [](uintptr_t z, uintptr_t x, uintptr_t y, size_t n, int dt, int op) {
        py::gil_scoped_release r;
        transform2(reinterpret_cast<void *>(z), reinterpret_cast<const void *>(x), reinterpret_cast<const void *>(y),
                   n, static_cast<DType>(dt), static_cast<ReduceOp>(op));
    });
    m.def("dtype_size", [](int dt) { return dtype_size(static_cast<DType>(dt)); });

    // ---- plan utilities (pure logic; used by tests and the launcher shim) ----------
    m.def("strategy_names", [] {
        std::vector<std::string> out;
        for (auto s : all_strategies()) out.push_back(strategy_name(s));
        return out;
    });
    m.def("gen_strategy_graphs", [](const std::string &peers, const std::string &strategy) {
        Strategy st;
        if (!parse_strategy(strategy, &st)) throw std::invalid_argument("bad strategy " + strategy);
        auto sl = make_strategies(PeerList::parse(peers), st);
        py::list out;
        for (auto &p : sl) out.append(py::make_tuple(graph_to_dict(p.reduce), graph_to_dict(p.bcast)));
        return out;
    });
    m.def("strategy_pairs", [](const std::string &peers, const std::string &strategy) {
        Strategy st;
        if (!parse_strategy(strategy, &st)) throw std::invalid_argument("bad strategy " + strategy);
        std::vector<std::pair<std::vector<int>, std::vector<int>>> out;
        for (auto &p : make_strategies(PeerList::parse(peers), st)) out.push_back(graph_pair_fathers(p.reduce, p.bcast));
        return out;
    }, "(reduce father, bcast father) per graph pair of a strategy over a peer list");
    m.def("global_strategy_pairs", [] { return require_session()->global_strategy_pairs(); },
          "(reduce father, bcast father) per graph pair of the session's current global strategy");
    m.def("plan_graph_all_reduce", [](const std::vector<std::pair<std::vector<int>, std::vector<int>>> &pairs, int rank,
                                      int64_t count) {
        auto plan = plan_graph_all_reduce(pairs, rank, count);
        py::list rounds;
        for (auto &r : plan.rounds) {
            py::list ops;
            for (auto &x : r.ops) ops.append(py::make_tuple(x.recv ? 1 : 0, x.peer, x.off, x.len, x.scratch));
            rounds.append(ops);
        }
        return py::make_tuple(rounds, plan.scratch_elems);
    }, "round schedule of a graph all-reduce: ([[(recv, peer, off, len, scratch), ...], ...], scratch elems)");
    m.def("graph_from_forest", [](const std::vector<int> &f) {
        Graph g;
        int roots = 0;
        bool ok = Graph::from_forest(f, &g, &roots);
        if (!ok) return py::object(py::none());
        py::dict d = graph_to_dict(g);
        d["roots"] = roots;
        return py::object(d);
    });
    m.def("minimum_spanning_tree", [](const std::vector<double> &w, int n, int root) {
        return minimum_spanning_tree(w, n, root);
    }, py::arg("weights"), py::arg("n"), py::arg("root") = 0);
    m.def("cluster_resize", [](const std::string &cluster_json, int n) {
        return json::dump(Cluster::from_json(json::parse(cluster_json)).resize(n).to_json());
    });
    m.def("cluster_validate",
          [](const std::string &cluster_json) { return Cluster::from_json(json::parse(cluster_json)).validate(); });
    m.def("gen_peer_list", [](const std::string &hosts, int np, const std::string &port_range) {
        return HostList::parse(hosts).gen_peer_list(np, PortRange::parse(port_range)).str();
    });
    m.def("parse_hostfile", [](const std::string &content) { return HostList::parse_hostfile(content).str(); });
    m.def("partition_by_host", [](const std::string &peers) {
        std::vector<int> masters, master_of;
        PeerList::parse(peers).partition_by_host(&masters, &master_of);
        return py::make_tuple(masters, master_of);
    });
    m.def("even_partition", [](size_t n, size_t k) {
        std::vector<std::pair<size_t, size_t>> out;
        for (auto &iv : even_partition(n, k)) out.emplace_back(iv.begin, iv.end);
        return out;
    });

    // ---- config server --------------------------------------------------------------
    py::class_<ConfigServer>(m, "ConfigServer")
        .def(py::init<uint16_t, const std::string &>(), py::arg("port"), py::arg("path") = "/config")
        .def("start", &ConfigServer::start)
        .def("stop", &ConfigServer::stop, py::call_guard<py::gil_scoped_release>())
        .def("port", &ConfigServer::port)
        .def("version", &ConfigServer::version)
        .def("stopped", &ConfigServer::stopped)
        .def("set_cluster",
             [](ConfigServer &s, const std::string &cj) { s.set_cluster(Cluster::from_json(json::parse(cj))); });

    m.def("http_request", [](const std::string &method, const std::string &url, const std::string &body) {
        std::string resp;
        int st;
        {
            py::gil_scoped_release r;
            st = http_request(method, url, body, &resp);
        }
        return py::make_tuple(st, resp);
    });
}
