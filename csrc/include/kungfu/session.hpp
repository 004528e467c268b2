// Session: the collective engine for one cluster version (immutable peer list).
//
// Parity (reference paths relative to /root/reference/srcs/go/kungfu/session):
//   Session fields / New          session.go:20-66
//   Barrier / Consensus           session.go:92-151
//   Reduce / Broadcast / Local*   session.go:153-176
//   Gather / AllGather            session.go:185-207, allgather.go:13-45
//   graph executor runGraphs      session.go:218-286
//   1 MiB chunked multi-strategy  session.go:288-317, shard.go:11-31 (NAME hash = sum c^2)
//   strategies                    strategy.go:90-210
//   AllReduce / Cross / With      allreduce.go:11-40
//   SetGlobalStrategy             adaptation.go:8-28
//   stats / CheckInterference     strategy.go:15-56, adaptiveStrategies.go:12-127, monitoring.go:15-72
//
// Execution model: every chunk of a collective runs its reduce+bcast graph on
// a task of a growable thread pool (never blocks on pool capacity, so chunks
// that wait on peers cannot starve each other), mirroring the goroutine-per-
// chunk model of the reference without a Go runtime.
#pragma once

#include <kungfu/base.hpp>
#include <kungfu/plan.hpp>
#include <kungfu/transport.hpp>

#include <chrono>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace kungfu {

// Cached thread pool: reuse idle threads, grow when none is idle.
class TaskPool {
  public:
    static TaskPool &get();
    void run(std::function<void()> f);
    ~TaskPool();

  private:
    TaskPool() = default;
    void worker();
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    std::vector<std::thread> threads_;
    int idle_ = 0;
    bool stop_ = false;
};

// Run fs in parallel on the pool and wait; rethrows the first error.
void par_run(std::vector<std::function<void()>> fs);

struct StrategyStat {
    double throughput = 0;  // bytes/s of the last window
    double ref_throughput = 0;
    uint64_t acc_bytes = 0;
    double first_begin = -1, last_end = 0;
    std::mutex mu;
    void update(double begin, double end, uint64_t bytes);
    void reset();
};

struct GraphPair {
    Graph reduce, bcast;
    std::shared_ptr<StrategyStat> stat = std::make_shared<StrategyStat>();
};
using StrategyList = std::vector<GraphPair>;

StrategyList make_strategies(const PeerList &peers, Strategy s);
StrategyList make_local_strategies(const PeerList &peers);
StrategyList make_cross_strategies(const PeerList &peers, Strategy s);
Strategy auto_select(const PeerList &peers);
std::string strategy_list_digest(const StrategyList &sl);

class Session {
  public:
    Session(Strategy strategy, PeerID self, PeerList peers, Router *router);

    int size() const { return static_cast<int>(peers_.size()); }
    int rank() const { return rank_; }
    int local_rank() const { return local_rank_; }
    int local_size() const { return local_size_; }
    int host_count() const { return host_count_; }
    const PeerList &peers() const { return peers_; }
    Strategy strategy() const { return strategy_; }

    void barrier();
    bool bytes_consensus(const void *data, size_t len, const std::string &name);
    void all_reduce(const Workspace &w);
    void monitored_all_reduce(const Workspace &w, const std::vector<int> *tree = nullptr);
    void cross_all_reduce(const Workspace &w);
    void all_reduce_with(const std::vector<int> &forest, const Workspace &w);
    void reduce(const Workspace &w);     // to rank 0
    void broadcast(const Workspace &w);  // from rank 0
    void local_reduce(const Workspace &w);
    void local_broadcast(const Workspace &w);
    void gather(const Workspace &w);      // recv has count*np on root
    void all_gather(const Workspace &w);  // recv has count*np everywhere
    // Gather every peer's `send` (count x dtype) to rank 0, let rank 0 compute
    // `out_bytes` of output from the gathered [np x count] buffer with `f`, and
    // broadcast that output to every peer (parity: kungfu::Peer::AllGatherTransform,
    // srcs/cpp/src/session.cpp:162-181; used for topology-from-latencies flows).
    void all_gather_transform(const void *send, size_t count, DType dtype, void *out, size_t out_bytes,
                              const std::function<void(const void *gathered, void *out)> &f,
                              const std::string &name);

    // Adaptation
    bool set_global_strategy(const StrategyList &sl);  // barrier+consensus+swap+barrier
    void simple_set_global_strategy(const std::vector<int> &forest);
    bool set_tree(const std::vector<int> &forest);  // consensus-checked swap
    std::vector<double> strategy_throughputs();
    // (reduce father, bcast father) of every current global graph pair (device graph plane).
    std::vector<std::pair<std::vector<int>, std::vector<int>>> global_strategy_pairs();
    void log_stats();
    // Vote: true if the majority observed a throughput drop below 0.8x ref.
    bool check_interference();
    void calc_stats();

    std::vector<double> peer_latencies();

    // Named point-to-point transfers on the collective channel: the host-staged
    // backend of the device graph plane runs plan_graph_all_reduce rounds with them.
    void send_to(int rank, const std::string &name, const void *data, size_t len);
    void recv_from(int rank, const std::string &name, void *buf, size_t len);
    // Device planes (RCCL graph all-reduce timed with HIP events) report monitored
    // collectives here, so calc_stats / check_interference see GPU traffic too
    // (adaptiveStrategies.go:61-121, monitoring.go:15-35).  Times are seconds on
    // any clock that is consistent within one stats window.
    void record_strategy_stat(double begin, double end, uint64_t bytes);

  private:
    void run_graphs(const Workspace &w, const std::vector<const Graph *> &graphs);
    void run_strategies(const Workspace &w, StrategyList &sl, bool monitored);
    uint64_t chunk_hash(size_t i, const std::string &name) const;

    Strategy strategy_;
    PeerID self_;
    PeerList peers_;
    Router *router_;
    int rank_, local_rank_, local_size_, host_count_;
    std::mutex strat_mu_;
    StrategyList local_, global_, cross_;
    bool hash_by_name_;
    size_t chunk_bytes_;
};

double now_sec();

}  // namespace kungfu
