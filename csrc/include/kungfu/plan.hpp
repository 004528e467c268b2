// Planning layer: peer identities, peer lists, host specs, clusters, graphs and
// the all-reduce topology generators.
//
// Parity (reference paths relative to /root/reference/srcs/go/plan):
//   PeerID / addr          id.go:9-54, addr.go:11-59
//   PeerList               peerlist.go:11-191
//   HostSpec / HostList     hostspec.go:15-218 (port range 10000-11000, runner port 38080)
//   hostfile               hostfile/hostfile.go:14-81
//   Cluster                cluster.go:10-113 (Validate, Resize/growOne, Bytes)
//   Graph                  graph/graph.go:18-147 (self-loop = reduce into self)
//   topology generators    topology.go:17-160
//   subgraph generators    subgraph/subgraph.go:5-31
//   EvenPartition          interval.go:12-27 (see base.hpp even_partition)
#pragma once

#include <kungfu/base.hpp>
#include <kungfu/json.hpp>

#include <cstdint>
#include <string>
#include <vector>

namespace kungfu {

uint32_t parse_ipv4(const std::string &s);  // throws on error
// dotted IPv4, or a host / DNS name resolved to its first IPv4 address (throws on error)
uint32_t resolve_ipv4(const std::string &host);
std::string format_ipv4(uint32_t ip);

struct PeerID {
    uint32_t ipv4 = 0;
    uint16_t port = 0;

    bool operator==(const PeerID &o) const { return ipv4 == o.ipv4 && port == o.port; }
    bool operator!=(const PeerID &o) const { return !(*this == o); }
    bool operator<(const PeerID &o) const { return ipv4 != o.ipv4 ? ipv4 < o.ipv4 : port < o.port; }
    bool colocated_with(const PeerID &o) const { return ipv4 == o.ipv4; }
    std::string str() const;
    static PeerID parse(const std::string &s);  // "a.b.c.d:port"
    uint64_t hash() const { return (static_cast<uint64_t>(ipv4) << 16) | port; }
};

struct PeerList : std::vector<PeerID> {
    using std::vector<PeerID>::vector;

    int rank(const PeerID &p) const;        // -1 if absent
    int local_rank(const PeerID &p) const;  // -1 if absent
    int local_size(const PeerID &p) const;
    int host_count() const;
    bool contains(const PeerID &p) const { return rank(p) >= 0; }
    PeerList select(const std::vector<int> &ranks) const;
    PeerList others(const PeerID &self) const;
    PeerList on(uint32_t host) const;
    PeerList minus(const PeerList &q) const;
    PeerList intersection(const PeerList &q) const;
    bool disjoint(const PeerList &q) const { return intersection(q).empty(); }
    // masters: ranks of the first peer on each host; master_of[i] = master rank of peer i.
    void partition_by_host(std::vector<int> *masters, std::vector<int> *master_of) const;
    std::string str() const;  // comma-separated
    std::string bytes() const;
    static PeerList parse(const std::string &s);
};

struct PortRange {
    uint16_t begin = 10000, end = 11000;
    int cap() const { return end - begin + 1; }
    static PortRange parse(const std::string &s);  // "a-b"
    std::string str() const;
};

constexpr uint16_t kDefaultRunnerPort = 38080;

struct HostSpec {
    uint32_t ipv4 = 0;
    int slots = 1;
    std::string public_addr;
    std::string str() const;
    static HostSpec parse(const std::string &s);  // ip[:slots[:public_addr]]
};

struct HostList : std::vector<HostSpec> {
    int cap() const;
    int slot_of(uint32_t ipv4) const;
    std::string lookup_host(uint32_t ipv4) const;
    HostList shrink_to_fit(int np) const;
    PeerList gen_runner_list(uint16_t port) const;
    PeerList gen_peer_list(int np, const PortRange &pr) const;  // throws if no capacity
    std::string str() const;
    static HostList parse(const std::string &s);
    // OpenMPI-style hostfile: "ip slots=N public_addr=X", '#' comments.
    static HostList parse_hostfile(const std::string &content);
};

struct Cluster {
    PeerList runners;
    PeerList workers;

    bool operator==(const Cluster &o) const { return runners == o.runners && workers == o.workers; }
    std::string validate() const;  // "" if ok, else error message
    Cluster resize(int n) const;   // grow on the least loaded host / truncate
    std::string bytes() const;     // digest used for consensus
    std::string debug_string() const;
    json::Value to_json() const;
    static Cluster from_json(const json::Value &v);
};

class Graph {
  public:
    struct Node {
        bool self_loop = false;
        std::vector<int> prevs, nexts;
    };

    explicit Graph(int n = 0) : nodes_(n) {}
    int size() const { return static_cast<int>(nodes_.size()); }
    void add_edge(int i, int j);
    bool self_loop(int i) const { return nodes_[i].self_loop; }
    bool isolated(int i) const { return nodes_[i].prevs.empty() && nodes_[i].nexts.empty(); }
    const std::vector<int> &prevs(int i) const { return nodes_[i].prevs; }
    const std::vector<int> &nexts(int i) const { return nodes_[i].nexts; }
    Graph reverse() const;
    std::string digest() const;
    std::string debug_string() const;
    // father array: f[i] == i marks a root.  Returns false if invalid (range or cycle).
    static bool from_forest(const std::vector<int> &f, Graph *g, int *roots);

  private:
    std::vector<Node> nodes_;
};

// Topology generators (bcast graphs unless noted).
Graph gen_tree(const PeerList &peers);
Graph gen_binary_tree(int k);
Graph gen_binary_tree_star(const PeerList &peers, int offset = 0);
std::vector<Graph> gen_multi_binary_tree_star(const PeerList &peers);
Graph gen_multi_star(const PeerList &peers, int root_host);
std::vector<Graph> gen_multi_star_all(const PeerList &peers);
Graph gen_star_bcast(int k, int r);
// Ring: reduce chain ending at r and bcast chain starting at r.
void gen_circular_pair(int k, int r, Graph *reduce, Graph *bcast);
// reverse(bcast) + self-loops on every node.
Graph gen_default_reduce(const Graph &bcast);
// Minimum spanning tree (Prim) over an n x n weight matrix (row-major), which
// is symmetrised as w'[i][j] = w[i][j] + w[j][i].  Returns a father array
// rooted at `root` (f[root] == root).  Parity: srcs/cpp/include/kungfu/mst.hpp:9-58.
std::vector<int> minimum_spanning_tree(const std::vector<double> &w, int n, int root = 0);

// ---- Round schedule of a graph all-reduce for a two-sided, group-batched device data
// plane (RCCL send/recv over xGMI).  The host executor (session.cpp) walks the graphs
// with blocking per-edge transfers; a GPU plane instead needs every rank to issue the same
// sequence of batched send/recv groups.  Each strategy graph pair (reduce in-tree, bcast
// out-tree) owns one chunk of the buffer (even partition, like the reference's
// chunk->strategy map, srcs/go/kungfu/session/session.go:300-317).  Reduce round r
// (1..H) moves every chunk one tree level up: nodes of height r-1 send to their reduce
// father, fathers receive into scratch and reduce after the round; bcast round d moves
// every chunk one level down.  All chunks share the rounds, so CLIQUE becomes a
// link-parallel reduce-scatter + all-gather and RING the classic ring schedule.
struct GraphXfer {
    bool recv = false;
    int peer = 0;
    int64_t off = 0, len = 0;  // element range of the buffer
    int64_t scratch = -1;      // recv only: >= 0 -> land in scratch[scratch..], then buf[off..] op= it
};
struct GraphRound {
    std::vector<GraphXfer> ops;
};
struct GraphPlan {
    std::vector<GraphRound> rounds;
    int64_t scratch_elems = 0;
};
// pairs[c] = (reduce father array, bcast father array); f[i] == i marks the root.
GraphPlan plan_graph_all_reduce(const std::vector<std::pair<std::vector<int>, std::vector<int>>> &pairs, int rank,
                                int64_t count);
// (reduce father, bcast father) of a strategy graph pair; throws if a graph is not a tree.
std::pair<std::vector<int>, std::vector<int>> graph_pair_fathers(const Graph &reduce, const Graph &bcast);

// Subgraphs over a subset of vertices vs (used for cross-host all-reduce).
void gen_sub_circular_pair(int n, const std::vector<int> &vs, int r, Graph *reduce, Graph *bcast);
Graph gen_sub_binary_tree(int n, const std::vector<int> &vs);

}  // namespace kungfu
