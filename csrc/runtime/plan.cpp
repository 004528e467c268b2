// Planning layer implementation.  See plan.hpp for the parity map.
#include <kungfu/plan.hpp>

#include <netdb.h>
#include <netinet/in.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <set>
#include <sstream>
#include <stdexcept>

namespace kungfu {

namespace {

std::vector<std::string> split(const std::string &s, char sep) {
    std::vector<std::string> out;
    std::string cur;
    for (char c : s) {
        if (c == sep) {
            out.push_back(cur);
            cur.clear();
        } else cur.push_back(c);
    }
    out.push_back(cur);
    return out;
}

std::string trim(const std::string &s) {
    size_t b = s.find_first_not_of(" \t\r\n");
    if (b == std::string::npos) return "";
    size_t e = s.find_last_not_of(" \t\r\n");
    return s.substr(b, e - b + 1);
}

void put_u32(std::string &b, uint32_t v) {
    for (int i = 0; i < 4; ++i) b.push_back(static_cast<char>((v >> (8 * i)) & 0xff));
}

void put_u16(std::string &b, uint16_t v) {
    b.push_back(static_cast<char>(v & 0xff));
    b.push_back(static_cast<char>(v >> 8));
}

}  // namespace

uint32_t parse_ipv4(const std::string &s) {
    auto parts = split(s, '.');
    if (parts.size() != 4) throw std::invalid_argument("invalid IPv4: " + s);
    uint32_t ip = 0;
    for (auto &p : parts) {
        if (p.empty() || p.size() > 3) throw std::invalid_argument("invalid IPv4: " + s);
        for (char c : p)
            if (c < '0' || c > '9') throw std::invalid_argument("invalid IPv4: " + s);
        int v = std::stoi(p);
        if (v > 255) throw std::invalid_argument("invalid IPv4: " + s);
        ip = (ip << 8) | static_cast<uint32_t>(v);
    }
    return ip;
}

uint32_t resolve_ipv4(const std::string &host) {
    try {
        return parse_ipv4(host);
    } catch (const std::invalid_argument &) {
    }
    // hostname / DNS name (parity: runner/discovery.go resolution of -H entries)
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res)
        throw std::invalid_argument("cannot resolve host: " + host);
    uint32_t ip = ntohl(reinterpret_cast<sockaddr_in *>(res->ai_addr)->sin_addr.s_addr);
    freeaddrinfo(res);
    return ip;
}

std::string format_ipv4(uint32_t ip) {
    char buf[32];
    std::snprintf(buf, sizeof(buf), "%u.%u.%u.%u", (ip >> 24) & 0xff, (ip >> 16) & 0xff, (ip >> 8) & 0xff,
                  ip & 0xff);
    return buf;
}

std::string PeerID::str() const { return format_ipv4(ipv4) + ":" + std::to_string(port); }

PeerID PeerID::parse(const std::string &s) {
    auto pos = s.rfind(':');
    if (pos == std::string::npos) throw std::invalid_argument("invalid peer id: " + s);
    PeerID p;
    p.ipv4 = parse_ipv4(s.substr(0, pos));
    int port = std::stoi(s.substr(pos + 1));
    if (port < 0 || port > 65535) throw std::invalid_argument("invalid port: " + s);
    p.port = static_cast<uint16_t>(port);
    return p;
}

// ---- PeerList ----------------------------------------------------------------

int PeerList::rank(const PeerID &p) const {
    for (size_t i = 0; i < size(); ++i)
        if ((*this)[i] == p) return static_cast<int>(i);
    return -1;
}

int PeerList::local_rank(const PeerID &p) const {
    int i = 0;
    for (auto &q : *this) {
        if (q == p) return i;
        if (q.colocated_with(p)) ++i;
    }
    return -1;
}

int PeerList::local_size(const PeerID &p) const {
    int n = 0;
    for (auto &q : *this) n += q.colocated_with(p) ? 1 : 0;
    return n;
}

int PeerList::host_count() const {
    std::set<uint32_t> h;
    for (auto &q : *this) h.insert(q.ipv4);
    return static_cast<int>(h.size());
}

PeerList PeerList::select(const std::vector<int> &ranks) const {
    PeerList out;
    for (int r : ranks) out.push_back((*this)[r]);
    return out;
}

PeerList PeerList::others(const PeerID &self) const {
    PeerList out;
    for (auto &q : *this)
        if (q != self) out.push_back(q);
    return out;
}

PeerList PeerList::on(uint32_t host) const {
    PeerList out;
    for (auto &q : *this)
        if (q.ipv4 == host) out.push_back(q);
    return out;
}

PeerList PeerList::minus(const PeerList &q) const {
    PeerList out;
    for (auto &p : *this)
        if (!q.contains(p)) out.push_back(p);
    return out;
}

PeerList PeerList::intersection(const PeerList &q) const {
    PeerList out;
    for (auto &p : *this)
        if (q.contains(p)) out.push_back(p);
    return out;
}

void PeerList::partition_by_host(std::vector<int> *masters, std::vector<int> *master_of) const {
    std::map<uint32_t, int> host_master;
    masters->clear();
    master_of->assign(size(), 0);
    for (size_t r = 0; r < size(); ++r) {
        auto it = host_master.find((*this)[r].ipv4);
        if (it == host_master.end()) {
            host_master[(*this)[r].ipv4] = static_cast<int>(r);
            masters->push_back(static_cast<int>(r));
            (*master_of)[r] = static_cast<int>(r);
        } else (*master_of)[r] = it->second;
    }
}

std::string PeerList::str() const {
    std::string s;
    for (size_t i = 0; i < size(); ++i) {
        if (i) s.push_back(',');
        s += (*this)[i].str();
    }
    return s;
}

std::string PeerList::bytes() const {
    std::string b;
    for (auto &p : *this) {
        put_u32(b, p.ipv4);
        put_u16(b, p.port);
    }
    return b;
}

PeerList PeerList::parse(const std::string &s) {
    PeerList pl;
    if (trim(s).empty()) return pl;
    for (auto &p : split(s, ',')) pl.push_back(PeerID::parse(trim(p)));
    return pl;
}

// ---- hosts ---------------------------------------------------------------------

PortRange PortRange::parse(const std::string &s) {
    auto parts = split(s, '-');
    if (parts.size() != 2) throw std::invalid_argument("invalid port range: " + s);
    PortRange pr;
    int b = std::stoi(parts[0]), e = std::stoi(parts[1]);
    if (b < 0 || e > 65535 || e < b) throw std::invalid_argument("invalid port range: " + s);
    pr.begin = static_cast<uint16_t>(b);
    pr.end = static_cast<uint16_t>(e);
    return pr;
}

std::string PortRange::str() const { return std::to_string(begin) + "-" + std::to_string(end); }

std::string HostSpec::str() const { return format_ipv4(ipv4) + ":" + std::to_string(slots) + ":" + public_addr; }

HostSpec HostSpec::parse(const std::string &s) {
    auto parts = split(s, ':');
    if (parts.empty() || parts.size() > 3) throw std::invalid_argument("invalid host spec: " + s);
    HostSpec h;
    h.ipv4 = resolve_ipv4(parts[0]);
    h.slots = parts.size() >= 2 ? std::stoi(parts[1]) : 1;
    h.public_addr = parts.size() == 3 ? parts[2] : parts[0];
    if (h.slots < 0) throw std::invalid_argument("invalid slots: " + s);
    return h;
}

int HostList::cap() const {
    int c = 0;
    for (auto &h : *this) c += h.slots;
    return c;
}

int HostList::slot_of(uint32_t ipv4) const {
    for (auto &h : *this)
        if (h.ipv4 == ipv4) return h.slots;
    return 0;
}

std::string HostList::lookup_host(uint32_t ipv4) const {
    for (auto &h : *this)
        if (h.ipv4 == ipv4) return h.public_addr;
    return format_ipv4(ipv4);
}

HostList HostList::shrink_to_fit(int np) const {
    HostList out;
    int c = 0;
    for (auto &h : *this) {
        out.push_back(h);
        c += h.slots;
        if (c >= np) break;
    }
    return out;
}

PeerList HostList::gen_runner_list(uint16_t port) const {
    PeerList pl;
    for (auto &h : *this) pl.push_back({h.ipv4, port});
    return pl;
}

PeerList HostList::gen_peer_list(int np, const PortRange &pr) const {
    if (cap() < np) throw std::runtime_error("not enough capacity: need " + std::to_string(np));
    for (auto &h : *this)
        if (pr.cap() < h.slots) throw std::runtime_error("port range too small for host slots");
    PeerList pl;
    for (auto &h : *this)
        for (int j = 0; j < h.slots && static_cast<int>(pl.size()) < np; ++j)
            pl.push_back({h.ipv4, static_cast<uint16_t>(pr.begin + j)});
    return pl;
}

std::string HostList::str() const {
    std::string s;
    for (size_t i = 0; i < size(); ++i) {
        if (i) s.push_back(',');
        s += (*this)[i].str();
    }
    return s;
}

HostList HostList::parse(const std::string &s) {
    HostList hl;
    if (trim(s).empty()) return hl;
    for (auto &p : split(s, ',')) hl.push_back(HostSpec::parse(trim(p)));
    return hl;
}

HostList HostList::parse_hostfile(const std::string &content) {
    HostList hl;
    std::istringstream in(content);
    std::string line;
    while (std::getline(in, line)) {
        auto hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        line = trim(line);
        if (line.empty()) continue;
        std::istringstream ls(line);
        std::string tok;
        ls >> tok;
        HostSpec h;
        h.ipv4 = parse_ipv4(tok);
        h.slots = 1;
        h.public_addr = tok;
        while (ls >> tok) {
            auto eq = tok.find('=');
            if (eq == std::string::npos) throw std::invalid_argument("invalid hostfile token: " + tok);
            std::string k = tok.substr(0, eq), v = tok.substr(eq + 1);
            if (k == "slots") h.slots = std::stoi(v);
            else if (k == "public_addr") h.public_addr = v;
            else throw std::invalid_argument("unknown hostfile key: " + k);
        }
        hl.push_back(h);
    }
    return hl;
}

// ---- Cluster -------------------------------------------------------------------

std::string Cluster::validate() const {
    std::set<uint32_t> hosts;
    std::set<uint64_t> ids;
    for (auto &r : runners) {
        if (!ids.insert(r.hash()).second) return "duplicated port";
        if (!hosts.insert(r.ipv4).second) return "duplicated runner";
    }
    for (auto &w : workers) {
        if (!ids.insert(w.hash()).second) return "duplicated port";
        if (!hosts.count(w.ipv4)) return "missing runner";
    }
    return "";
}

Cluster Cluster::resize(int n) const {
    Cluster d = *this;
    if (static_cast<int>(d.workers.size()) > n) d.workers.resize(n);
    while (static_cast<int>(d.workers.size()) < n) {
        if (d.runners.empty()) throw std::runtime_error("resize: no runner");
        std::map<uint32_t, int> used;
        for (auto &r : d.runners) used[r.ipv4] = 0;
        for (auto &w : d.workers) used[w.ipv4]++;
        uint32_t ip = d.runners[0].ipv4;
        for (auto &r : d.runners)
            if (used[r.ipv4] < used[ip]) ip = r.ipv4;
        uint32_t port = 0;
        for (auto &w : d.workers)
            if (w.ipv4 == ip && port <= w.port) port = w.port + 1u;
        if (port == 0) port = PortRange().begin;
        d.workers.push_back({ip, static_cast<uint16_t>(port)});
    }
    return d;
}

std::string Cluster::bytes() const {
    std::string b = "R" + runners.bytes() + "W" + workers.bytes();
    return b;
}

std::string Cluster::debug_string() const {
    return "[" + std::to_string(workers.size()) + "@" + std::to_string(runners.size()) + "]{" + workers.str() +
           "}@{" + runners.str() + "}";
}

json::Value Cluster::to_json() const {
    auto v = json::Value::object();
    auto rs = json::Value::array(), ws = json::Value::array();
    for (auto &r : runners) rs.push(json::Value::string(r.str()));
    for (auto &w : workers) ws.push(json::Value::string(w.str()));
    v.set("Runners", rs);
    v.set("Workers", ws);
    return v;
}

Cluster Cluster::from_json(const json::Value &v) {
    Cluster c;
    if (auto *rs = v.get("Runners"))
        for (auto &r : rs->a) c.runners.push_back(PeerID::parse(r.s));
    if (auto *ws = v.get("Workers"))
        for (auto &w : ws->a) c.workers.push_back(PeerID::parse(w.s));
    return c;
}

// ---- Graph -----------------------------------------------------------------------

void Graph::add_edge(int i, int j) {
    if (i == j) {
        nodes_[i].self_loop = true;
        return;
    }
    nodes_[i].nexts.push_back(j);
    nodes_[j].prevs.push_back(i);
}

Graph Graph::reverse() const {
    Graph r(size());
    for (int i = 0; i < size(); ++i) {
        for (int j : nodes_[i].nexts) r.nodes_[j].nexts.push_back(i);
        for (int j : nodes_[i].prevs) r.nodes_[j].prevs.push_back(i);
    }
    return r;
}

std::string Graph::digest() const {
    std::string b;
    put_u32(b, static_cast<uint32_t>(size()));
    for (auto &n : nodes_) {
        auto vs = n.nexts;
        std::sort(vs.begin(), vs.end());
        put_u32(b, n.self_loop ? 1u : 0u);
        put_u32(b, static_cast<uint32_t>(vs.size()));
        for (int j : vs) put_u32(b, static_cast<uint32_t>(j));
    }
    return b;
}

std::string Graph::debug_string() const {
    std::string s = "[" + std::to_string(size()) + "]{";
    for (int i = 0; i < size(); ++i)
        if (nodes_[i].self_loop) s += "(" + std::to_string(i) + ")";
    for (int i = 0; i < size(); ++i)
        for (int j : nodes_[i].nexts) s += "(" + std::to_string(i) + "->" + std::to_string(j) + ")";
    return s + "}";
}

bool Graph::from_forest(const std::vector<int> &f, Graph *g, int *roots) {
    int n = static_cast<int>(f.size());
    *g = Graph(n);
    int m = 0;
    for (int i = 0; i < n; ++i) {
        if (f[i] < 0 || f[i] >= n) return false;
        if (f[i] == i) ++m;
        else g->add_edge(f[i], i);
    }
    // cycle check: every node must reach a root by following fathers.
    for (int i = 0; i < n; ++i) {
        int x = i, steps = 0;
        while (f[x] != x) {
            x = f[x];
            if (++steps > n) return false;
        }
    }
    if (roots) *roots = m;
    return true;
}

// ---- generators --------------------------------------------------------------

static void local_masters(const PeerList &peers, std::vector<int> *masters, std::map<uint32_t, int> *hm) {
    for (size_t r = 0; r < peers.size(); ++r) {
        if (!hm->count(peers[r].ipv4)) {
            (*hm)[peers[r].ipv4] = static_cast<int>(r);
            masters->push_back(static_cast<int>(r));
        }
    }
}

static void add_host_stars(const PeerList &peers, const std::map<uint32_t, int> &hm, Graph *g) {
    for (size_t r = 0; r < peers.size(); ++r) {
        int m = hm.at(peers[r].ipv4);
        if (m != static_cast<int>(r)) g->add_edge(m, static_cast<int>(r));
    }
}

Graph gen_tree(const PeerList &peers) {
    Graph g(static_cast<int>(peers.size()));
    std::vector<int> masters;
    std::map<uint32_t, int> hm;
    local_masters(peers, &masters, &hm);
    add_host_stars(peers, hm, &g);
    for (size_t i = 1; i < masters.size(); ++i) g.add_edge(masters[0], masters[i]);
    return g;
}

Graph gen_binary_tree(int k) {
    Graph g(k);
    for (int i = 0; i < k; ++i) {
        if (2 * i + 1 < k) g.add_edge(i, 2 * i + 1);
        if (2 * i + 2 < k) g.add_edge(i, 2 * i + 2);
    }
    return g;
}

Graph gen_binary_tree_star(const PeerList &peers, int offset) {
    Graph g(static_cast<int>(peers.size()));
    std::vector<int> masters;
    std::map<uint32_t, int> hm;
    local_masters(peers, &masters, &hm);
    add_host_stars(peers, hm, &g);
    int k = static_cast<int>(masters.size());
    if (k > 1) {
        auto idx = [&](int i) { return masters[(i + offset) % k]; };
        for (int i = 0; i < k; ++i) {
            if (2 * i + 1 < k) g.add_edge(idx(i), idx(2 * i + 1));
            if (2 * i + 2 < k) g.add_edge(idx(i), idx(2 * i + 2));
        }
    }
    return g;
}

std::vector<Graph> gen_multi_binary_tree_star(const PeerList &peers) {
    std::vector<int> masters;
    std::map<uint32_t, int> hm;
    local_masters(peers, &masters, &hm);
    std::vector<Graph> gs;
    for (size_t i = 0; i < masters.size(); ++i) gs.push_back(gen_binary_tree_star(peers, static_cast<int>(i)));
    return gs;
}

Graph gen_multi_star(const PeerList &peers, int root_host) {
    Graph g(static_cast<int>(peers.size()));
    std::vector<int> masters;
    std::map<uint32_t, int> hm;
    local_masters(peers, &masters, &hm);
    add_host_stars(peers, hm, &g);
    int k = static_cast<int>(masters.size());
    if (k > 1)
        for (int i = 0; i < k; ++i)
            if (i != root_host) g.add_edge(masters[root_host], masters[i]);
    return g;
}

std::vector<Graph> gen_multi_star_all(const PeerList &peers) {
    std::vector<int> masters;
    std::map<uint32_t, int> hm;
    local_masters(peers, &masters, &hm);
    std::vector<Graph> gs;
    for (size_t i = 0; i < masters.size(); ++i) gs.push_back(gen_multi_star(peers, static_cast<int>(i)));
    return gs;
}

Graph gen_star_bcast(int k, int r) {
    Graph g(k);
    for (int i = 0; i < k; ++i)
        if (i != r) g.add_edge(r, i);
    return g;
}

void gen_circular_pair(int k, int r, Graph *reduce, Graph *bcast) {
    *reduce = Graph(k);
    *bcast = Graph(k);
    for (int i = 0; i < k; ++i) reduce->add_edge(i, i);
    for (int i = 1; i < k; ++i) {
        reduce->add_edge((r + i) % k, (r + i + 1) % k);
        bcast->add_edge((r + i - 1) % k, (r + i) % k);
    }
}

Graph gen_default_reduce(const Graph &bcast) {
    Graph g = bcast.reverse();
    for (int i = 0; i < g.size(); ++i) g.add_edge(i, i);
    return g;
}

std::vector<int> minimum_spanning_tree(const std::vector<double> &w, int n, int root) {
    if (static_cast<int>(w.size()) != n * n) throw std::invalid_argument("mst: weight matrix must be n*n");
    std::vector<int> father(n, root);
    if (n == 0) return father;
    std::vector<double> best(n, 1e300);
    std::vector<bool> in(n, false);
    best[root] = 0;
    father[root] = root;
    for (int it = 0; it < n; ++it) {
        int u = -1;
        for (int v = 0; v < n; ++v)
            if (!in[v] && (u < 0 || best[v] < best[u])) u = v;
        in[u] = true;
        for (int v = 0; v < n; ++v) {
            if (in[v]) continue;
            double c = w[u * n + v] + w[v * n + u];
            if (c < best[v]) {
                best[v] = c;
                father[v] = u;
            }
        }
    }
    return father;
}

void gen_sub_circular_pair(int n, const std::vector<int> &vs, int r, Graph *reduce, Graph *bcast) {
    *reduce = Graph(n);
    *bcast = Graph(n);
    int k = static_cast<int>(vs.size());
    for (int i = 0; i < k; ++i) reduce->add_edge(vs[i], vs[i]);
    for (int i = 1; i < k; ++i) {
        reduce->add_edge(vs[(r + i) % k], vs[(r + i + 1) % k]);
        bcast->add_edge(vs[(r + i - 1) % k], vs[(r + i) % k]);
    }
}

Graph gen_sub_binary_tree(int n, const std::vector<int> &vs) {
    Graph g(n);
    int k = static_cast<int>(vs.size());
    for (int i = 0; i < k; ++i) {
        if (2 * i + 1 < k) g.add_edge(vs[i], vs[2 * i + 1]);
        if (2 * i + 2 < k) g.add_edge(vs[i], vs[2 * i + 2]);
    }
    return g;
}

// ---------------------------------------------------------------- device graph rounds

namespace {

struct TreeInfo {
    int root = -1;
    std::vector<std::vector<int>> children;
    std::vector<int> level;  // height (reduce) or depth (bcast)
};

TreeInfo tree_info(const std::vector<int> &f, bool heights) {
    const int n = static_cast<int>(f.size());
    TreeInfo t;
    t.children.assign(n, {});
    t.level.assign(n, 0);
    for (int i = 0; i < n; ++i) {
        if (f[i] < 0 || f[i] >= n) throw std::invalid_argument("graph plan: father out of range");
        if (f[i] == i) {
            if (t.root >= 0) throw std::invalid_argument("graph plan: forest with several roots");
            t.root = i;
        } else {
            t.children[f[i]].push_back(i);
        }
    }
    if (n > 0 && t.root < 0) throw std::invalid_argument("graph plan: no root");
    // BFS order from the root (also detects cycles / unreachable nodes)
    std::vector<int> order;
    if (n > 0) order.push_back(t.root);
    for (size_t k = 0; k < order.size(); ++k)
        for (int c : t.children[order[k]]) order.push_back(c);
    if (static_cast<int>(order.size()) != n) throw std::invalid_argument("graph plan: not a tree");
    if (heights) {
        for (auto it = order.rbegin(); it != order.rend(); ++it)
            for (int c : t.children[*it]) t.level[*it] = std::max(t.level[*it], t.level[c] + 1);
    } else {
        for (int v : order)
            for (int c : t.children[v]) t.level[c] = t.level[v] + 1;
    }
    return t;
}

}  // namespace

std::pair<std::vector<int>, std::vector<int>> graph_pair_fathers(const Graph &reduce, const Graph &bcast) {
    const int n = bcast.size();
    std::vector<int> rf(n), bf(n);
    for (int i = 0; i < n; ++i) {
        std::vector<int> nx;
        for (int j : reduce.nexts(i))
            if (j != i) nx.push_back(j);
        if (nx.size() > 1) throw std::invalid_argument("graph_pair_fathers: reduce graph is not an in-tree");
        rf[i] = nx.empty() ? i : nx[0];
        const auto &pv = bcast.prevs(i);
        if (pv.size() > 1) throw std::invalid_argument("graph_pair_fathers: bcast graph is not an out-tree");
        bf[i] = pv.empty() ? i : pv[0];
    }
    return {rf, bf};
}

GraphPlan plan_graph_all_reduce(const std::vector<std::pair<std::vector<int>, std::vector<int>>> &pairs, int rank,
                                int64_t count) {
    GraphPlan plan;
    const size_t k = pairs.size();
    if (k == 0 || count <= 0) return plan;
    const auto parts = even_partition(static_cast<size_t>(count), k);
    std::vector<TreeInfo> red(k), bc(k);
    int hmax = 0, dmax = 0;
    for (size_t c = 0; c < k; ++c) {
        if (pairs[c].first.size() != pairs[c].second.size())
            throw std::invalid_argument("graph plan: reduce/bcast sizes differ");
        if (rank < 0 || rank >= static_cast<int>(pairs[c].first.size()))
            throw std::invalid_argument("graph plan: rank out of range");
        red[c] = tree_info(pairs[c].first, true);
        bc[c] = tree_info(pairs[c].second, false);
        if (red[c].root != bc[c].root) throw std::invalid_argument("graph plan: reduce and bcast roots differ");
        hmax = std::max(hmax, red[c].level[red[c].root]);
        for (int v : bc[c].level) dmax = std::max(dmax, v);
    }
    // reduce rounds
    for (int r = 1; r <= hmax; ++r) {
        GraphRound round;
        int64_t scratch = 0;
        for (size_t c = 0; c < k; ++c) {
            const int64_t off = static_cast<int64_t>(parts[c].begin), len = static_cast<int64_t>(parts[c].len());
            if (len == 0) continue;
            const auto &t = red[c];
            if (rank != t.root && t.level[rank] == r - 1) {
                GraphXfer x;
                x.recv = false;
                x.peer = pairs[c].first[rank];
                x.off = off;
                x.len = len;
                round.ops.push_back(x);
            }
            for (int ch : t.children[rank]) {
                if (t.level[ch] != r - 1) continue;
                GraphXfer x;
                x.recv = true;
                x.peer = ch;
                x.off = off;
                x.len = len;
                x.scratch = scratch;
                scratch += len;
                round.ops.push_back(x);
            }
        }
        plan.scratch_elems = std::max(plan.scratch_elems, scratch);
        plan.rounds.push_back(std::move(round));
    }
    // bcast rounds
    for (int d = 1; d <= dmax; ++d) {
        GraphRound round;
        for (size_t c = 0; c < k; ++c) {
            const int64_t off = static_cast<int64_t>(parts[c].begin), len = static_cast<int64_t>(parts[c].len());
            if (len == 0) continue;
            const auto &t = bc[c];
            if (t.level[rank] == d && rank != t.root) {
                GraphXfer x;
                x.recv = true;
                x.peer = pairs[c].second[rank];
                x.off = off;
                x.len = len;
                round.ops.push_back(x);
            }
            if (t.level[rank] == d - 1) {
                for (int ch : t.children[rank]) {
                    GraphXfer x;
                    x.recv = false;
                    x.peer = ch;
                    x.off = off;
                    x.len = len;
                    round.ops.push_back(x);
                }
            }
        }
        plan.rounds.push_back(std::move(round));
    }
    return plan;
}

}  // namespace kungfu
