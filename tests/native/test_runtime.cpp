// Native tests of the host runtime (no GPU): base kernels, planning, and an
// IN-PROCESS fake cluster (parity: tests/cpp/unit/*.cpp and
// tests/cpp/integration/fake_in_proc_trainer.cpp) -- N peers as threads on
// loopback ports running every collective and P2P concurrently.  Built also
// with -fsanitize=thread and -fsanitize=address,undefined (make native-test-tsan / -asan).
#include <kungfu/base.hpp>
#include <kungfu/peer.hpp>
#include <kungfu/plan.hpp>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

using namespace kungfu;

static std::atomic<int> g_fail{0};
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                         \
        }                                                                     \
    } while (0)

static void test_base() {
    CHECK(dtype_size(DType::BF16) == 2 && dtype_size(DType::F64) == 8 && dtype_size(DType::BOOL) == 1);
    std::vector<float> x(37), y(37), z(37);
    for (int i = 0; i < 37; ++i) x[i] = i, y[i] = 2 * i;
    transform2(z.data(), x.data(), y.data(), 37, DType::F32, ReduceOp::SUM);
    for (int i = 0; i < 37; ++i) CHECK(z[i] == 3 * i);
    std::vector<uint16_t> a(19), b(19), c(19);
    for (int i = 0; i < 19; ++i) a[i] = f32_to_bf16(i * 0.5f), b[i] = f32_to_bf16(1.0f);
    transform2(c.data(), a.data(), b.data(), 19, DType::BF16, ReduceOp::SUM);
    for (int i = 0; i < 19; ++i) CHECK(bf16_to_f32(c[i]) == i * 0.5f + 1.0f);
    for (int i = 0; i < 19; ++i) a[i] = f32_to_f16(i * 0.25f);
    transform2(c.data(), a.data(), a.data(), 19, DType::F16, ReduceOp::MAX);
    for (int i = 0; i < 19; ++i) CHECK(f16_to_f32(c[i]) == i * 0.25f);
    auto parts = even_partition(10, 3);
    CHECK(parts.size() == 3 && parts[0].len() == 4 && parts[2].end == 10);
}

static void test_plan() {
    auto pl = PeerList::parse("10.0.0.1:1,10.0.0.1:2,10.0.0.2:1");
    CHECK(pl.rank(PeerID::parse("10.0.0.2:1")) == 2 && pl.local_rank(PeerID::parse("10.0.0.1:2")) == 1);
    CHECK(pl.host_count() == 2 && pl.local_size(PeerID::parse("10.0.0.1:1")) == 2);
    Graph g;
    int roots = 0;
    CHECK(Graph::from_forest({0, 0, 1}, &g, &roots) && roots == 1);
    CHECK(!Graph::from_forest({1, 0}, &g, &roots));
    std::vector<double> w = {0, 1, 5, 1, 0, 2, 5, 2, 0};
    auto f = minimum_spanning_tree(w, 3, 0);
    CHECK(f[1] == 0 && f[2] == 1);
    Cluster c;
    c.runners = PeerList::parse("10.0.0.1:38080,10.0.0.2:38080");
    c.workers = PeerList::parse("10.0.0.1:10000");
    auto d = c.resize(3);
    CHECK(d.workers.size() == 3 && d.validate().empty());
    CHECK(Cluster::from_json(json::parse(json::dump(d.to_json()))) == d);
}

static void peer_main(int rank, int np, int base, Strategy s) {
    PeerConfig cfg;
    for (int i = 0; i < np; ++i) cfg.init_peers.push_back(PeerID::parse("127.0.0.1:" + std::to_string(base + i)));
    cfg.self = cfg.init_peers[rank];
    cfg.strategy = s;
    cfg.single = false;
    Peer peer(cfg);
    peer.start();
    auto sess = peer.session();
    CHECK(sess->rank() == rank && sess->size() == np);
    for (size_t n : {size_t(1), size_t(1000), size_t(600000)}) {
        std::vector<float> x(n), y(n);
        for (size_t i = 0; i < n; ++i) x[i] = float(i % 1000) * (rank + 1);
        sess->all_reduce({x.data(), y.data(), n, DType::F32, ReduceOp::SUM, "ar" + std::to_string(n)});
        for (size_t i = 0; i < n; i += 997) CHECK(y[i] == float(i % 1000) * (np * (np + 1) / 2));
    }
    // concurrent collectives from several threads
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; ++t)
        ts.emplace_back([&, t] {
            std::vector<int32_t> v(5000, rank), o(5000);
            sess->all_reduce({v.data(), o.data(), v.size(), DType::I32, ReduceOp::MAX, "conc" + std::to_string(t)});
            CHECK(o[4999] == np - 1);
        });
    for (auto &t : ts) t.join();
    std::vector<int64_t> g(np * 3);
    std::vector<int64_t> me(3, rank);
    sess->all_gather({me.data(), g.data(), 3, DType::I64, ReduceOp::SUM, "ag"});
    for (int r = 0; r < np; ++r) CHECK(g[r * 3 + 2] == r);
    std::vector<double> bc(4, rank);
    sess->broadcast({bc.data(), bc.data(), 4, DType::F64, ReduceOp::SUM, "bc"});
    CHECK(bc[3] == 0);
    CHECK(sess->bytes_consensus("same", 4, "c1"));
    sess->barrier();
    std::vector<float> blob(100, float(rank));
    peer.save("w", blob.data(), blob.size() * 4);
    sess->barrier();
    std::vector<float> got(100);
    CHECK(peer.request((rank + 1) % np, "", "w", got.data(), got.size() * 4));
    CHECK(got[99] == float((rank + 1) % np));
    CHECK(!peer.request((rank + 1) % np, "", "missing", got.data(), got.size() * 4));
    sess->barrier();
    peer.close();
}

static void test_cluster(int np, Strategy s, int base) {
    std::vector<std::thread> ts;
    for (int r = 0; r < np; ++r) ts.emplace_back(peer_main, r, np, base, s);
    for (auto &t : ts) t.join();
}

int main(int argc, char **argv) {
    int base = argc > 1 ? std::atoi(argv[1]) : 41000;
    test_base();
    test_plan();
    int off = 0;
    for (int np : {1, 2, 4})
        for (auto s : {Strategy::STAR, Strategy::RING, Strategy::CLIQUE, Strategy::BINARY_TREE_STAR}) {
            test_cluster(np, s, base + off);
            off += 8;
        }
    if (g_fail) {
        std::fprintf(stderr, "NATIVE_TESTS_FAILED %d\n", g_fail.load());
        return 1;
    }
    std::printf("NATIVE_TESTS_OK\n");
    return 0;
}
