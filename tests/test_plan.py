"""Pure-logic tests of the native planning layer (parity: srcs/go/plan/*_test.go)."""
import json

import pytest

from kungfu_amd._lib import runtime as K


def peers(spec):
    return ",".join(spec)


def test_strategy_names():
    names = K.strategy_names()
    for s in ["STAR", "MULTI_STAR", "RING", "CLIQUE", "TREE", "BINARY_TREE", "BINARY_TREE_STAR",
              "MULTI_BINARY_TREE_STAR", "AUTO"]:
        assert s in names


def _check_pair(reduce, bcast, n):
    # every node reaches the bcast root; reduce has self loops where needed
    rn, bn = reduce["nodes"], bcast["nodes"]
    assert len(rn) == len(bn) == n
    roots = [i for i, x in enumerate(bn) if not x["prevs"]]
    assert len(roots) == 1, bcast["debug"]
    for i, x in enumerate(bn):
        assert len(x["prevs"]) <= 1


@pytest.mark.parametrize("strategy", ["STAR", "MULTI_STAR", "RING", "CLIQUE", "TREE", "BINARY_TREE",
                                      "BINARY_TREE_STAR", "MULTI_BINARY_TREE_STAR", "AUTO"])
@pytest.mark.parametrize("hosts", [1, 2, 3])
@pytest.mark.parametrize("per_host", [1, 2, 4])
def test_strategy_graphs(strategy, hosts, per_host):
    pl = ",".join("10.0.0.%d:%d" % (h + 1, 10000 + i) for h in range(hosts) for i in range(per_host))
    n = hosts * per_host
    gs = K.gen_strategy_graphs(pl, strategy)
    assert len(gs) >= 1
    for r, b in gs:
        _check_pair(r, b, n)


def test_ring_graph_shape():
    pl = ",".join("127.0.0.1:%d" % (10000 + i) for i in range(4))
    gs = K.gen_strategy_graphs(pl, "RING")
    assert len(gs) == 4  # one per root
    r, b = gs[0]
    # reduce chain ends at root 0: 1->2->3->0 ; bcast chain 0->1->2->3
    assert r["debug"] == "[4]{(0)(1)(2)(3)(1->2)(2->3)(3->0)}"
    assert b["debug"] == "[4]{(0->1)(1->2)(2->3)}"


def test_binary_tree_star_two_hosts():
    pl = "10.0.0.1:10000,10.0.0.1:10001,10.0.0.2:10000,10.0.0.2:10001"
    (r, b), = K.gen_strategy_graphs(pl, "BINARY_TREE_STAR")
    assert b["debug"] == "[4]{(0->1)(0->2)(2->3)}"


def test_forest():
    g = K.graph_from_forest([0, 0, 1, 1])
    assert g["roots"] == 1
    assert g["nodes"][1]["prevs"] == [0]
    assert K.graph_from_forest([1, 0]) is None  # cycle
    assert K.graph_from_forest([0, 5]) is None  # out of range
    assert K.graph_from_forest([0, 1, 1])["roots"] == 2


def test_cluster_resize_validate():
    c = {"Runners": ["10.0.0.1:38080", "10.0.0.2:38080"],
         "Workers": ["10.0.0.1:10000", "10.0.0.1:10001", "10.0.0.2:10000"]}
    cj = json.dumps(c)
    assert K.cluster_validate(cj) == ""
    grown = json.loads(K.cluster_resize(cj, 5))
    assert grown["Workers"][:3] == c["Workers"]
    assert grown["Workers"][3] == "10.0.0.2:10001"  # least-loaded host first
    assert len(grown["Workers"]) == 5
    shrunk = json.loads(K.cluster_resize(cj, 1))
    assert shrunk["Workers"] == ["10.0.0.1:10000"]
    bad = json.dumps({"Runners": ["10.0.0.1:38080"], "Workers": ["10.0.0.3:10000"]})
    assert K.cluster_validate(bad) == "missing runner"
    dup = json.dumps({"Runners": ["10.0.0.1:38080"], "Workers": ["10.0.0.1:10000", "10.0.0.1:10000"]})
    assert K.cluster_validate(dup) == "duplicated port"


def test_host_list_and_hostfile():
    pl = K.gen_peer_list("192.168.1.1:2,192.168.1.2:2", 3, "10000-11000")
    assert pl == "192.168.1.1:10000,192.168.1.1:10001,192.168.1.2:10000"
    with pytest.raises(Exception):
        K.gen_peer_list("127.0.0.1:2", 3, "10000-11000")
    hl = K.parse_hostfile("# comment\n192.168.1.1 slots=4 public_addr=node1\n192.168.1.2\n")
    assert hl == "192.168.1.1:4:node1,192.168.1.2:1:192.168.1.2"


def test_partition_by_host():
    masters, master_of = K.partition_by_host("10.0.0.1:1,10.0.0.2:1,10.0.0.1:2,10.0.0.2:2")
    assert masters == [0, 1]
    assert master_of == [0, 1, 0, 1]


def test_even_partition():
    assert K.even_partition(10, 3) == [(0, 4), (4, 7), (7, 10)]
    assert K.even_partition(2, 4) == [(0, 1), (1, 2), (2, 2), (2, 2)]


def test_mst():
    w = [0, 1, 5, 1, 0, 2, 5, 2, 0]
    assert K.minimum_spanning_tree(w, 3, 0) == [0, 0, 1]


# ---- device graph all-reduce round schedule (plan_graph_all_reduce) -----------------

def _simulate(pairs, n, count, rng):
    """Run every rank's round schedule in lock step with matched send/recv per
    (sender, receiver) in issue order -- the semantics of a grouped RCCL send/recv."""
    import numpy as np

    bufs = [rng.integers(-1000, 1000, size=count).astype(np.int64) for _ in range(n)]
    want = sum(bufs)
    plans = [K.plan_graph_all_reduce(pairs, r, count) for r in range(n)]
    nrounds = {len(p[0]) for p in plans}
    assert len(nrounds) == 1, "every rank runs the same number of rounds"
    for ri in range(nrounds.pop()):
        sends, recvs = {}, {}
        for r in range(n):
            for (is_recv, peer, off, ln, scratch) in plans[r][0][ri]:
                if is_recv:
                    recvs.setdefault((peer, r), []).append((off, ln, scratch))
                else:
                    sends.setdefault((r, peer), []).append(bufs[r][off:off + ln].copy())
        assert sorted(sends) == sorted(recvs), ("unmatched ops in round", ri)
        scratch = [np.zeros(max(plans[r][1], 1), dtype=np.int64) for r in range(n)]
        pend = []
        for (src, dst), rl in recvs.items():
            sl = sends[(src, dst)]
            assert len(sl) == len(rl)
            for data, (off, ln, sc) in zip(sl, rl):
                assert len(data) == ln
                if sc >= 0:
                    assert sc + ln <= plans[dst][1]
                    scratch[dst][sc:sc + ln] = data
                    pend.append((dst, off, ln, sc))
                else:
                    bufs[dst][off:off + ln] = data
        for dst, off, ln, sc in pend:  # reduce kernels after the group
            bufs[dst][off:off + ln] += scratch[dst][sc:sc + ln]
    for r in range(n):
        assert (bufs[r] == want).all(), ("rank", r)


@pytest.mark.parametrize("strategy", ["STAR", "MULTI_STAR", "RING", "CLIQUE", "TREE", "BINARY_TREE",
                                      "BINARY_TREE_STAR", "MULTI_BINARY_TREE_STAR", "AUTO"])
@pytest.mark.parametrize("hosts", [[1], [2], [3], [8], [4, 4], [2, 3, 1]])
def test_graph_round_plan_all_strategies(strategy, hosts):
    import numpy as np

    spec = []
    for h, k in enumerate(hosts):
        spec += ["10.0.0.%d:%d" % (h + 1, 10000 + i) for i in range(k)]
    n = len(spec)
    pairs = K.strategy_pairs(",".join(spec), strategy)
    assert pairs
    rng = np.random.default_rng(n)
    for count in (1, 7, n * 5 + 3, 1000):
        _simulate(pairs, n, count, rng)


def test_graph_round_plan_shapes():
    import numpy as np

    n = 8
    # CLIQUE on one host = link-parallel reduce-scatter + all-gather: 2 rounds, each rank
    # talks to all 7 peers per round
    pairs = K.strategy_pairs(",".join("127.0.0.1:%d" % (10000 + i) for i in range(n)), "CLIQUE")
    rounds, scratch = K.plan_graph_all_reduce(pairs, 0, 800)
    assert len(rounds) == 2 and scratch == 7 * 100
    assert {op[1] for op in rounds[0]} == set(range(1, n))
    # RING: 2 (n - 1) rounds with one send per round
    pairs = K.strategy_pairs(",".join("127.0.0.1:%d" % (10000 + i) for i in range(n)), "RING")
    rounds, _ = K.plan_graph_all_reduce(pairs, 3, 800)
    assert len(rounds) == 2 * (n - 1)
    assert all(sum(1 for op in r if op[0] == 0) == 1 for r in rounds)
    # random set_tree forests (reduce along the tree, bcast down the same tree)
    rng = np.random.default_rng(0)
    for _ in range(20):
        m = int(rng.integers(1, 9))
        root = int(rng.integers(0, m))
        order = [root] + [i for i in rng.permutation(m).tolist() if i != root]
        f = [0] * m
        f[root] = root
        for j in range(1, m):
            f[order[j]] = order[int(rng.integers(0, j))]
        _simulate([(f, f)], m, 37, rng)
    with pytest.raises(Exception):
        K.plan_graph_all_reduce([([1, 0], [1, 0])], 0, 10)  # cycle


def test_host_list_resolves_hostnames():
    """-H entries may be host / DNS names (parity: runner/discovery.go); the public
    address keeps the name, the worker list gets the resolved IPv4."""
    pl = K.gen_peer_list("localhost:2", 2, "10000-11000")
    assert pl == "127.0.0.1:10000,127.0.0.1:10001"
    with pytest.raises(Exception):
        K.gen_peer_list("no-such-host.invalid:2", 2, "10000-11000")


def test_kungfu_run_with_hostname_host_list(tmp_path):
    import os
    import subprocess
    import sys

    from conftest import ROOT, free_port_block

    s = tmp_path / "w.py"
    s.write_text("import os; print('HOSTNAME_OK', os.environ['KUNGFU_SELF_SPEC'])\n")
    base = free_port_block(6)
    r = subprocess.run([os.path.join(ROOT, "bin", "kungfu-run"), "-q", "-np", "2", "-H", "localhost:2",
                        "-port-range", "%d-%d" % (base + 1, base + 5), "-port", str(base), sys.executable, str(s)],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=60)
    assert r.returncode == 0, r.stdout
    assert r.stdout.count("HOSTNAME_OK 127.0.0.1:") == 2
