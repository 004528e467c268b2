"""Multi-process host collectives through kungfu-run for np=1..4 x every
strategy (parity: scripts/tests/run-integration-tests.sh:10-38)."""
import pytest

from conftest import kungfu_run, worker

STRATEGIES = ["STAR", "MULTI_STAR", "RING", "CLIQUE", "TREE", "BINARY_TREE", "BINARY_TREE_STAR",
              "MULTI_BINARY_TREE_STAR", "AUTO"]


@pytest.mark.parametrize("np_", [1, 2, 3, 4])
@pytest.mark.parametrize("strategy", STRATEGIES)
def test_collectives(np_, strategy):
    if np_ == 3 and strategy not in ("RING", "CLIQUE", "BINARY_TREE_STAR"):
        pytest.skip("np=3 covered for a subset")
    r = kungfu_run(np_, [worker("collectives.py")], strategy=strategy, timeout=180)
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count("COLLECTIVES_OK") == np_, r.stdout[-4000:]


@pytest.mark.parametrize("np_", [2, 3])
def test_model_averaging_ops(np_):
    r = kungfu_run(np_, [worker("model_avg.py")], timeout=180)
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count("MODEL_AVG_OK") == np_, r.stdout[-4000:]


def test_p2p_send_recv_and_device_stats():
    r = kungfu_run(2, [worker("p2p_stats.py")], timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    assert r.stdout.count("P2P_STATS_OK") == 2


def test_all_gather_transform_mst():
    r = kungfu_run(3, [worker("agt.py")], timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    assert r.stdout.count("AGT_OK") == 3
    assert r.stdout.count("AGT_ERR_OK") == 3, r.stdout[-3000:]


def test_monitored_ssgd_adapts_strategy_on_interference():
    """bucket-engine S-SGD with monitor/adapt: strategy statistics accrue,
    an injected slowdown flips the strategy on every peer at the same step."""
    r = kungfu_run(2, [worker("adapt_ssgd.py"), "cpu"], timeout=180)
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count("ADAPT_OK") == 2, r.stdout[-4000:]
