"""Worker: native AllGatherTransform and the MST-from-latency-rows flow (np = 3)."""
import torch

import kungfu_amd as kf
from kungfu_amd.ops.topology import all_gather_transform, global_minimum_spanning_tree

kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
calls = []


def total(g):
    calls.append(1)
    return g.sum(dim=0)


out = all_gather_transform(torch.arange(4, dtype=torch.float32) + 10 * r, torch.zeros(4), total)
assert torch.equal(out, torch.arange(4, dtype=torch.float32) * n + 10 * sum(range(n))), out
assert len(calls) == (1 if r == 0 else 0)  # the transform runs on the root only
# latency rows: a chain 0-1-2-... is the cheapest spanning tree
w = torch.tensor([abs(r - j) * 1.0 + (0 if abs(r - j) == 1 else 5.0) for j in range(n)])
edges = global_minimum_spanning_tree(w)
assert sorted(tuple(sorted(e)) for e in edges.tolist()) == [(i, i + 1) for i in range(n - 1)], edges
print("AGT_OK rank=%d" % r, flush=True)

# a transform that raises on the root must not leave the other peers blocked in the
# broadcast: every peer raises (session.cpp all_gather_transform)


def boom(g):
    raise ValueError("transform exploded")


try:
    all_gather_transform(torch.ones(3), torch.zeros(3), boom, name="agt-boom")
    raise AssertionError("all_gather_transform did not raise")
except AssertionError:
    raise
except Exception as e:  # noqa: BLE001
    assert r != 0 or "exploded" in str(e), e
# the session is still usable afterwards
assert torch.equal(kf.ops.all_reduce(torch.ones(2)), torch.full((2,), float(n)))
print("AGT_ERR_OK rank=%d" % r, flush=True)
