"""Worker: exercises every host collective on CPU tensors (run under kungfu-run).

Parity: tests/cpp/integration/fake_agent.cpp (y[i] = i*np all-reduce check),
tests/go/cmd/kungfu-test-public-apis (SUM/MAX on i32/u8, AllGather, P2P),
tests/python/integration/test_operators.py.
"""
import sys

import torch

import kungfu_amd as kf
from kungfu_amd import ops

kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()

# all-reduce: sum/min/max/prod over several dtypes and sizes (incl. > 1 MiB chunks)
for count in [1, 10, 1000, 300_000, (1 << 19) + 3]:
    x = torch.arange(count, dtype=torch.float32)
    y = ops.all_reduce(x, "sum")
    assert torch.equal(y, x * n), ("sum", count)
for dt in [torch.int32, torch.int64, torch.uint8, torch.float64, torch.bfloat16, torch.float16]:
    x = torch.full((17,), r + 1).to(dt)
    assert torch.equal(ops.all_reduce(x, "max"), torch.full((17,), n).to(dt)), dt
    assert torch.equal(ops.all_reduce(x, "min"), torch.full((17,), 1).to(dt)), dt
x = torch.full((5,), 2.0)
assert torch.equal(ops.all_reduce(x, "prod"), torch.full((5,), 2.0 ** n))
assert torch.allclose(ops.all_reduce(torch.full((3,), float(r)), "avg"), torch.full((3,), (n - 1) / 2))

# async + group (None entries skipped)
ts = [torch.ones(100) * r, None, torch.ones(7, dtype=torch.int32)]
ops.group_all_reduce_(ts, op="sum")
assert torch.equal(ts[0], torch.ones(100) * (n * (n - 1) // 2)) and torch.equal(ts[2], torch.full((7,), n, dtype=torch.int32))
hs = [ops.inplace_all_reduce_async_op(t, name="async%d" % i) for i, t in enumerate([torch.ones(10), torch.ones(20)])]
ops.wait_all_handles(hs)

# broadcast / all_gather / gather / reduce
b = torch.full((9,), float(r))
assert torch.equal(ops.broadcast(b), torch.zeros(9))
g = ops.all_gather(torch.full((2, 3), r, dtype=torch.int64))
assert g.shape == (n, 2, 3) and all(torch.equal(g[i], torch.full((2, 3), i, dtype=torch.int64)) for i in range(n))
ga = ops.gather(torch.tensor([float(r)]))
if r == 0:
    assert torch.equal(ga.reshape(-1), torch.arange(n, dtype=torch.float32))
red = ops.reduce(torch.tensor([1.0]))
if r == 0:
    assert red.item() == n

# barrier / consensus
kf.run_barrier()
assert ops.consensus(b"same")
assert ops.consensus(torch.tensor([r])) == (n == 1)

# monitored all-reduce with an explicit tree (star at 0) and stats
t = torch.ones(1000)
ops.monitored_all_reduce_(t, tree=[0] * n)
assert torch.equal(t, torch.full((1000,), float(n)))

# local / cross / hierarchical (single host: cross is among one master)
h = torch.ones(10) * (r + 1)
ops.hierarchical_all_reduce_(h)
assert torch.equal(h, torch.full((10,), n * (n + 1) / 2))

# p2p store: versioned and unversioned
ops.save_variable(torch.full((4,), float(r)), name="w")
ops.save_variable(torch.full((4,), float(10 + r)), name="w", version=1)
kf.run_barrier()
peer = (r + 1) % n
got = ops.request_variable(peer, "w", (4,), torch.float32)
assert torch.equal(got, torch.full((4,), float(peer))), got
got = ops.request_variable(peer, "w", (4,), torch.float32, version=1)
assert torch.equal(got, torch.full((4,), float(10 + peer)))
assert ops.request_variable(peer, "missing", (4,), torch.float32) is None
assert ops.request_variable(peer, "w", (4,), torch.float32, version=7) is None
kf.run_barrier()

# set_tree: chain 0 <- 1 <- 2 ... then all-reduce still correct
if n > 1:
    assert ops.set_tree([max(i - 1, 0) for i in range(n)])
    x = torch.arange(5000, dtype=torch.float32)
    assert torch.equal(ops.all_reduce(x), x * n)

# broadcast_parameters of a state dict
sd = {"a": torch.full((3,), float(r)), "b": torch.full((2, 2), r, dtype=torch.int32)}
ops.broadcast_parameters(sd)
assert torch.equal(sd["a"], torch.zeros(3)) and torch.equal(sd["b"], torch.zeros(2, 2, dtype=torch.int32))

# native ordered scheduler: ranks observe different completion orders, auto_order
# makes every rank adopt rank 0's (the reference NCCLScheduler's auto-order)
sched = kf._lib.runtime.OrderedScheduler(4)
arr = [3, 1, 0, 2] if r == 0 else [0, 1, 2, 3]
launched = []
for i in arr:
    launched += sched.ready(i)
assert launched == [0, 1, 2, 3] and sched.arrivals() == arr
sched.auto_order()
assert sched.order() == [3, 1, 0, 2], sched.order()
sched.reset()
assert sched.ready(0) == [] and sched.ready(3) == [3] and sched.ready(1) == [1, 0] and sched.flush() == [2]

lat = ops.get_peer_latencies()
assert lat.shape == (n,) and (lat[torch.arange(n) != r] >= 0).all()
print("COLLECTIVES_OK rank=%d np=%d strategy=%s" % (r, n, kf._lib.runtime.strategy()), flush=True)
kf.finalize()
