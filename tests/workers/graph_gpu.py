"""Worker: device graph all-reduce (KungFu strategy graphs as round plans + the K1 reduce
kernel) for every strategy and a set_tree forest, plus the bucketed S-SGD reducer in graph
mode, plus device strategy statistics (monitored all-reduce -> calc_stats ->
check_interference).  The transfers are grouped RCCL send/recv rounds, or -- with
KUNGFU_GPU_DATAPLANE=host, for ranks sharing one GPU -- the same rounds over the host
transport.  When RCCL refuses ranks that share a GPU, prints GRAPH_GPU_SKIP."""
import os

import torch

import kungfu_amd as kf
from kungfu_amd._lib import runtime

kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
dev = torch.device("cuda", kf.get_hip_index())
torch.cuda.set_device(dev)
from kungfu_amd.parallel.comm import get_device_comm  # noqa: E402

try:
    comm = get_device_comm()
    t = torch.ones(4, device=dev)
    comm.all_reduce(t, op="sum", stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert float(t[0]) == n
except Exception as e:  # noqa: BLE001
    print("GRAPH_GPU_SKIP rank=%d: %s" % (r, str(e)[:200]), flush=True)
    kf.finalize()
    raise SystemExit(0)
peers = runtime.peers()
for strategy in runtime.strategy_names():
    pairs = runtime.strategy_pairs(peers, strategy)
    for dt in (torch.float32, torch.bfloat16):
        for count in (1, 1000, (1 << 20) + 5):
            x = torch.full((count,), float(r + 1), dtype=dt, device=dev)
            comm.graph_all_reduce(x, op="sum", pairs=pairs, stream=torch.cuda.current_stream())
            torch.cuda.synchronize()
            want = n * (n + 1) / 2
            assert torch.all(x.float() == want), (strategy, dt, count, x[:4])
# set_tree-style forest: chain rooted at the last rank
f = [min(i + 1, n - 1) for i in range(n)]
x = torch.arange(10, dtype=torch.float32, device=dev) * (r + 1)
kf.ops.all_reduce_with(x, f)
# S-SGD buckets through the graph plane
os.environ["KUNGFU_GPU_ALLREDUCE"] = "graph"
m = torch.nn.Linear(256, 256).to(dev)
opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), bucket_mb=0.1)
assert opt.reducer.graph
kf.broadcast_parameters(m.state_dict())
for step in range(3):
    opt.zero_grad()
    m(torch.randn(8, 256, device=dev) * (r + 1)).pow(2).mean().backward()
    opt.step()
torch.cuda.synchronize()
w = opt.space.flat_param.double().sum().reshape(1)
ws = kf.ops.all_gather(w.cpu())
assert torch.all(ws == ws[0]), ws
# device strategy statistics: one active strategy (a tree), monitored device all-reduces
assert kf.ops.set_tree([0] * n)
for _ in range(4):
    x = torch.ones(1 << 18, device=dev)
    kf.ops.monitored_all_reduce_(x)
    assert float(x[0]) == n
kf.ops.calc_stats()
tp = runtime.strategy_throughputs()
assert len(tp) == 1 and tp[0] > 0, tp
assert kf.ops.check_interference() is False  # first call sets the reference window
print("GRAPH_GPU_OK rank=%d np=%d throughput=%.1fMiB/s" % (r, n, tp[0] / (1 << 20)), flush=True)
kf.finalize()
