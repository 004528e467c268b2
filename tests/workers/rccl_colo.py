"""Worker: a REAL multi-rank RCCL communicator on one GPU (KUNGFU_RCCL_COLOCATE=1 gives
every rank its own RCCL host identity, so the ranks talk over RCCL's socket transport):
every collective the engine uses, with value checks, plus the watchdog bookkeeping."""
import torch

import kungfu_amd as kf
from kungfu_amd._lib import hip
from kungfu_amd.parallel.comm import get_device_comm

kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
dev = torch.device("cuda", kf.get_hip_index())
torch.cuda.set_device(dev)
comm = get_device_comm()
assert comm.plane == "rccl" and comm.size == n and comm.rank == r, (comm.plane, comm.size)
assert not comm.comm.blocking()  # non-blocking init + polled deadline
s = torch.cuda.current_stream()
for dt in (torch.float32, torch.bfloat16, torch.int32):
    for count in (1, 1000, (1 << 20) + 5):
        x = torch.full((count,), r + 1, dtype=dt, device=dev)
        comm.all_reduce(x, op="sum", stream=s, tag="colo-sum")
        torch.cuda.synchronize()
        assert torch.all(x == n * (n + 1) // 2), (dt, count, x[:4])
# ncclAvg (what the S-SGD buckets use with > 1 rank)
x = torch.full((4097,), float(2 * r), device=dev)
comm.all_reduce(x, op="avg", stream=s)
y = torch.full((4097,), float(r), device=dev)
comm.all_reduce(y, op="max", stream=s)
# broadcast from a non-zero root
b = torch.full((333,), float(r), device=dev)
comm.broadcast(b, root=n - 1, stream=s)
# all-gather / reduce-scatter
g = torch.empty(n * 5, device=dev)
comm.all_gather(torch.full((5,), float(r), device=dev), g, stream=s)
rs_in = torch.arange(n * 7, dtype=torch.float32, device=dev)
rs_out = torch.empty(7, device=dev)
comm.reduce_scatter(rs_in, rs_out, op="sum", stream=s)
torch.cuda.synchronize()
assert torch.allclose(x, torch.full_like(x, float(n - 1))), x[:4]
assert torch.all(y == n - 1)
assert torch.all(b == n - 1)
assert torch.equal(g.view(n, 5)[:, 0].cpu(), torch.arange(n, dtype=torch.float32))
assert torch.equal(rs_out.cpu(), (torch.arange(7) + 7 * r).float() * n)
# the collectives were registered with the watchdog and have all completed
info = hip().rccl_watchdog_info()
assert info["registered"] >= 10 and info["pending"] == 0, info
# group + public ops surface
ts = [torch.full((17,), float(r + i), device=dev) for i in range(3)]
from kungfu_amd.ops.collective import group_all_reduce_  # noqa: E402

group_all_reduce_(ts, op="sum")
torch.cuda.synchronize()
for i, t in enumerate(ts):
    assert torch.all(t == n * (n - 1) / 2 + n * i), (i, t[:3])
print("RCCL_COLO_OK rank=%d np=%d watched=%d" % (r, n, info["registered"]), flush=True)
kf.finalize()
