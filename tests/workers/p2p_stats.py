"""Worker: named point-to-point transfers and device-plane strategy statistics on the host
runtime (np = 2)."""
import torch

import kungfu_amd as kf
from kungfu_amd._lib import runtime

kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
buf = torch.arange(1000, dtype=torch.float32) * (r + 1)
if r == 0:
    runtime.send_to(1, "p2p:x", buf.data_ptr(), buf.numel() * 4)
    got = torch.empty(1000)
    runtime.recv_from(1, "p2p:y", got.data_ptr(), got.numel() * 4)
    assert torch.equal(got, torch.arange(1000, dtype=torch.float32) * 2)
else:
    got = torch.empty(1000)
    runtime.recv_from(0, "p2p:x", got.data_ptr(), got.numel() * 4)
    assert torch.equal(got, torch.arange(1000, dtype=torch.float32))
    runtime.send_to(0, "p2p:y", buf.data_ptr(), buf.numel() * 4)
assert kf.ops.set_tree([0] * n)
runtime.record_strategy_stat(10.0, 10.5, 1 << 20)
runtime.record_strategy_stat(10.5, 11.0, 1 << 20)
kf.ops.calc_stats()
tp = runtime.strategy_throughputs()
assert abs(tp[0] - 2 * (1 << 20)) < 1e-6, tp
print("P2P_STATS_OK rank=%d" % r, flush=True)
