"""Worker: PairAveragingOptimizer on GPU with the HIP-IPC device store."""
import torch

import kungfu_amd as kf

kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
dev = torch.device("cuda", kf.get_hip_index())
torch.cuda.set_device(dev)
torch.manual_seed(r)
m = torch.nn.Linear(64, 8).to(dev)
opt = kf.optimizers.PairAveragingOptimizer(torch.optim.SGD(m.parameters(), lr=0.0))
assert opt.store is not None and opt.store.local[1 - r]
w_before = m.weight.detach().clone()
for step in range(3):
    opt.zero_grad()
    m(torch.randn(4, 64, device=dev)).sum().backward()
    opt.step()
    torch.cuda.synchronize()
    kf.run_barrier()
# lr = 0: pair averaging alone must contract the two replicas towards each other
other = kf.ops.request_variable(1 - r, "kf:pair:rec" + "model", (2,), torch.int64)
assert other is not None and int(other[1]) >= 1
diff = (m.weight.detach() - w_before).abs().max().item()
assert diff > 0, "model did not move towards the peer"
print("PAIR_GPU_OK rank=%d moved=%.3e" % (r, diff), flush=True)
kf.finalize()
