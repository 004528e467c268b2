"""Worker: PairAveragingOptimizer on GPU with the HIP-IPC device store (2 peers, one GPU).

lr = 0: after the first step each replica must hold EXACTLY 0.5 * (own + peer's initial
model) -- the one-sided pull reads a complete snapshot and the K4 kernel averages it."""
import torch

import kungfu_amd as kf


def make(seed, dev):
    torch.manual_seed(seed)
    return torch.nn.Linear(64, 8).to(dev)


kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
dev = torch.device("cuda", kf.get_hip_index())
torch.cuda.set_device(dev)
m = make(r, dev)
peer0 = make(1 - r, dev)
own0 = [p.detach().clone() for p in m.parameters()]
opt = kf.optimizers.PairAveragingOptimizer(torch.optim.SGD(m.parameters(), lr=0.0))
assert opt.store is not None and opt.store.local[1 - r]
for step in range(3):
    opt.zero_grad()
    m(torch.randn(4, 64, device=dev)).sum().backward()
    opt.step()
    torch.cuda.synchronize()
    if step == 0:
        assert opt.store.last_pulled == (1 - r, 1), opt.store.last_pulled
        for p, a, b in zip(m.parameters(), own0, peer0.parameters()):
            want = 0.5 * a + 0.5 * b.detach()
            assert torch.equal(p.detach(), want), (p - want).abs().max()
    kf.run_barrier()
other = kf.ops.request_variable(1 - r, "kf:pair:rec" + "model", (2,), torch.int64)
assert other is not None and int(other[1]) >= 1
print("PAIR_GPU_OK rank=%d dropped=%d" % (r, opt.store.dropped), flush=True)
kf.finalize()
