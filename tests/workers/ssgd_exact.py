"""Worker: S-SGD on the GPU engine with np ranks must reproduce ONE process training on
the concatenated global batch (the multi-rank test checked replica
equality only).  A BN-free net (so sharding the batch is exact), f32, mean loss: the
global-batch gradient is the average of the per-rank gradients.  Also pins the bf16-wire
gradient error against the f32 average (--comm-dtype bf16).

argv: [f32|bf16]"""
import os
import sys

import torch
import torch.nn.functional as F

import kungfu_amd as kf

comm_dtype = sys.argv[1] if len(sys.argv) > 1 else "f32"
device = sys.argv[2] if len(sys.argv) > 2 else "cuda"
hier = len(sys.argv) > 3 and sys.argv[3] == "hier"
os.environ["KUNGFU_TAIL_BUCKET_MB"] = "0.05"  # several buckets for this 0.5 MB model
kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
if device == "cuda":
    dev = torch.device("cuda", kf.get_hip_index())
    torch.cuda.set_device(dev)
else:
    dev = torch.device("cpu")
    torch.set_num_threads(2)
B, STEPS = 8, 4


def net():
    torch.manual_seed(7)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3, padding=1), torch.nn.ReLU(), torch.nn.Conv2d(16, 32, 3, 2, 1),
                               torch.nn.ReLU(), torch.nn.Flatten(), torch.nn.Linear(32 * 8 * 8, 64), torch.nn.Tanh(),
                               torch.nn.Linear(64, 10)).to(dev)


g = torch.Generator(device="cpu").manual_seed(11)
data = [(torch.randn(n * B, 3, 16, 16, generator=g), torch.randint(0, 10, (n * B,), generator=g)) for _ in range(STEPS)]

# reference: one process, global batch n*B
ref = net()
ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
ref_grads = []
for x, y in data:
    ropt.zero_grad()
    F.cross_entropy(ref(x.to(dev)), y.to(dev)).backward()
    ref_grads.append(torch.cat([p.grad.reshape(-1) for p in ref.parameters()]).clone())
    ropt.step()

# S-SGD: each rank its contiguous shard
m = net()
opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4),
                                            named_parameters=m.named_parameters(), bucket_mb=0.1,
                                            first_bucket_mb=0.05,
                                            comm_dtype=torch.bfloat16 if comm_dtype == "bf16" else None,
                                            flat=True, hierarchical=hier)
kf.broadcast_parameters(m.state_dict())
assert opt.reducer is not None and len(opt.reducer.buckets) >= 3, len(opt.reducer.buckets)
errs = []
for step, (x, y) in enumerate(data):
    xs, ys = x[r * B:(r + 1) * B].to(dev), y[r * B:(r + 1) * B].to(dev)
    opt.zero_grad()
    F.cross_entropy(m(xs), ys).backward()
    opt.reducer.synchronize()
    got = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    want = ref_grads[step]
    errs.append(((got.double() - want.double()).norm() / want.double().norm()).item())
    opt.step()
if device == "cuda":
    torch.cuda.synchronize()
w_got = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).double()
w_ref = torch.cat([p.detach().reshape(-1) for p in ref.parameters()]).double()
werr = ((w_got - w_ref).norm() / w_ref.norm()).item()
d = opt.reducer.describe()
assert d["comm_ranks"] == n, d
if comm_dtype == "f32":
    # same math, different summation order only
    assert max(errs) < 1e-5 and werr < 1e-5, (errs, werr)
else:
    # every rank rounds its shard gradient to bf16 and RCCL sums in bf16: relative error
    # of the averaged gradient is bounded by a few bf16 ulps (2^-8 = 3.9e-3)
    assert max(errs) < 8e-3 and werr < 8e-3, (errs, werr)
ck = kf.ops.all_gather(w_got.sum().reshape(1).cpu())
assert torch.all(ck == ck[0]), ck
assert d["hierarchical"] == hier, d
print("SSGD_EXACT_OK rank=%d np=%d plane=%s dtype=%s hier=%s grad_err=%.2e w_err=%.2e" % (
    r, n, d["comm_plane"], comm_dtype, hier, max(errs), werr), flush=True)
kf.finalize()
