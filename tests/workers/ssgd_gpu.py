"""Worker: the S-SGD engine (bucketed reducer, ordered scheduler, bf16 shadow weights,
fused BN) with np ranks; every replica must stay bit-identical.  With
KUNGFU_GPU_DATAPLANE=host several ranks can share one GPU (RCCL refuses that)."""
import torch
import torch.nn.functional as F

import kungfu_amd as kf
from kungfu_amd.models import resnet18
from kungfu_amd.parallel.mixed import enable_bf16_shadow

kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
dev = torch.device("cuda", kf.get_hip_index())
torch.cuda.set_device(dev)
torch.manual_seed(100 + r)  # different init per rank: broadcast must fix it
m = resnet18(fused_bn=True, num_classes=10).to(dev).to(memory_format=torch.channels_last)
opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9),
                                            named_parameters=m.named_parameters(), bucket_mb=2.0)
kf.broadcast_parameters(m.state_dict())
enable_bf16_shadow(m, opt)
assert opt.reducer is not None and len(opt.reducer.buckets) > 2
torch.manual_seed(r)  # different data per rank
for step in range(4):
    x = torch.randn(4, 3, 32, 32, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), device=dev)
    opt.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    opt.step()
torch.cuda.synchronize()
assert opt.reducer._ordered, "auto-order did not run"
w = opt.space.flat_param.double().sum().reshape(1)
ws = kf.ops.all_gather(w.cpu())
assert torch.all(ws == ws[0]), ws
print("SSGD_GPU_OK rank=%d np=%d order=%s" % (r, n, opt.reducer.tracker.order()), flush=True)
kf.finalize()
