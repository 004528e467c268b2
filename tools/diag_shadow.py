"""Diagnostic: per-parameter first-step gradient differences, shadow vs stock autocast (ResNet-18)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kungfu_amd as kf  # noqa: E402
from kungfu_amd.models import resnet18  # noqa: E402
from kungfu_amd.ops import conv as conv_ops  # noqa: E402
from kungfu_amd.parallel.mixed import enable_bf16_shadow  # noqa: E402

kf.init()
x = torch.randn(8, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (8,), device="cuda")


def run(shadow):
    torch.manual_seed(0)
    m = resnet18(fused_bn=True).cuda().to(memory_format=torch.channels_last)
    o = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9))
    if shadow:
        enable_bf16_shadow(m, o)
    o.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    o.reducer.synchronize() if getattr(o, "reducer", None) is not None else None
    return loss.item(), o.space.flat_grad.clone(), [(n, o.space.grad_view(i).clone()) for i, n in enumerate(o.space.names)]


conv_ops.set_enabled(False)
la, ga, pa = run(False)
lb, gb, pb = run(False)
ls, gs, ps = run(True)
print("loss", la, lb, ls)
fro = lambda a, b: ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()
print("flat a-b %.4f s-a %.4f" % (fro(gb, ga), fro(gs, ga)))
for (n, a), (_, b), (_, s) in zip(pa, pb, ps):
    print("%-40s a-b %.4f s-a %.4f |a| %.3e" % (n, fro(b, a), fro(s, a), a.norm().item()))
