"""Diagnostic: backward determinism on one model (same weights, same input, BN in eval-free
training mode with momentum 0 so running stats do not matter)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import kungfu_amd as kf  # noqa: E402
from kungfu_amd.models import resnet18  # noqa: E402
from kungfu_amd.ops import conv as conv_ops  # noqa: E402

kf.init()
torch.manual_seed(0)
x = torch.randn(8, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (8,), device="cuda")
conv_ops.set_enabled(os.environ.get("CONV", "1") == "1")
m = resnet18(fused_bn=True).cuda().to(memory_format=torch.channels_last)
gs = []
for _ in range(3):
    m.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    gs.append([p.grad.detach().float().clone() for p in m.parameters()])
fro = lambda a, b: ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()
names = [n for n, _ in m.named_parameters()]
worst = sorted(((fro(a, b), n) for n, a, b in zip(names, gs[1], gs[0])), reverse=True)[:8]
print("conv=%s worst run-to-run param grad diffs:" % os.environ.get("CONV", "1"), ["%s %.2e" % (n, d) for d, n in worst])
