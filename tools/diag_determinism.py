"""Diagnostic: run-to-run determinism of the fused ResNet forward/backward (same weights, same input)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kungfu_amd as kf  # noqa: E402
from kungfu_amd._lib import hip  # noqa: E402
from kungfu_amd.models import resnet18  # noqa: E402

kf.init()
H = hip()
torch.manual_seed(0)
x = torch.randn(8, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).bfloat16().contiguous(memory_format=torch.channels_last)
x4 = H.stem_pad4(x)
wp = H.stem_pack_weight(w)
ys = [H.stem_forward(x4, wp, None) for _ in range(3)]
print("stem fwd bitwise equal:", all(torch.equal(ys[0], t) for t in ys[1:]))
dy = torch.randn_like(ys[0])
dws = [H.stem_wgrad(dy, x4) for _ in range(3)]
print("stem wgrad bitwise equal:", all(torch.equal(dws[0], t) for t in dws[1:]))

m = resnet18(fused_bn=True).cuda().to(memory_format=torch.channels_last)
m.eval()  # no running-stat updates between the runs
outs = {}


def hook(name):
    def f(mod, inp, out):
        outs.setdefault(name, []).append(out.detach().float().clone())
    return f


for n, mod in m.named_modules():
    if n and "." not in n:
        mod.register_forward_hook(hook(n))
m.train()
for _ in range(2):
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        m(x)
for n, v in outs.items():
    d = ((v[0] - v[1]).norm() / (v[0].norm() + 1e-30)).item()
    print("%-10s rel diff %.3e" % (n, d))
