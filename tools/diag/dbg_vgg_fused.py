"""Per-parameter gradient agreement of the fused VGG stack vs the layered modules (debug aid)."""
import sys

import torch

sys.path.insert(0, ".")
from kungfu_amd.models.vgg import vgg16  # noqa: E402
from kungfu_amd.ops.vgg_fused import FusedVGGFeatures  # noqa: E402

torch.manual_seed(33)
m = vgg16(fused_bn=True).cuda().to(memory_format=torch.channels_last).eval()
x = torch.randn(4, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
tgt = torch.randint(0, 1000, (4,), device="cuda")


def run(fused, amp=True):
    m.zero_grad(set_to_none=True)
    orig = FusedVGGFeatures.forward
    if not fused:
        FusedVGGFeatures.forward = torch.nn.Sequential.forward
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = m(x)
            loss = torch.nn.functional.cross_entropy(out.float(), tgt)
        loss.backward()
    finally:
        FusedVGGFeatures.forward = orig
    return out.float().detach(), {k: p.grad.detach().float().clone() for k, p in m.named_parameters()}


o1, g1 = run(True)
o0, g0 = run(False)
of, gf = run(False, amp=False)  # f32 reference
print("logits vs f32: fused %.4f layered %.4f" % (((o1 - of).norm() / of.norm()).item(), ((o0 - of).norm() / of.norm()).item()))
for k in g0:
    e1 = ((g1[k] - gf[k]).norm() / (gf[k].norm() + 1e-12)).item()
    e0 = ((g0[k] - gf[k]).norm() / (gf[k].norm() + 1e-12)).item()
    print("%-24s vs f32: fused %.4f  layered %.4f" % (k, e1, e0))
