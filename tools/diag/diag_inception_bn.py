"""Per-layer relative error of Inception-v3 with the HIP BN+ReLU vs stock BN (bf16 autocast)."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from kungfu_amd.models import get_model
from kungfu_amd.models.inception import BasicConv2d

torch.manual_seed(7)
ref = get_model("inception_v3").cuda().to(memory_format=torch.channels_last)
fused = get_model("inception_v3", fused_bn=True).cuda().to(memory_format=torch.channels_last)
fused.load_state_dict(ref.state_dict())
x = torch.randn(4, 3, 128, 128, device="cuda").to(memory_format=torch.channels_last)
acts = {0: [], 1: []}
for k, m in enumerate((ref, fused)):
    for name, mod in m.named_modules():
        if isinstance(mod, BasicConv2d):
            mod.register_forward_hook(lambda mo, i, o, k=k, name=name: acts[k].append((name, i[0].detach(), o.detach())))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        m(x)
for (n, i0, o0), (_, i1, o1) in zip(acts[0], acts[1]):
    # same-input check: rerun the fused layer on the reference input
    mod = dict(fused.named_modules())[n]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        o1s = mod(i0)
    e = ((o1.float() - o0.float()).norm() / o0.float().norm()).item()
    es = ((o1s.float() - o0.float()).norm() / o0.float().norm()).item()
    print("%-22s C=%4d %s cl=%d  chain %.3e  same-input %.3e" % (n, o0.shape[1], tuple(o0.shape[2:]), int(
        i0.is_contiguous(memory_format=torch.channels_last)), e, es))
