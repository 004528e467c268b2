"""1x1 weight gradients (ResNet-50 bottleneck shapes at batch 256, BERT-base linear layers at
16384 tokens as 1 x T "images") on every tap-tiled wgrad variant with the planner's split
count: time and TF/s per variant (csrc/kernels/conv_wgrad.hip)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

H_ = hip()
# (N, H, W, Cin, Cout)
SHAPES = [(256, 56, 56, 64, 256), (256, 56, 56, 256, 64), (256, 28, 28, 128, 512), (256, 28, 28, 512, 128),
          (256, 14, 14, 256, 1024), (256, 14, 14, 1024, 256), (256, 7, 7, 512, 2048), (256, 7, 7, 2048, 512),
          (1, 1, 16384, 768, 2304), (1, 1, 16384, 768, 768), (1, 1, 16384, 768, 3072), (1, 1, 16384, 3072, 768)]
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,4,5,7").split(",")]


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def timeit(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for N, Hh, Ww, C, K in SHAPES:
    x = cl(torch.randn(N, C, Hh, Ww, device="cuda")).bfloat16()
    dy = cl(torch.randn(N, K, Hh, Ww, device="cuda")).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x[:1].float(), (K, C, 1, 1), dy[:1].float()) if N > 1 else None
    flop = 2.0 * N * Hh * Ww * C * K
    res = []
    for v in VARIANTS:
        try:
            pl = H_.conv_wgrad_plan(N, Hh, Ww, C, K, 1, 1, v, -1)
        except Exception:  # noqa: BLE001
            continue
        if ref is not None:
            got = H_.conv_wgrad(cl(dy[:1]), cl(x[:1]), 1, 1, variant=v).float()
            if ((got - ref).norm() / ref.norm()).item() > 1e-2:
                res.append("v%d:ERR" % v)
                continue
        us = timeit(lambda: H_.conv_wgrad(dy, x, 1, 1, variant=v))
        res.append("v%d(%d):%.0fus/%.0fTF" % (v, pl[1], us, flop / us / 1e6))
    dflt = H_.conv_wgrad_plan(N, Hh, Ww, C, K, 1, 1, -1, -1)[0]
    print("%4dx%2dx%5d %4d->%4d default v%d  %s" % (N, Hh, Ww, C, K, dflt, " ".join(res)), flush=True)
