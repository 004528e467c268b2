"""3x3 / stride-1 weight gradients on every wgrad variant, incl. the row-image kernel
(variant 6, csrc/kernels/conv_wgrad.hip wgrad_rows_kernel): ResNet-50 layer1/2 and VGG-16
shapes, batch 256 (VGG's 224x224 layer at the per-launch pixel cap), TF/s per variant."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

H_ = hip()
# (N, H, Cin, Cout)
SHAPES = [(256, 56, 64, 64), (256, 28, 128, 128), (256, 14, 256, 256), (256, 7, 512, 512), (160, 224, 64, 64),
          (256, 112, 64, 128), (256, 112, 128, 128), (256, 56, 128, 256), (256, 56, 256, 256)]
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,3,4,5,6").split(",")]


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def timeit(f, n=10):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for N, Hh, C, K in SHAPES:
    x = cl(torch.randn(N, C, Hh, Hh, device="cuda")).bfloat16()
    dy = cl(torch.randn(N, K, Hh, Hh, device="cuda")).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x[:2].float(), (K, C, 3, 3), dy[:2].float(), stride=1, padding=1)
    flop = 2.0 * N * Hh * Hh * C * K * 9
    res = []
    for v in VARIANTS:
        try:
            H_.conv_wgrad_plan(N, Hh, Hh, C, K, 3, 1, v, -1)
        except Exception:  # noqa: BLE001
            continue
        err = ((H_.conv_wgrad(dy[:2].contiguous(memory_format=torch.channels_last),
                              x[:2].contiguous(memory_format=torch.channels_last), 3, 1, variant=v).float() - ref).norm()
               / ref.norm()).item()
        us = timeit(lambda: H_.conv_wgrad(dy, x, 3, 1, variant=v))
        res.append("v%d:%.0fus/%.0fTF%s" % (v, us, flop / us / 1e6, "" if err < 1e-2 else "/ERR%.3g" % err))
    print("N=%d H=%3d %3d->%3d  %s" % (N, Hh, C, K, " ".join(res)), flush=True)
