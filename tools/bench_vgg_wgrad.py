"""Weight gradient of the VGG-16 3x3 convolutions (batch 256, NHWC bf16) on the split-K MFMA
kernel: every tile variant x a few split counts per shape (TF/s), the default plan, and
MIOpen for reference.  Shapes whose output exceeds the kernel's 2^23-pixel launch limit are
timed on a 128-image half (the engine sums two such launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

H_ = hip()
SHAPES = [(224, 64, 64), (112, 64, 128), (112, 128, 128), (56, 128, 256), (56, 256, 256), (28, 256, 512),
          (28, 512, 512), (14, 512, 512)]


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


for Hh, C, K in SHAPES:
    N = 256 if 256 * Hh * Hh < (1 << 23) else 128
    x = cl(torch.randn(N, C, Hh, Hh, device="cuda")).bfloat16()
    dy = cl(torch.randn(N, K, Hh, Hh, device="cuda")).bfloat16()
    flop = 2.0 * N * Hh * Hh * K * C * 9
    res = ["default:%.0fus/%.0fTF" % ((lambda us: (us, flop / us / 1e6))(timeit(lambda: H_.conv_wgrad(dy, x, 3, 1))))]
    for v in range(H_.conv_wgrad_variants()):
        for sp in (-1, 16, 32, 64, 128, 256, 512):
            try:
                us = timeit(lambda: H_.conv_wgrad(dy, x, 3, 1, variant=v, splits=sp))
            except Exception:  # noqa: BLE001
                continue
            res.append("v%d/s%d:%.0fTF" % (v, sp, flop / us / 1e6))
    w = cl(torch.randn(K, C, 3, 3, device="cuda")).bfloat16()
    us = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                            [False, True, False]))
    res.append("miopen:%.0fTF" % (flop / us / 1e6))
    print("N=%d H=%3d %3d->%3d  %s" % (N, Hh, C, K, " ".join(res)), flush=True)
    del x, dy
