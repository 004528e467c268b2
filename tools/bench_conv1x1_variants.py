"""ResNet-50 1x1 convolution shapes (batch 256, NHWC bf16) on every tile variant of the MFMA
conv kernel, with the fused BN-statistics epilogue the bottleneck uses: time, achieved HBM
bandwidth (input + output bytes) and TF/s.  Picks the memory-bound shapes' best tile."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

H_ = hip()
# (H, Cin, Cout, stride[, ks]); KS3=1 adds ResNet-50's stride-1 3x3 shapes
SHAPES = [(56, 64, 64, 1), (56, 64, 256, 1), (56, 256, 64, 1), (56, 256, 128, 1), (28, 128, 512, 1),
          (28, 512, 128, 1), (14, 256, 1024, 1), (14, 1024, 256, 1), (7, 512, 2048, 1), (7, 2048, 512, 1)]
if os.environ.get("KS3") == "1":
    SHAPES = [(56, 64, 64, 1, 3), (28, 128, 128, 1, 3), (14, 256, 256, 1, 3), (7, 512, 512, 1, 3)]


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


N = int(os.environ.get("BATCH", "256"))
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,5,6").split(",")]
MODES = os.environ.get("MODES", "st,").split(",")
for shp in SHAPES:
    Hh, C, K, s = shp[:4]
    ks = shp[4] if len(shp) > 4 else 1
    x = cl(torch.randn(N, C, Hh, Hh, device="cuda")).bfloat16()
    w = cl(torch.randn(K, C, ks, ks, device="cuda") * 0.05).bfloat16()
    st = torch.zeros(H_.conv_stat_slots * 2 * K, dtype=torch.float64, device="cuda")
    M = N * (Hh // s) * (Hh // s)
    nbytes = 2.0 * (N * Hh * Hh * C + M * K)
    flop = 2.0 * M * K * C * ks * ks
    res = []
    OH = Hh // s
    out = cl(torch.randn(N, K, OH, OH, device="cuda")).bfloat16()
    bx = torch.empty_like(out)
    mask = torch.zeros(out.numel() // 8, dtype=torch.uint8, device="cuda")
    fc = torch.cat([torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.2])
    modes = {"st": (lambda v: H_.conv(x, w, s, st, None, v), 0),
             "": (lambda v: H_.conv(x, w, s, None, None, v), 0),
             # dgrad-style: accumulate into `out` + BN-backward sums over bx and the ReLU mask
             "ab": (lambda v: H_.conv(x, w, s, st, out, v, bn_x=bx, bn_mask=mask), 4.0 * M * K),
             # dgrad-style without accumulation: BN-backward sums over bx with the forward coefficients
             "bc": (lambda v: H_.conv(x, w, s, st, None, v, bn_x=bx, bn_fcoef=fc), 2.0 * M * K)}
    for v in VARIANTS:
        for tag in MODES:
            f, extra = modes[tag]
            try:
                us = timeit(lambda: f(v))
            except Exception:  # noqa: BLE001
                continue
            res.append("v%d%s:%.0fus/%.1fTB/s/%.0fTF" % (v, tag, us, (nbytes + extra) / us / 1e6, flop / us / 1e6))
    print("H=%2d %4d->%4d k%d  %6.0fMB %5.1fGF  %s" % (Hh, C, K, ks, nbytes / 1e6, flop / 1e9, " ".join(res)), flush=True)
