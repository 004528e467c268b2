"""The stride-1 3x3 convolutions of ResNet-50 at batch 256 (fwd with the BN-statistics epilogue,
and the data gradient as the same conv on flipped weights), ours only, for PMC passes and A/Bs of
the conv kernel's tile variants:  python tools/bench_conv3x3_s1.py [variant ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

H_ = hip()
SHAPES = [(56, 64, 64), (28, 128, 128), (14, 256, 256), (7, 512, 512)]
if os.environ.get("SHAPES"):
    SHAPES = [SHAPES[int(i)] for i in os.environ["SHAPES"].split(",")]
N = int(os.environ.get("BATCH", "256"))
ITERS = int(os.environ.get("ITERS", "20"))
variants = [int(v) for v in sys.argv[1:]] or [-1]


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def timeit(f, n=ITERS):
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


for Hh, C, K in SHAPES:
    x = cl(torch.randn(N, C, Hh, Hh, device="cuda")).bfloat16()
    w = cl(torch.randn(K, C, 3, 3, device="cuda") * 0.05).bfloat16()
    st = torch.zeros(H_.conv_stat_slots * 2 * K, dtype=torch.float64, device="cuda")
    fl = 2.0 * N * Hh * Hh * K * C * 9
    # the data gradient as the bottleneck runs it: dy (K channels) on flipped weights, BN-backward sums
    dy = cl(torch.randn(N, K, Hh, Hh, device="cuda")).bfloat16()
    wt = H_.conv_flip_weight(w)
    bx = cl(torch.randn(N, C, Hh, Hh, device="cuda")).bfloat16()
    fc = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2])
    st2 = torch.zeros(H_.conv_stat_slots * 2 * C, dtype=torch.float64, device="cuda")
    res = []
    for v in variants:
        for tag, f in (("fwd", lambda: H_.conv(x, w, 1, st, None, v)),
                       ("dgrad", lambda: H_.conv(dy, wt, 1, st2, None, v, bn_x=bx, bn_fcoef=fc))):
            try:
                us = timeit(f)
            except Exception as e:  # noqa: BLE001
                res.append("v%d %s: %s" % (v, tag, str(e).splitlines()[0][:40]))
                continue
            res.append("v%d %s %.1f us %.0f TF" % (v, tag, us, fl / us / 1e6))
    print("H=%2d %3d->%3d  %s" % (Hh, C, K, "  ".join(res)), flush=True)
