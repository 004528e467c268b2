"""ResNet-50's 1x1 bottleneck convolutions (batch 256, NHWC bf16) with the exact fused epilogues the
fused block uses (ops/fused_block.py), on the default tile of the MFMA conv kernel: time and achieved
HBM bandwidth of the bytes the op must move (input + output + the epilogue's reads).

  c1f  conv1 forward, BN-statistics epilogue           Cb -> w
  c3f  conv3 forward, BN-statistics epilogue           w -> 4w
  c3d  conv3 data gradient, BN-backward sums (coef)    4w -> w     (+ reads bn_x)
  c1d  conv1 data gradient in place: accumulate into the masked residual gradient, BN3-backward
       sums of the previous block (1-bit mask)         w -> 4w     (+ reads old, bn_x, 2 masks)

Usage: python tools/bench_conv_epi.py [--ops c1f,c3f,c3d,c1d] [--iters 30]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

STAGES = [(56, 256, 64), (28, 512, 128), (14, 1024, 256), (7, 2048, 512)]  # (H, block in/out channels, width)


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def timeit(f, n):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="c1f,c3f,c3d,c1d")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    H_ = hip()
    N = a.batch
    tot = {}
    for Hh, Cb, w in STAGES:
        M = N * Hh * Hh
        for op in a.ops.split(","):
            cin, cout = {"c1f": (Cb, w), "c3f": (w, Cb), "c3d": (Cb, w), "c1d": (w, Cb)}[op]
            x = cl(torch.randn(N, cin, Hh, Hh, device="cuda")).bfloat16()
            wt = cl(torch.randn(cout, cin, 1, 1, device="cuda") * 0.05).bfloat16()
            st = torch.zeros(H_.conv_stat_slots * 2 * cout, dtype=torch.float64, device="cuda")
            nbytes = 2.0 * M * (cin + cout)
            if op in ("c1f", "c3f"):
                f = lambda: H_.conv(x, wt, 1, st)  # noqa: E731
            elif op == "c3d":
                bx = cl(torch.randn(N, cout, Hh, Hh, device="cuda")).bfloat16()
                fc = torch.cat([torch.rand(cout, device="cuda") + 0.5, torch.randn(cout, device="cuda") * 0.2])
                nbytes += 2.0 * M * cout
                f = lambda: H_.conv(x, wt, 1, st, None, -1, bx, fc, None)  # noqa: E731
            else:
                out = cl(torch.randn(N, cout, Hh, Hh, device="cuda")).bfloat16()
                bx = cl(torch.randn(N, cout, Hh, Hh, device="cuda")).bfloat16()
                bm = torch.randint(0, 256, (M * cout // 8,), dtype=torch.uint8, device="cuda")
                am = torch.randint(0, 256, (M * cout // 8,), dtype=torch.uint8, device="cuda")
                nbytes += 2.0 * M * cout * 2 + M * cout / 4
                f = lambda: H_.conv(x, wt, 1, st, out, -1, bx, None, bm, acc_mask=am)  # noqa: E731
            us = timeit(f, a.iters)
            tot[op] = tot.get(op, 0.0) + us
            print("%-4s H=%2d %4d->%4d  %7.1f us  %6.0f MB  %.2f TB/s" % (op, Hh, cin, cout, us, nbytes / 1e6,
                                                                         nbytes / us / 1e6), flush=True)
    print("totals: " + "  ".join("%s %.1f us" % kv for kv in tot.items()) + "  all %.1f us" % sum(tot.values()))


if __name__ == "__main__":
    main()
