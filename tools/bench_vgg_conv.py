"""MFMA 3x3 conv on the VGG-16 shapes (batch 256, NHWC bf16): TF/s per tile variant, and a
single-shape mode for PMC counter passes.

    python tools/bench_vgg_conv.py                 # all shapes x variants (fwd) + dgrad default
    python tools/bench_vgg_conv.py --shape 2 --variant -1 --iters 50   # one shape, for rocprofv3 --pmc
"""
import argparse
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

H_ = hip()
SHAPES = [(224, 64, 64), (112, 128, 128), (56, 256, 256), (28, 512, 512), (14, 512, 512)]


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
    ap.add_argument("--shape", type=int, default=-1)
    ap.add_argument("--variant", type=int, default=None)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--gemm", action="store_true", help="also time hipBLASLt on the equivalent im2col GEMM")
    a = ap.parse_args()
    N = a.batch
    shapes = SHAPES if a.shape < 0 else [SHAPES[a.shape]]
    variants = list(range(H_.conv3x3_variants())) if a.variant is None else [a.variant]
    for Hh, C, K in shapes:
        x = cl(torch.randn(N, C, Hh, Hh, device="cuda")).bfloat16()
        w = cl(torch.randn(K, C, 3, 3, device="cuda") * 0.05).bfloat16()
        flop = 2.0 * N * Hh * Hh * K * C * 9
        res = []
        for v in variants:
            try:
                us = timeit(lambda: H_.conv(x, w, 1, None, None, v), a.iters)
            except Exception as e:  # noqa: BLE001
                res.append("v%d:n/a" % v)
                continue
            res.append("v%d:%.0fus/%.0fTF" % (v, us, flop / us / 1e6))
        if a.gemm:  # the library ceiling for the same GEMM (M = N*H*W, K = 9*C), no im2col cost counted
            A = torch.randn(N * Hh * Hh, 9 * C, device="cuda").bfloat16()
            B = torch.randn(9 * C, K, device="cuda").bfloat16()
            us = timeit(lambda: torch.mm(A, B), a.iters)
            res.append("hipblaslt:%.0fus/%.0fTF" % (us, flop / us / 1e6))
            del A, B
        print("H=%3d C=%3d K=%3d  %s" % (Hh, C, K, "  ".join(res)), flush=True)


if __name__ == "__main__":
    main()
