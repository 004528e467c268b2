"""Every default-eligible tile variant (0 128x128, 1 256x128, 2 256x64, 7 256x256) of the MFMA conv
kernel on ResNet-50's bottleneck convolutions (batch 256) WITH the fused epilogue each one runs in
the step (tools/bench_conv_epi.py's ops plus the stride-1 3x3 forward / data gradient), next to the
launcher's default: us per variant, best marked.  A default that loses by > 5 % is a retune candidate.

Usage: python tools/bench_conv_tiles.py [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

STAGES = [(56, 256, 64), (28, 512, 128), (14, 1024, 256), (7, 2048, 512)]


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def timeit(f, n):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    H_ = hip()
    N = a.batch
    for Hh, Cb, w in STAGES:
        M = N * Hh * Hh
        for op in ("c1f", "c3f", "c3d", "c1d", "f3", "d3"):
            ks = 3 if op in ("f3", "d3") else 1
            cin, cout = {"c1f": (Cb, w), "c3f": (w, Cb), "c3d": (Cb, w), "c1d": (w, Cb), "f3": (w, w),
                         "d3": (w, w)}[op]
            x = cl(torch.randn(N, cin, Hh, Hh, device="cuda")).bfloat16()
            wt = cl(torch.randn(cout, cin, ks, ks, device="cuda") * 0.05).bfloat16()
            st = torch.zeros(H_.conv_stat_slots * 2 * cout, dtype=torch.float64, device="cuda")
            if op in ("c1f", "c3f", "f3"):
                f = lambda v: H_.conv(x, wt, 1, st, None, v)  # noqa: E731
            elif op in ("c3d", "d3"):
                bx = cl(torch.randn(N, cout, Hh, Hh, device="cuda")).bfloat16()
                fc = torch.cat([torch.rand(cout, device="cuda") + 0.5, torch.randn(cout, device="cuda") * 0.2])
                f = lambda v: H_.conv(x, wt, 1, st, None, v, bx, fc, None)  # noqa: E731
            else:
                out = cl(torch.randn(N, cout, Hh, Hh, device="cuda")).bfloat16()
                bx = cl(torch.randn(N, cout, Hh, Hh, device="cuda")).bfloat16()
                bm = torch.randint(0, 256, (M * cout // 8,), dtype=torch.uint8, device="cuda")
                am = torch.randint(0, 256, (M * cout // 8,), dtype=torch.uint8, device="cuda")
                f = lambda v: H_.conv(x, wt, 1, st, out, v, bx, None, bm, acc_mask=am)  # noqa: E731
            res = {}
            ok = []
            for v in (0, 1, 2, 7, -1):
                try:
                    f(v)
                    ok.append(v)
                except Exception:  # noqa: BLE001
                    pass
            for _ in range(3):  # interleaved rounds, min: the first timing of a fresh op runs slow (clocks)
                for v in ok:
                    t = timeit(lambda: f(v), a.iters)
                    res[v] = min(res.get(v, t), t)
            best = min((t, v) for v, t in res.items() if v >= 0)
            flag = "  RETUNE" if res[-1] > 1.05 * best[0] else ""
            print("%-3s H=%2d %4d->%4d  default %6.1f us | %s | best v%d%s" % (
                op, Hh, cin, cout, res[-1], "  ".join("v%d %6.1f" % (v, t) for v, t in sorted(res.items()) if v >= 0),
                best[1], flag), flush=True)


if __name__ == "__main__":
    main()
