"""Correctness + speed of the split-K MFMA weight-gradient kernel (csrc/kernels/conv_wgrad.hip)
against MIOpen (aten.convolution_backward, weight only) on every ResNet-50 bottleneck conv
shape at batch 256, NHWC bf16, weighted by how often each shape occurs in one step.

Usage: python tools/bench_wgrad.py [--sweep]   (--sweep: time every tile variant x split count)
"""
import sys

import torch

sys.path.insert(0, ".")
from kungfu_amd._lib import hip  # noqa: E402

torch.backends.cudnn.benchmark = False
H_ = hip()
dev = torch.device("cuda")
# (H_in, Cin, Cout, ks, stride, occurrences per ResNet-50 step)
SHAPES = [
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (56, 256, 512, 1, 2, 1),
    (28, 128, 512, 1, 1, 4), (28, 512, 128, 1, 1, 3), (28, 128, 128, 3, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (28, 512, 1024, 1, 2, 1),
    (14, 256, 1024, 1, 1, 6), (14, 1024, 256, 1, 1, 5), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (14, 1024, 2048, 1, 2, 1),
    (7, 512, 2048, 1, 1, 3), (7, 2048, 512, 1, 1, 2), (7, 512, 512, 3, 1, 2),
]


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


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
    return e0.elapsed_time(e1) / n * 1e3  # us


def main():
    sweep = "--sweep" in sys.argv
    only = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--h=")]
    ok = True
    tot_m = tot_o = 0.0
    for Hh, C, K, ks, s, cnt in SHAPES:
        if only and Hh not in only:
            continue
        pad = (ks - 1) // 2
        OH = (Hh + 2 * pad - ks) // s + 1
        # ---- correctness at batch 3 (odd pixel count: exercises the K tail) against f32
        x = cl(torch.randn(3, C, Hh, Hh, device=dev)).bfloat16()
        dy = cl(torch.randn(3, K, OH, OH, device=dev)).bfloat16()
        ref = torch.nn.grad.conv2d_weight(x.float(), (K, C, ks, ks), dy.float(), stride=s, padding=pad)
        e1 = rel(H_.conv_wgrad(dy, x, ks, s), ref)
        e2 = rel(H_.conv_wgrad(dy, x, ks, s, splits=1), ref)
        out = cl(torch.randn(K, C, ks, ks, device=dev))
        base = out.clone()
        H_.conv_wgrad(dy, x, ks, s, out=out, accumulate=True)
        e3 = rel(out, ref + base)
        ok &= max(e1, e2) < 1e-2 and e3 < 1e-3
        # ---- speed at batch 256
        N = 256
        x = cl(torch.randn(N, C, Hh, Hh, device=dev)).bfloat16()
        dy = cl(torch.randn(N, K, OH, OH, device=dev)).bfloat16()
        w = cl(torch.randn(K, C, ks, ks, device=dev)).bfloat16()
        t_m = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [pad, pad], [1, 1], False,
                                                                 [0, 0], 1, [False, True, False]))
        t_o = timeit(lambda: H_.conv_wgrad(dy, x, ks, s))
        of32 = cl(torch.zeros(K, C, ks, ks, device=dev))
        t_at = timeit(lambda: H_.conv_wgrad(dy, x, ks, s, out=of32, accumulate=True))
        tot_a = globals().setdefault("_tot_a", [0.0])
        tot_a[0] += cnt * t_at
        plan = H_.conv_wgrad_plan(N, Hh, Hh, C, K, ks, s)
        e4 = rel(H_.conv_wgrad(dy, x, ks, s), torch.ops.aten.convolution_backward(
            dy, x, w, None, [s, s], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False])[1])
        ok &= e4 < 2e-2
        tot_m += cnt * t_m
        tot_o += cnt * t_o
        gb = (x.numel() / (s * s if ks == 1 else 1) + dy.numel()) * 2 / 1e9
        line = ("H=%2d C=%4d K=%4d ks=%d s=%d x%d  err %.1e/%.1e/%.1e/%.1e | miopen %7.1f ours %7.1f atomic-f32 %7.1f us "
                "(plan v%d splits %d; %.0f GB/s, %.0f TF/s)" % (
                    Hh, C, K, ks, s, cnt, e1, e2, e3, e4, t_m, t_o, t_at, plan[0], plan[1], gb / t_o * 1e6,
                    2.0 * N * OH * OH * K * C * ks * ks / t_o / 1e6))
        if sweep:
            res = []
            for v in range(H_.conv_wgrad_variants()):
                try:
                    H_.conv_wgrad_plan(N, Hh, Hh, C, K, ks, s, v, -1)
                except Exception:
                    continue
                seen = set()
                for sp in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024):
                    sp = H_.conv_wgrad_plan(N, Hh, Hh, C, K, ks, s, v, sp)[1]
                    if sp in seen:
                        continue
                    seen.add(sp)
                    res.append((timeit(lambda: H_.conv_wgrad(dy, x, ks, s, variant=v, splits=sp), n=10), v, sp))
                    res.append((timeit(lambda: H_.conv_wgrad(dy, x, ks, s, out=of32, accumulate=True, variant=v,
                                                             splits=sp), n=10), v, -sp))
            res.sort()
            line += " | best: " + " ".join("v%d/%s%d %.0f" % (v, "a" if sp < 0 else "s", abs(sp), t)
                                           for t, v, sp in res[:5])
        print(line, flush=True)
    print("TOTAL per step (weighted by occurrences, us): miopen %.0f ours %.0f atomic-f32 %.0f" % (
        tot_m, tot_o, globals().get("_tot_a", [0.0])[0]))
    print("WGRAD_OK" if ok else "WGRAD_MISMATCH")


if __name__ == "__main__":
    main()
