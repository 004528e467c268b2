"""Correctness + speed of the MFMA 3x3 implicit-GEMM convolution (csrc/kernels/conv.hip)
against MIOpen (torch.nn.functional.conv2d / aten.convolution_backward) for the ResNet-50 3x3
shapes at batch 256, NHWC bf16.  Correctness vs an f32 reference at batch 2."""
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from kungfu_amd._lib import hip  # noqa: E402

torch.backends.cudnn.benchmark = False
H_ = hip()
dev = torch.device("cuda")
SHAPES = [(56, 64, 64, 1), (56, 128, 128, 2), (28, 128, 128, 1), (28, 256, 256, 2), (14, 256, 256, 1),
          (14, 512, 512, 2), (7, 512, 512, 1)]


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


ok = True
for Hh, C, K, s in SHAPES:
    # correctness (small batch, f32 reference)
    x = cl(torch.randn(2, C, Hh, Hh, device=dev)).bfloat16()
    w = cl(torch.randn(K, C, 3, 3, device=dev) * 0.05).bfloat16()
    ref = F.conv2d(x.float(), w.float(), stride=s, padding=1)
    y = H_.conv3x3(x, w, s)
    e_f = rel(y, ref)
    line = "H=%3d C=%4d K=%4d s=%d  fwd rel %.2e" % (Hh, C, K, s, e_f)
    if s == 1:
        dy = cl(torch.randn_like(ref)).bfloat16()
        dx_ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), stride=1, padding=1)
        dx = H_.conv3x3(dy, H_.conv3x3_flip_weight(w), 1)
        e_d = rel(dx, dx_ref)
        line += "  dgrad rel %.2e" % e_d
        ok &= e_d < 1e-2
    ok &= e_f < 1e-2
    # speed at batch 256
    N = 256
    x = cl(torch.randn(N, C, Hh, Hh, device=dev)).bfloat16()
    w = cl(torch.randn(K, C, 3, 3, device=dev) * 0.05).bfloat16()
    OH = (Hh + 2 - 3) // s + 1
    fl = 2.0 * N * OH * OH * K * C * 9
    t_m = timeit(lambda: F.conv2d(x, w, stride=s, padding=1))
    t_o = timeit(lambda: H_.conv3x3(x, w, s))
    line += " | fwd miopen %6.1f us (%4.0f TF)  ours %6.1f us (%4.0f TF)" % (t_m, fl / t_m / 1e6, t_o, fl / t_o / 1e6)
    vs = []
    for v in range(H_.conv3x3_variants()):
        if v in (0, 1) and K % 128:
            continue
        yv = H_.conv3x3(x[:2].contiguous(memory_format=torch.channels_last), w, s, v)
        assert rel(yv, F.conv2d(x[:2].float(), w.float(), stride=s, padding=1)) < 1e-2, ("variant", v)
        vs.append("v%d %.1f" % (v, timeit(lambda: H_.conv3x3(x, w, s, v))))
    line += " [" + ", ".join(vs) + "]"
    if s == 1:
        dy = cl(torch.randn(N, K, OH, OH, device=dev)).bfloat16()
        wt = H_.conv3x3_flip_weight(w)
        t_md = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False,
                                                                  [0, 0], 1, [True, False, False]))
        t_od = timeit(lambda: H_.conv3x3(dy, wt, 1))
        t_fl = timeit(lambda: H_.conv3x3_flip_weight(w))
        line += " | dgrad miopen %6.1f us  ours %6.1f us (+flip %.1f)" % (t_md, t_od, t_fl)
    print(line, flush=True)
print("CONV3X3_OK" if ok else "CONV3X3_MISMATCH")
