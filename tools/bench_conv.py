"""Correctness + speed of the general MFMA convolution kernel (csrc/kernels/conv.hip) on the
ResNet-50 1x1 shapes (and a few 3x3) at batch 256, NHWC bf16, against MIOpen:
forward, forward + fused BN statistics, stride-1 data gradient, data gradient accumulated
into an existing tensor (the residual-gradient add)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from kungfu_amd._lib import hip  # noqa: E402

torch.backends.cudnn.benchmark = False
H_ = hip()
dev = torch.device("cuda")
# (H, Cin, Cout, ks, stride)
SHAPES = [(56, 64, 64, 1, 1), (56, 64, 256, 1, 1), (56, 256, 64, 1, 1), (56, 256, 128, 1, 1), (56, 256, 512, 1, 2),
          (28, 128, 512, 1, 1), (28, 512, 128, 1, 1), (28, 512, 256, 1, 1), (28, 512, 1024, 1, 2),
          (14, 256, 1024, 1, 1), (14, 1024, 256, 1, 1), (14, 1024, 512, 1, 1), (14, 1024, 2048, 1, 2),
          (7, 512, 2048, 1, 1), (7, 2048, 512, 1, 1), (56, 64, 64, 3, 1), (14, 256, 256, 3, 1)]


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
tot = {"fwd_m": 0.0, "fwd_o": 0.0, "fst_o": 0.0, "bn_stats_m": 0.0, "dg_m": 0.0, "dg_o": 0.0, "dga_o": 0.0,
       "add_m": 0.0}
for Hh, C, K, ks, s in SHAPES:
    pad = (ks - 1) // 2
    # ---- correctness at batch 2 against f32
    x = cl(torch.randn(2, C, Hh, Hh, device=dev)).bfloat16()
    w = cl(torch.randn(K, C, ks, ks, device=dev) * 0.05).bfloat16()
    ref = F.conv2d(x.float(), w.float(), stride=s, padding=pad)
    st = torch.zeros(H_.conv_stat_slots, 2 * K, dtype=torch.float64, device=dev)
    y = H_.conv(x, w, s, st)
    st = st.sum(0)
    e_f = rel(y, ref)
    yf = y.float()
    s1 = yf.sum((0, 2, 3)).double()
    s2 = (yf * yf).sum((0, 2, 3)).double()
    e_s = max(rel(st[:K], s1), rel(st[K:], s2))
    line = "H=%3d C=%4d K=%4d ks=%d s=%d  fwd %.1e stats %.1e" % (Hh, C, K, ks, s, e_f, e_s)
    ok &= e_f < 1e-2 and e_s < 1e-3
    if s == 1:
        dy = cl(torch.randn_like(ref)).bfloat16()
        dx_ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), stride=1, padding=pad)
        wt = H_.conv_flip_weight(w)
        dx = H_.conv(dy, wt, 1)
        base = cl(torch.randn_like(x.float())).bfloat16()
        acc = base.clone()
        H_.conv(dy, wt, 1, None, acc)
        e_d = rel(dx, dx_ref)
        e_a = rel(acc, dx_ref + base.float())
        line += " dgrad %.1e accum %.1e" % (e_d, e_a)
        ok &= e_d < 1e-2 and e_a < 1e-2
    # ---- speed at batch 256
    N = 256
    x = cl(torch.randn(N, C, Hh, Hh, device=dev)).bfloat16()
    w = cl(torch.randn(K, C, ks, ks, device=dev) * 0.05).bfloat16()
    OH = (Hh + 2 * pad - ks) // s + 1
    st = torch.zeros(H_.conv_stat_slots * 2 * K, dtype=torch.float64, device=dev)
    t_m = timeit(lambda: F.conv2d(x, w, stride=s, padding=pad))
    t_o = timeit(lambda: H_.conv(x, w, s))
    t_os = timeit(lambda: H_.conv(x, w, s, st))
    yb = H_.conv(x, w, s)
    t_bs = timeit(lambda: torch.ops.aten.var_mean(yb, (0, 2, 3)))  # stand-in for a stats pass
    tot["fwd_m"] += t_m
    tot["fwd_o"] += t_o
    tot["fst_o"] += t_os
    line += " | fwd miopen %6.1f ours %6.1f +stats %6.1f" % (t_m, t_o, t_os)
    byt = 2.0 * (N * Hh * Hh * C + N * OH * OH * K + K * C * ks * ks)
    fl = 2.0 * N * OH * OH * K * C * ks * ks
    line += " (%.2f TB/s %.0f TF/s)" % (byt / t_o / 1e6, fl / t_o / 1e6)
    vs = []
    for v in range(H_.conv3x3_variants()):
        if v in (0, 1) and K % 128:
            continue
        try:
            vs.append((timeit(lambda: H_.conv(x, w, s, None, None, v)), v))
        except ValueError:  # tile does not fit this shape
            pass
    vs.sort()
    line += " [best v%d %.1f, %s]" % (vs[0][1], vs[0][0], " ".join("v%d %.0f" % (v, t) for t, v in sorted(vs, key=lambda z: z[1])))
    if s == 1:
        dy = cl(torch.randn(N, K, OH, OH, device=dev)).bfloat16()
        wt = H_.conv_flip_weight(w)
        acc = cl(torch.randn(N, C, Hh, Hh, device=dev)).bfloat16()
        t_md = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [pad, pad], [1, 1], False,
                                                                  [0, 0], 1, [True, False, False]))
        t_od = timeit(lambda: H_.conv(dy, wt, 1))
        t_oa = timeit(lambda: H_.conv(dy, wt, 1, None, acc))
        t_add = timeit(lambda: acc.add_(x))
        tot["dg_m"] += t_md
        tot["dg_o"] += t_od
        tot["dga_o"] += t_oa
        tot["add_m"] += t_add
        line += " | dgrad miopen %6.1f ours %6.1f accum %6.1f (torch add %5.1f)" % (t_md, t_od, t_oa, t_add)
    print(line, flush=True)
print("TOTAL (one of each shape, us): " + " ".join("%s=%.0f" % kv for kv in tot.items()))
print("CONV_OK" if ok else "CONV_MISMATCH")
