"""BERT-base linear-layer GEMMs (T = batch * seq tokens, bf16) on the MFMA conv kernel (a linear
layer is a 1x1 convolution over T "pixels") vs hipBLASLt (``F.linear`` / ``torch.mm``): time and
TF/s per tile variant, forward (x W^T) and data gradient (dy W) shapes."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

H_ = hip()
T = int(os.environ.get("TOKENS", "16384"))
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,3").split(",")]
# (name, in, out): forward products; the data gradient of (in -> out) is the (out -> in) product
SHAPES = [("qkv", 768, 2304), ("out", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768),
          ("qkv.dg", 2304, 768), ("fc1.dg", 3072, 768), ("fc2.dg", 768, 3072)]


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


for name, cin, cout in SHAPES:
    x = torch.randn(T, cin, device="cuda").bfloat16()
    w = (torch.randn(cout, cin, device="cuda") * 0.05).bfloat16()
    b = torch.zeros(cout, device="cuda").bfloat16()
    flop = 2.0 * T * cin * cout
    ref = F.linear(x, w)
    res = ["blas:%.0fus/%.0fTF" % ((us := timeit(lambda: F.linear(x, w, b))), flop / us / 1e6)]
    for v in VARIANTS:
        try:
            y = H_.gemm(x, w, variant=v)[0]
            err = (y.float() - ref.float()).abs().max().item()
            us = timeit(lambda: H_.gemm(x, w, variant=v))
            usb = timeit(lambda: H_.gemm(x, w, b, variant=v))
        except Exception as e:  # noqa: BLE001
            res.append("v%d:-" % v)
            continue
        res.append("v%d:%.0fus/%.0fTF(bias %.0f)%s" % (v, us, flop / us / 1e6, usb,
                                                    "" if err < 0.5 else "(err %.2f)" % err))
    u = torch.randn(T, cout, device="cuda").bfloat16()
    st = torch.zeros(H_.conv_stat_slots * 2 * cout, dtype=torch.float64, device="cuda")
    res.append("geluG:%.0fus" % timeit(lambda: H_.gemm(x, w, gelu_u=u, stats=st)))
    res.append("acc:%.0fus" % timeit(lambda: H_.gemm(x, w, out=u)))
    print("%-7s %4d->%4d %5.1fGF  %s" % (name, cin, cout, flop / 1e9, " ".join(res)), flush=True)

# weight gradients dW[out, in] = dy^T x over T tokens: split-K MFMA kernel (ops/linear.py) vs hipBLASLt
print("weight gradients (T=%d)" % T, flush=True)


def as4d(t2):
    n, c = t2.shape
    return t2.as_strided((1, c, 1, n), (n * c, 1, n * c, c))


for name, cin, cout in SHAPES[:4]:
    x = torch.randn(T, cin, device="cuda").bfloat16()
    dy = torch.randn(T, cout, device="cuda").bfloat16()
    flop = 2.0 * T * cin * cout
    t_blas = timeit(lambda: torch.mm(dy.t(), x))
    t_blas2 = timeit(lambda: torch.matmul(x.t(), dy))
    t_ours = timeit(lambda: H_.conv_wgrad(as4d(dy), as4d(x), 1, 1))
    ref = torch.mm(dy.t().float(), x.float())
    err = ((H_.conv_wgrad(as4d(dy), as4d(x), 1, 1).view(cout, cin).float() - ref).norm() / ref.norm()).item()
    print("%-7s %4d->%4d  blas dy^T x %.0fus/%.0fTF  blas x^T dy %.0fus  ours %.0fus/%.0fTF (rel %.1e)" % (
        name, cin, cout, t_blas, flop / t_blas / 1e6, t_blas2, t_ours, flop / t_ours / 1e6, err), flush=True)
