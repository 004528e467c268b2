"""Stem conv (7x7/2, 3 -> 64) on the MFMA kernels of csrc/kernels/stem.hip vs MIOpen at batch 256:
forward (+ BN statistics) and weight gradient, us."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from kungfu_amd._lib import hip  # noqa: E402

torch.backends.cudnn.benchmark = False
H_ = hip()


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


x = torch.randn(256, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
xb = x.bfloat16()
w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).bfloat16().contiguous(memory_format=torch.channels_last)
st = torch.zeros(H_.conv_stat_slots * 2 * 64, dtype=torch.float64, device="cuda")
x4 = H_.stem_pad4(x)
wp = H_.stem_pack_weight(w)
y = H_.stem_forward(x4, wp, None)
dy = torch.randn_like(y)
yref = F.conv2d(xb, w, stride=2, padding=3)
print("fwd rel err %.2e" % ((y.float() - yref.float()).norm() / yref.float().norm()).item())
t = {
    "miopen fwd (bf16 input)": timeit(lambda: F.conv2d(xb, w, stride=2, padding=3)),
    "miopen cast f32->bf16": timeit(lambda: x.bfloat16()),
    "ours pad4+cast": timeit(lambda: H_.stem_pad4(x)),
    "ours fwd": timeit(lambda: H_.stem_forward(x4, wp, None)),
    "ours fwd+stats": timeit(lambda: H_.stem_forward(x4, wp, st)),
    "y memset (write roofline)": timeit(lambda: y.zero_()),
    "miopen wgrad": timeit(lambda: torch.ops.aten.convolution_backward(dy, xb, w, None, [2, 2], [3, 3], [1, 1], False,
                                                                        [0, 0], 1, [False, True, False])),
    "ours wgrad": timeit(lambda: H_.stem_wgrad(dy, x4)),
}
for sp in (128, 256, 512, 1024, 2048):
    t["ours wgrad splits=%d" % sp] = timeit(lambda: H_.stem_wgrad(dy, x4, sp))
for k, v in t.items():
    print("%-28s %8.1f us" % (k, v))

# fused backward (pool gather + BN backward + weight gradient) vs the layered HIP path
from kungfu_amd.ops.fused_bn import BatchNormAct2d  # noqa: E402

bn = BatchNormAct2d(64).cuda()
st = torch.zeros(H_.conv_stat_slots * 2 * 64, dtype=torch.float64, device="cuda")
yc = H_.stem_forward(x4, wp, st)
yp, mean, invstd, coef, arg, xarg = H_.bn_pool_forward(yc, bn.weight, bn.bias, bn.running_mean, bn.running_var, 0.1, 1e-5,
                                                 True, None, st)
dyp = torch.randn_like(yp)
def layered():
    return H_.stem_wgrad(H_.bn_pool_backward(dyp, arg, yc, mean, invstd, bn.weight, coef, True, xarg)[0], x4)


def fused():
    bc = H_.bn_pool_backward(dyp, arg, yc, mean, invstd, bn.weight, coef, True, xarg, apply=False)[3]
    return H_.stem_wgrad_bnp(yc, x4, dyp, arg, coef, bc)


t2 = {
    "layered: bn_pool_backward": timeit(lambda: H_.bn_pool_backward(dyp, arg, yc, mean, invstd, bn.weight, coef, True,
                                                                    xarg)),
    "layered: + stem_wgrad": timeit(layered),
    "fused: stats only (apply=False)": timeit(lambda: H_.bn_pool_backward(dyp, arg, yc, mean, invstd, bn.weight, coef,
                                                                          True, xarg, apply=False)),
    "fused: + stem_wgrad_bnp": timeit(fused),
}
print("fused vs layered dw rel err %.2e" % ((fused().float() - layered().float()).norm() / layered().float().norm()))
for k, v in t2.items():
    print("%-28s %8.1f us" % (k, v))
