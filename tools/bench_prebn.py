"""BN normalise-on-load A/B: is it cheaper to apply a BN(+ReLU) inside the
consuming convolution's A-operand load (conv.hip kEpiPreBN: relu(x*scale+shift) on every A fragment
after its ds_read, padding rows zeroed) than to run the BN apply pass and convolve its output?

For ResNet-50's bottleneck consumers at batch 256 -- conv2 (3x3, stride 1, input = BN1's output) and
conv3 (1x1, input = BN2's output), both with the BN-statistics epilogue they run with in training:

  A  bn_forward(x, sums, apply=True)  -> y ; conv(y, w, stats)           (the current path)
  B  bn_forward(x, sums, apply=False) -> coef ; conv(x, w, stats, pre_coef=coef)

prints us per arm (median of 20, events), the saving, and whether the two outputs are bitwise equal.
Only the forward is compared: the backward of B would also need the transform in the weight-gradient
kernels (their B operand), which this prototype does not have."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

H = hip()
SLOTS = H.conv_stat_slots
CL = torch.channels_last


def timed(fn, reps=20):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def case(name, n, c, hw, cout, ks):
    torch.manual_seed(0)
    x = (torch.randn(n, c, hw, hw, device="cuda") * 2 + 0.5).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(cout, c, ks, ks, device="cuda") / (c * ks * ks) ** 0.5).bfloat16().contiguous(memory_format=CL)
    gamma = torch.rand(c, device="cuda") + 0.5
    beta = torch.randn(c, device="cuda") * 0.2
    rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    xf = x.float()
    sums0 = torch.zeros(SLOTS * 2 * c, dtype=torch.float64, device="cuda")
    sums0[:c] = xf.sum(dim=(0, 2, 3)).double()
    sums0[c:2 * c] = (xf * xf).sum(dim=(0, 2, 3)).double()
    sums = sums0.clone()
    st = torch.zeros(SLOTS * 2 * cout, dtype=torch.float64, device="cuda")

    def bn(apply):
        sums.copy_(sums0)  # the finalize consumes (re-zeroes) the slots
        return H.bn_forward(x, None, gamma, beta, rm, rv, 0.0, 1e-5, True, True, sums=sums, apply=apply)

    def arm_a():
        y = bn(True)[0]
        return H.conv(y, w, 1, st), y

    def arm_b():
        coef = bn(False)[3]
        return H.conv(x, w, 1, st, pre_coef=coef)

    (ya, ybn), yb = arm_a(), arm_b()
    torch.cuda.synchronize()
    same = torch.equal(ya, yb)
    rel = ((ya.float() - yb.float()).norm() / ya.float().norm()).item()
    ta, tb = timed(arm_a), timed(arm_b)
    t_apply = timed(lambda: bn(True)) - timed(lambda: bn(False))
    t_conv = timed(lambda: H.conv(ybn, w, 1, st))
    t_pre = timed(lambda: H.conv(x, w, 1, st, pre_coef=bn(False)[3])) - timed(lambda: bn(False))
    print("%-28s A %7.1f us  B %7.1f us  saving %+6.1f us (%+5.1f %%) | apply pass %6.1f us, conv %6.1f -> %6.1f us "
          "with the on-load BN | outputs bitwise equal: %s (rel %.1e)" % (
              name, ta, tb, ta - tb, 100 * (ta - tb) / ta, t_apply, t_conv, t_pre, same, rel), flush=True)
    return ta, tb


def main():
    shapes = [
        ("layer1 conv3 1x1 64->256", 256, 64, 56, 256, 1),
        ("layer2 conv3 1x1 128->512", 256, 128, 28, 512, 1),
        ("layer3 conv3 1x1 256->1024", 256, 256, 14, 1024, 1),
        ("layer4 conv3 1x1 512->2048", 256, 512, 7, 2048, 1),
        ("layer1 conv2 3x3 64->64", 256, 64, 56, 64, 3),
        ("layer2 conv2 3x3 128->128", 256, 128, 28, 128, 3),
        ("layer3 conv2 3x3 256->256", 256, 256, 14, 256, 3),
        ("layer4 conv2 3x3 512->512", 256, 512, 7, 512, 3),
    ]
    per_block = {"layer1": 3, "layer2": 4, "layer3": 6, "layer4": 3}
    tot_a = tot_b = 0.0
    for s in shapes:
        ta, tb = case(*s)
        k = per_block[s[0].split()[0]]
        tot_a += k * ta
        tb_ = k * tb
        tot_b += tb_
    print("weighted by the blocks per stage (ResNet-50 forward, the stride-1 blocks' shapes): A %.2f ms, B %.2f ms, "
          "saving %+.2f ms/step" % (tot_a / 1e3, tot_b / 1e3, (tot_a - tot_b) / 1e3))


if __name__ == "__main__":
    main()
