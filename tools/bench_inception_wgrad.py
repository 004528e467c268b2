"""Inception-v3 weight gradients per conv shape (batch 256, 224x224 input, NHWC bf16): MIOpen
(``aten.convolution_backward``, weight only) vs the split-K MFMA kernels -- ``conv_wgrad`` (the
ResNet planner, 1x1 / 3x3-pad-1 with channels % 64) and ``conv_wgrad_rect`` (any window,
channels % 8) -- with the max relative error vs MIOpen's f32-accumulated result.  The shapes
are captured from one forward of the model's BasicConv2d layers.  Prints one line per
distinct shape (count = occurrences per step) and the weighted totals."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kungfu_amd._lib import hip
from kungfu_amd.models import get_model
from kungfu_amd.models.inception import BasicConv2d


def timeit(f, n=10):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / n


def main():
    H = hip()
    N = int(os.environ.get("N", "256"))
    model = get_model("inception_v3").cuda().to(memory_format=torch.channels_last)
    shapes = {}

    def hook(mod, inp, out):
        c = mod.conv
        x = inp[0]
        key = (int(x.shape[2]), int(x.shape[3]), c.in_channels, c.out_channels, c.kernel_size, c.stride[0], c.padding)
        shapes[key] = shapes.get(key, 0) + 1

    hs = [m.register_forward_hook(hook) for m in model.modules() if isinstance(m, BasicConv2d)]
    with torch.no_grad():
        model(torch.randn(2, 3, 224, 224, device="cuda").to(memory_format=torch.channels_last))
    for h in hs:
        h.remove()
    tot_lib = tot_ours = 0.0
    for (h, w, cin, cout, ks, s, pad), cnt in sorted(shapes.items()):
        if cin % 8:
            continue
        kh, kw = ks
        x = torch.randn(N, cin, h, w, device="cuda").bfloat16().to(memory_format=torch.channels_last)
        wt = torch.randn(cout, cin, kh, kw, device="cuda").bfloat16().to(memory_format=torch.channels_last)
        oh, ow = (h + 2 * pad[0] - kh) // s + 1, (w + 2 * pad[1] - kw) // s + 1
        dy = torch.randn(N, cout, oh, ow, device="cuda").bfloat16().to(memory_format=torch.channels_last)

        def lib():
            return torch.ops.aten.convolution_backward(dy, x, wt, None, [s, s], list(pad), [1, 1], False, [0, 0], 1,
                                                       [False, True, False])[1]

        ref = lib().float()
        t_lib = timeit(lib)
        row = "%3dx%-3d %4d->%4d %dx%d s%d p%d,%d x%d  miopen %7.1f" % (h, w, cin, cout, kh, kw, s, pad[0], pad[1], cnt,
                                                                       t_lib)
        best = t_lib
        if H.conv_wgrad_rect_supported(cin, cout, kh, kw, s) and N * oh * ow < (1 << 23):
            f = lambda: H.conv_wgrad_rect(dy, x, kh, kw, s, pad[0], pad[1])  # noqa: E731
            err = ((f().float() - ref).abs().max() / ref.abs().max()).item()
            t = timeit(f)
            best = min(best, t)
            row += "  rect %7.1f%s" % (t, "" if err < 2e-2 else " ERR%.3f" % err)
        if H.conv_wgrad_rows_rect_supported(N, h, w, cin, cout, kh, kw, pad[0], pad[1], s):
            if s == 1:
                f = lambda: H.conv_wgrad_rect(dy, x, kh, kw, s, pad[0], pad[1], 6)  # noqa: E731
                err = ((f().float() - ref).abs().max() / ref.abs().max()).item()
                t = timeit(f)
                best = min(best, t)
                row += "  rows %7.1f%s" % (t, "" if err < 2e-2 else " ERR%.3f" % err)
            for v in (8, 9, 10, 11, 12):  # the segment-sized ring variants (conv_wgrad.hip kRowsEx)
                f = lambda: H.conv_wgrad_rect(dy, x, kh, kw, s, pad[0], pad[1], v)  # noqa: E731
                err = ((f().float() - ref).abs().max() / ref.abs().max()).item()
                t = timeit(f)
                best = min(best, t)
                row += "  v%d %6.1f%s" % (v, t, "" if err < 2e-2 else " ERR%.3f" % err)
        if kh == kw and pad[0] == pad[1] == (kh - 1) // 2 and H.conv_wgrad_supported(cin, cout, kh, s):
            f = lambda: H.conv_wgrad(dy, x, kh, s)  # noqa: E731
            t = timeit(f)
            best = min(best, t)
            row += "  resnet-planner %7.1f" % t
        tot_lib += cnt * t_lib
        tot_ours += cnt * best
        print(row, flush=True)
    print("weighted total per step: miopen %.1f us, best-of %.1f us" % (tot_lib, tot_ours))


if __name__ == "__main__":
    main()
