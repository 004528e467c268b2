"""Stride-2 data gradients of ResNet-50 (batch 256, NHWC bf16): the parity-phase MFMA kernels
(``conv_dgrad_s2``, csrc/kernels/conv.hip) per tile variant (-1 = the default choice), against
MIOpen
(``aten.convolution_backward``, data only).  Prints us per call and the max relative error vs
the float32 torch data gradient."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kungfu_amd._lib import hip

SHAPES = [  # (OH, Cout, Cin, ks): dy [256, Cout, OH, OH] -> dx [256, Cin, 2OH, 2OH]
    (28, 128, 128, 3), (14, 256, 256, 3), (7, 512, 512, 3),
    (28, 512, 256, 1), (14, 1024, 512, 1), (7, 2048, 1024, 1),
]


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
    return e0.elapsed_time(e1) * 1000 / n


def main():
    H = hip()
    N = int(os.environ.get("N", "256"))
    for OH, K, C, ks in SHAPES:
        dy = torch.randn(N, K, OH, OH, device="cuda").bfloat16().to(memory_format=torch.channels_last)
        x = torch.empty(N, C, 2 * OH, 2 * OH, device="cuda", dtype=torch.bfloat16).to(
            memory_format=torch.channels_last)
        w = (torch.randn(K, C, ks, ks, device="cuda") * 0.05).bfloat16().to(memory_format=torch.channels_last)
        pad = (ks - 1) // 2
        ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [2, 2], [pad, pad], [1, 1],
                                                  False, [0, 0], 1, [True, False, False])[0]
        if ks == 1:
            ref = ref[:, :, 0::2, 0::2]
        wt = H.conv_flip_weight(w)
        t_lib = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [pad, pad], [1, 1], False,
                                                                    [0, 0], 1, [True, False, False]))
        row = ["%2d %4d->%4d k%d  miopen %7.1f" % (OH, K, C, ks, t_lib)]
        for v in ([-1, 0, 1, 2, 5]):
            try:
                out = H.conv_dgrad_s2(dy, wt, ks, variant=v)
            except Exception as e:  # noqa: BLE001
                row.append("v%d n/a" % v)
                continue
            o = out if ks == 3 else out[:, :, 0::2, 0::2]
            err = ((o.float() - ref).abs().max() / ref.abs().max()).item()
            t = timeit(lambda: H.conv_dgrad_s2(dy, wt, ks, variant=v))
            row.append("v%d %7.1f%s" % (v, t, "" if err < 1e-2 else " ERR%.3f" % err))
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
