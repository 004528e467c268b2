"""Fused attention (attention.hip) at BERT-base shapes: forward and backward kernel time per call
(median of 20, events), batch 128 x seq 128 x 12 heads x 64, dropout p = 0.1 and 0, plus the
HBM bytes each must move (qkv in, out + lse out; backward: qkv, out, dout in, dqkv out) and the
resulting fraction of a 5.3 TB/s streaming roofline.  argv[1] (optional): calls to time."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402


def med(fn, n):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    H = hip()
    B, S, NH = 128, 128, 12
    D = NH * 64
    torch.manual_seed(0)
    qkv = (torch.randn(B, S, 3 * D, device="cuda") * 0.5).bfloat16()
    dout = (torch.randn(B, S, D, device="cuda") * 0.1).bfloat16()
    scale = 64 ** -0.5
    for p in (0.1, 0.0):
        out, lse = H.attention_forward(qkv, NH, scale, 1234, p)
        tf = med(lambda: H.attention_forward(qkv, NH, scale, 1234, p), n)
        tb = med(lambda: H.attention_backward(qkv, out, lse, dout, NH, scale, 1234, p), n)
        fb = qkv.numel() * 2 + out.numel() * 2 + lse.numel() * 4
        bb = qkv.numel() * 2 * 2 + out.numel() * 2 * 2 + lse.numel() * 4
        print("p=%.1f  fwd %6.1f us (%.0f %% of roofline %.1f us)  bwd %6.1f us (%.0f %% of roofline %.1f us)" % (
            p, tf, 100 * fb / 5.3e6 / tf, fb / 5.3e6, tb, 100 * bb / 5.3e6 / tb, bb / 5.3e6), flush=True)


if __name__ == "__main__":
    main()
