"""Minimal driver for rocprofv3 --pmc passes: BERT's fc1 / qkv products (16384 tokens) on
gemm_nt (each tile width) and on hipBLASLt (F.linear), a few launches each."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kungfu_amd._lib import hip  # noqa: E402

H = hip()
for name, K, N in (("fc1", 768, 3072), ("qkv", 768, 2304)):
    x = (torch.rand(16384, K, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).bfloat16()
    b = torch.zeros(N, device="cuda").bfloat16()
    for _ in range(5):
        F.linear(x, w, b)
        for bn in (192, 256):
            if N % bn == 0:
                H.gemm_nt(x, w, b, bn=bn)
    torch.cuda.synchronize()
print("done")
