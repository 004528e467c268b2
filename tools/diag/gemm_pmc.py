"""Minimal driver for rocprofv3 --pmc passes over BERT-base's linear-layer GEMMs (16,384 tokens):
shape SHAPE (argv[1]: 0 qkv 768->2304, 1 out 768->768, 2 fc1 768->3072, 3 fc2 3072->768), its forward
y = x W^T and data gradient dx = dy W, each 5 times on hipBLASLt (F.linear / torch.mm) and 5 times on
the hand-written NT GEMM (gemm.hip, auto tile; W^T precomputed for the data gradient), in that order
(tools/runs/gpu_r5_pmc.sh splits the dispatches by kernel name and order)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kungfu_amd._lib import hip  # noqa: E402

SHAPES = [("qkv", 768, 2304), ("out", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)]
H = hip()
name, K, N = SHAPES[int(sys.argv[1]) if len(sys.argv) > 1 else 0]
T = 16384
x = (torch.rand(T, K, device="cuda") * 2 - 1).bfloat16()
w = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).bfloat16()
dy = (torch.rand(T, N, device="cuda") * 2 - 1).bfloat16()
wt = w.t().contiguous()  # [K, N]: dx = dy . W = dy . (W^T)^T
for _ in range(5):
    F.linear(x, w)
for _ in range(5):
    torch.mm(dy, w)
for _ in range(5):
    H.gemm_nt(x, w)
for _ in range(5):
    H.gemm_nt(dy, wt)
torch.cuda.synchronize()
print("done", name)
