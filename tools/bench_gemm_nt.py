"""BERT-base linear-layer products (T tokens) on gemm.hip's pipelined NT GEMM vs hipBLASLt
(``F.linear`` / ``torch.mm``), interleaved rounds in one process; us and TF/s per shape and tile
width, on random data (cdna_hip_programming.md §5.4 rules 24-25)."""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

H = hip()
T = int(os.environ.get("TOKENS", "16384"))
ROUNDS = int(os.environ.get("ROUNDS", "5"))
# (name, K = in-features of the product, N = out-features); forward then data-gradient products
SHAPES = [("qkv", 768, 2304), ("out", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768),
          ("qkv.dg", 2304, 768), ("fc1.dg", 3072, 768), ("fc2.dg", 768, 3072)]
# square reference shapes (steady-state throughput without BERT's short K): (name, M, K, N)
SQUARE = [("sq4k", 4096, 4096, 4096), ("sq8k", 8192, 8192, 8192)]


def timeit(f, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f()
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


tot = {"blas": 0.0, "ours": 0.0}
for name, M, K, N in [(n, T, k, nn) for n, k, nn in SHAPES] + SQUARE:
    T_ = M
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).bfloat16()
    b = (torch.rand(N, device="cuda") * 2 - 1).bfloat16()
    flop = 2.0 * M * K * N
    ref = F.linear(x, w, b).float()
    cands = {"blas": lambda: F.linear(x, w, b)}
    for bn in (128, 192, 256, 1128, 1256):
        if N % (bn % 1000) == 0 and (bn < 1000 or K % 64 == 0):
            err = (H.gemm_nt(x, w, b, bn=bn).float() - ref).abs().max().item()
            if err > 0.1:
                print("%s bn %d: max err %.3f" % (name, bn, err), flush=True)
            cands["bn%d" % bn] = (lambda bn=bn: H.gemm_nt(x, w, b, bn=bn))
    res = {k: [] for k in cands}
    for _ in range(ROUNDS):
        for k, f in cands.items():
            res[k].append(timeit(f))
    med = {k: statistics.median(v) for k, v in res.items()}
    auto = "bn%d" % H.gemm_nt_pick_bn(M, N)
    if not name.startswith("sq"):
        tot["blas"] += med["blas"]
        tot["ours"] += med[auto]
    print("%-7s K %4d N %4d %5.1f GF  " % (name, K, N, flop / 1e9) +
          "  ".join("%s %.1fus %.0fTF" % (k, v, flop / v / 1e6) for k, v in med.items()) + "  (auto %s)" % auto,
          flush=True)
print("sum over the 7 products: hipBLASLt %.1f us, gemm_nt(auto) %.1f us" % (tot["blas"], tot["ours"]), flush=True)
