"""BERT-base MLM head products (2,560 predicted tokens x vocab 30,522 x 768) on hipBLASLt variants
and gemm.hip's NT GEMM, interleaved rounds in one process (random data).  Forward logits,
data gradient, weight gradient and the decoder-bias column sum."""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

H = hip()
M, V, D = int(os.environ.get("ROWS", "2560")), 30522, 768
VP = (V + 127) // 128 * 128
ROUNDS = int(os.environ.get("ROUNDS", "5"))


def timeit(f, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f()
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


h = (torch.rand(M, D, device="cuda") * 2 - 1).bfloat16()
w = ((torch.rand(V, D, device="cuda") * 2 - 1) / D ** 0.5).bfloat16()
b = (torch.rand(V, device="cuda") * 2 - 1).bfloat16()
wp = torch.zeros(VP, D, device="cuda", dtype=torch.bfloat16)
wp[:V] = w
bp = torch.zeros(VP, device="cuda", dtype=torch.bfloat16)
bp[:V] = b
dl = ((torch.rand(M, V, device="cuda") * 2 - 1) * 1e-3).bfloat16()
dlp = torch.zeros(M, VP, device="cuda", dtype=torch.bfloat16)
dlp[:, :V] = dl
flop = 2.0 * M * V * D

cands = {
    "fwd blas bias": lambda: F.linear(h, w, b),
    "fwd blas nobias": lambda: torch.mm(h, w.t()),
    "fwd blas padded": lambda: F.linear(h, wp, bp),
    "dgrad blas": lambda: torch.mm(dl, w),
    "dgrad blas padded": lambda: torch.mm(dlp, wp),
    "wgrad blas": lambda: torch.mm(dl.t(), h),
    "wgrad blas padded": lambda: torch.mm(dlp.t(), h),
    "bias colsum torch": lambda: dl.sum(0),
    "bias colsum ours (padded)": lambda: H.colsum(dlp, torch.float32),
}
for bn in (128,):
    cands["fwd ours padded bn%d" % bn] = (lambda bn=bn: H.gemm_nt(h, wp, bp, bn=bn))
for bn in (128, 192, 256):
    cands["fwd ours ragged bn%d" % bn] = (lambda bn=bn: H.gemm_nt_ld(h, w, b, 0, bn))
    err = (H.gemm_nt_ld(h, w, b, 0, bn)[:, :V].float() - F.linear(h, w, b).float()).abs().max().item()
    print("ours ragged bn%d max err %.4f" % (bn, err), flush=True)
slot = torch.zeros(V, D, device="cuda")
try:
    torch.addmm(slot, dl.t(), h, out_dtype=torch.float32, out=slot)
    cands["wgrad blas f32 accumulate"] = lambda: torch.addmm(slot, dl.t(), h, out_dtype=torch.float32, out=slot)
except Exception as e:  # noqa: BLE001
    print("addmm out_dtype:", e, flush=True)
outp = torch.empty(M, (V + 7) // 8 * 8, device="cuda", dtype=torch.bfloat16)
outv = outp[:, :V]
cands["fwd blas out=padded view"] = lambda: torch.addmm(b, h, w.t(), out=outv)
torch.addmm(b, h, w.t(), out=outv)
print("blas padded-view max err %.4f" % (outv.float() - F.linear(h, w, b).float()).abs().max().item(), flush=True)
gs = torch.zeros(V, D, device="cuda")
torch.addmm(gs, dl.t(), h, out_dtype=torch.float32, out=gs)
torch.addmm(gs, dl.t(), h, out_dtype=torch.float32, out=gs)
print("f32 accumulate rel err %.2e" % ((gs - 2 * (dl.float().t() @ h.float())).norm() / gs.norm()).item(), flush=True)
ref_dh = (dlp[:, :V].float() @ w.float())
for S in (2, 3, 6):
    Kc = V // S
    A = dlp.as_strided((S, M, Kc), (Kc, dlp.stride(0), 1))
    B = w.as_strided((S, Kc, D), (Kc * D, D, 1))
    cands["dgrad split-K bmm S=%d bf16" % S] = (lambda A=A, B=B: torch.bmm(A, B).sum(0))
    try:
        r = torch.bmm(A, B, out_dtype=torch.float32).sum(0)
        print("split S=%d f32 rel err %.2e" % (S, ((r - ref_dh).norm() / ref_dh.norm()).item()), flush=True)
        cands["dgrad split-K bmm S=%d f32" % S] = (lambda A=A, B=B: torch.bmm(A, B, out_dtype=torch.float32).sum(0))
    except Exception as e:  # noqa: BLE001
        print("bmm out_dtype:", str(e)[:200], flush=True)
dlT = dl.t().contiguous()  # [V, M]: a transposed cross-entropy gradient
cands["dgrad blas from dlT (mm(dlT^T, W))"] = lambda: torch.mm(dlT.t(), w)
cands["dgrad blas W^T dlT -> dh^T"] = lambda: torch.mm(w.t(), dlT)
cands["wgrad blas from dlT (mm(dlT, h))"] = lambda: torch.mm(dlT, h)
gs2 = torch.zeros(V, D, device="cuda")
cands["wgrad f32 acc from dlT"] = lambda: torch.addmm(gs2, dlT, h, out_dtype=torch.float32, out=gs2)
dlv = dlp[:, :V]
cands["dgrad blas (padded view)"] = lambda: torch.mm(dlv, w)
cands["wgrad blas (padded view)"] = lambda: torch.mm(dlv.t(), h)
lab = torch.randint(0, V, (M,), device="cuda")
lg = H.gemm_nt_ld(h, w, b, 0, 256)[:, :V]
lgc = lg.contiguous()
cands["xent fwd padded"] = lambda: H.xent_forward(lg, lab)
cands["xent fwd contiguous"] = lambda: H.xent_forward(lgc, lab)
lse = H.xent_forward(lg, lab)[0]
sc = torch.ones(1, device="cuda")
cands["xent bwd padded"] = lambda: H.xent_backward(lg, lab, lse, sc)
cands["xent bwd contiguous"] = lambda: H.xent_backward(lgc, lab, lse, sc)
ref = F.linear(h, w, b).float()
for bn in (128,):
    err = (H.gemm_nt(h, wp, bp, bn=bn)[:, :V].float() - ref).abs().max().item()
    print("ours bn%d max err %.4f" % (bn, err), flush=True)
res = {k: [] for k in cands}
for _ in range(ROUNDS):
    for k, f in cands.items():
        res[k].append(timeit(f))
for k, v in res.items():
    t = statistics.median(v)
    print("%-24s %7.1f us  %6.0f TF/s" % (k, t, flop / t / 1e6 if "colsum" not in k else 0), flush=True)
