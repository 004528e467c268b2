import torch, sys
sys.path.insert(0, '.')
from kungfu_amd._lib import hip
H = hip()
T, O = 16384, 3072
u = torch.randn(T, O, device="cuda").bfloat16(); dy = torch.randn(T, O, device="cuda").bfloat16()
def tm(f, n=20):
    for _ in range(3): f()
    torch.cuda.synchronize(); e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True); e0.record()
    for _ in range(n): f()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1) / n * 1e3
print("torch gelu_bwd %.1f us, colsum %.1f us, fused %.1f us" % (tm(lambda: torch.ops.aten.gelu_backward(dy, u)),
      tm(lambda: H.colsum(dy, torch.bfloat16)), tm(lambda: H.gelu_backward_colsum(dy, u, torch.bfloat16))))
