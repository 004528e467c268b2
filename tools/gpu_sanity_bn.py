"""GPU numerics of the fused NHWC BN(+add)+ReLU kernels vs a float32 torch reference."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from kungfu_amd.ops.fused_bn import bn_act, available
assert available()
dev = torch.device("cuda")
torch.manual_seed(0)
ok = True
def rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()
for (N, C, H, W) in [(4, 64, 16, 16), (8, 256, 14, 14), (2, 2048, 7, 7), (3, 128, 5, 9)]:
    for relu in [True, False]:
        for with_res in [False, True]:
            x = (torch.randn(N, C, H, W, device=dev) * 2 + 0.5).to(torch.bfloat16).to(memory_format=torch.channels_last)
            res = torch.randn_like(x) if with_res else None
            w = torch.rand(C, device=dev) + 0.5; b = torch.randn(C, device=dev)
            rm = torch.zeros(C, device=dev); rv = torch.ones(C, device=dev)
            rm2, rv2 = rm.clone(), rv.clone()
            xr = x.detach().float().requires_grad_(); wr = w.clone().requires_grad_(); br = b.clone().requires_grad_()
            resr = res.detach().float().requires_grad_() if with_res else None
            yr = F.batch_norm(xr, rm2, rv2, wr, br, True, 0.1, 1e-5)
            if with_res: yr = yr + resr
            if relu: yr = F.relu(yr)
            xa = x.detach().requires_grad_(); wa = w.clone().requires_grad_(); ba = b.clone().requires_grad_()
            resa = res.detach().requires_grad_() if with_res else None
            ya = bn_act(xa, wa, ba, rm, rv, True, 0.1, 1e-5, relu=relu, res=resa)
            g = torch.randn_like(yr)
            yr.backward(g); ya.backward(g.to(torch.bfloat16).to(memory_format=torch.channels_last))
            errs = {"y": rel(ya, yr), "dx": rel(xa.grad, xr.grad), "dw": rel(wa.grad, wr.grad),
                    "db": rel(ba.grad, br.grad), "rm": rel(rm, rm2), "rv": rel(rv, rv2)}
            if with_res: errs["dres"] = rel(resa.grad, resr.grad)
            good = all(v < 3e-2 for v in errs.values())
            ok &= good
            print((N, C, H, W), "relu=%d res=%d" % (relu, with_res), {k: "%.1e" % v for k, v in errs.items()},
                  "OK" if good else "FAIL", flush=True)
print("BN_ALL_OK" if ok else "BN_SOME_FAILED")
sys.exit(0 if ok else 1)
