"""Quick GPU numerics check of the HIP kernels against torch f32 references."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import kungfu_amd as kf
from kungfu_amd._lib import hip
H = hip()
dev = torch.device("cuda")
torch.manual_seed(0)
ok = True
def check(name, a, b, tol):
    global ok
    err = (a.float() - b.float()).abs().max().item()
    good = err <= tol
    ok &= good
    print("%-28s max_err=%.3e %s" % (name, err, "OK" if good else "FAIL"), flush=True)
for n in [1, 7, 1000, 1 << 20, (1 << 20) + 3]:
    for dt in [torch.float32, torch.bfloat16]:
        x = torch.randn(n, device=dev).to(dt); y = torch.randn(n, device=dev).to(dt); z = torch.empty_like(x)
        for op, f in [(0, torch.add), (1, torch.minimum), (2, torch.maximum), (3, torch.mul)]:
            H.reduce(z, x, y, op)
            check("reduce n=%d %s op=%d" % (n, dt, op), z, f(x.float(), y.float()).to(dt), 1e-6 if dt == torch.float32 else 2e-2)
n = (1 << 22) + 5
w = torch.randn(n, device=dev); g = torch.randn(n, device=dev); m = torch.randn(n, device=dev)
w0, m0 = w.clone(), m.clone()
H.sgd_step(w, g, m, None, 0.1, None, 0.9, 0.0, 1e-4, 0.5, False, False)
d = g * 0.5 + 1e-4 * w0; mr = 0.9 * m0 + d; wr = w0 - 0.1 * mr
check("sgd momentum", w, wr, 1e-5); check("sgd momentum buf", m, mr, 1e-5)
a = torch.randn(n, device=dev); b = torch.randn(n, device=dev)
s = H.sumsq2(a, b); ref = torch.stack([a.double().pow(2).sum(), b.double().pow(2).sum()]).float(); check("sumsq2 (rel)", s / ref, torch.ones_like(ref), 1e-5)
s1 = torch.randn(n, device=dev); s2 = s1 * s1 + torch.rand(n, device=dev)
v = H.variance(s1, s2, 0.25); ref = (s2.double() * 0.25 - (s1.double() * 0.25) ** 2).abs().sum()
check("variance", v / ref.float(), torch.ones(1, device=dev), 1e-4)
y = torch.randn(n, device=dev); x = torch.randn(n, device=dev); y0 = y.clone(); zz = torch.empty_like(y)
H.axpby(y, x, zz, 0.5, 0.5); check("axpby", y, 0.5 * (y0 + x), 1e-6); check("axpby copy", zz, y, 0)
ts = [torch.randn(k, device=dev) for k in [3, 100, 4097, 1]]
flat = kf.ops.fuse(ts, scale=2.0); check("pack", flat, torch.cat(ts) * 2, 1e-6)
outs = [torch.empty_like(t) for t in ts]; kf.ops.defuse(flat, outs, scale=0.5)
for t, o in zip(ts, outs): check("unpack", o, t, 1e-6)
kf.init()
torch.cuda.set_device(0)
t = torch.arange(1000, device=dev, dtype=torch.float32)
r = kf.ops.all_reduce(t, "sum"); check("rccl all_reduce np=1", r, t, 0)
torch.cuda.synchronize()
print("ALL_OK" if ok else "SOME_FAILED")
sys.exit(0 if ok else 1)
