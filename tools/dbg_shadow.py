import torch, torch.nn.functional as F, sys
sys.path.insert(0, "/root/repo")
import kungfu_amd as kf
from kungfu_amd.models import resnet18
from kungfu_amd.parallel.mixed import enable_bf16_shadow
kf.init()
torch.manual_seed(0)
x = torch.randn(8, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (8,), device="cuda")
def run(shadow, seed_model=None):
    torch.manual_seed(0)
    m = resnet18(fused_bn=True).cuda().to(memory_format=torch.channels_last)
    o = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9), named_parameters=m.named_parameters())
    if shadow: enable_bf16_shadow(m, o)
    o.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    o.reducer.synchronize() if o.reducer else None
    torch.cuda.synchronize()
    return o.space, o.space.flat_grad.clone(), loss.item()
sp, g0, l0 = run(False)
_, g0b, _ = run(False)
_, g1, l1 = run(True)
print("loss", l0, l1)
for i, name in enumerate(sp.names):
    o, n = sp.offsets[i]
    a, b, c = g0[o:o+n], g0b[o:o+n], g1[o:o+n]
    r = lambda u, v: ((u-v).abs().max()/(v.abs().max()+1e-12)).item()
    e1, e2 = r(b, a), r(c, a)
    if e2 > 1e-3 or e1 > 1e-3:
        print("%-40s stock-vs-stock %.3g shadow-vs-stock %.3g" % (name, e1, e2))
