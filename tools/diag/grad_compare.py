"""Where does the fused ResNet-50 engine's gradient differ from stock PyTorch?  One forward +
backward from identical weights on the same batch (bf16 autocast both), per-parameter relative
error of the engine's flat gradient vs the stock model's .grad, worst first; for the learnable
96x96 pattern task of tests/test_gpu_convergence.py and for a random 224x224 batch."""
import math
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import kungfu_amd as kf  # noqa: E402
from kungfu_amd.models import resnet50  # noqa: E402
from kungfu_amd.parallel.mixed import enable_bf16_shadow  # noqa: E402


def grads(engine, x, y, steps=1, lr=0.0, amp=True):
    torch.manual_seed(1234)
    m = resnet50(fused_bn=engine).cuda().to(memory_format=torch.channels_last)
    names = [n for n, _ in m.named_parameters()]
    base = torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9)
    if engine:
        opt = kf.optimizers.SynchronousSGDOptimizer(base, named_parameters=m.named_parameters())
        enable_bf16_shadow(m, opt)
    else:
        opt = base
    losses = []
    for _ in range(steps):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        if engine:
            opt.reducer.synchronize()
            g = {n: opt.space.grad_view(i).detach().float().clone() for i, n in enumerate(opt.space.names)}
        else:
            g = {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}
        losses.append(loss.item())
        opt.step()
    return losses, g, names


def cos_all(ga, gb, names):
    a = torch.cat([ga[n].flatten() for n in names])
    b = torch.cat([gb[n].flatten() for n in names])
    return F.cosine_similarity(a, b, 0).item(), ((b - a).norm() / a.norm()).item()


def compare(tag, x, y):
    lf, gf, names = grads(False, x, y, amp=False)
    ls, gs, names = grads(False, x, y)
    ls2, gs2, _ = grads(False, x, y)
    le, ge, _ = grads(True, x, y)
    print("== %s: loss stock-f32 %.5f stock-bf16 %.5f engine %.5f" % (tag, lf[0], ls[0], le[0]))
    for na, ga, nb, gb in (("stock-f32", gf, "stock-bf16", gs), ("stock-bf16", gs, "stock-bf16 again", gs2),
                           ("stock-f32", gf, "engine", ge), ("stock-bf16", gs, "engine", ge)):
        c, r = cos_all(ga, gb, names)
        print("  %-12s vs %-16s: cos %.5f rel %.4f" % (na, nb, c, r))
    # per-layer view against the f32 reference, the first 12 parameters in model order
    for n in names[:12]:
        a, b, c = gf[n].flatten(), gs[n].flatten(), ge[n].flatten()
        print("  %-32s cos(f32, bf16) %.4f  cos(f32, engine) %.4f" % (
            n, F.cosine_similarity(a, b, 0).item(), F.cosine_similarity(a, c, 0).item()))
    rows = []
    for n in names:
        a, b = gs[n], ge.get(n)
        if b is None:
            rows.append((float("inf"), n, "missing in engine"))
            continue
        b = b.view_as(a) if b.numel() == a.numel() else b
        if b.shape != a.shape:
            b = b.reshape(a.shape)
        rel = ((b - a).norm() / a.norm().clamp_min(1e-20)).item()
        rows.append((rel, n, "norm stock %.3e engine %.3e cos %.5f" % (a.norm().item(), b.norm().item(),
                                                                       F.cosine_similarity(a.flatten(), b.flatten(), 0).item())))
    rows.sort(key=lambda r: -r[0])
    for rel, n, info in rows[:25]:
        print("  %-40s rel %.4f  %s" % (n, rel, info))
    tot_a = torch.cat([gs[n].flatten() for n in names])
    tot_b = torch.cat([ge[n].flatten() for n in names])
    print("  overall rel %.4f" % ((tot_b - tot_a).norm() / tot_a.norm()).item())


def main():
    kf.init()
    from test_gpu_convergence import _pattern_dataset

    xa, ya = _pattern_dataset()
    x = xa[:64].cuda().to(memory_format=torch.channels_last)
    y = ya[:64].cuda()
    compare("pattern 96x96 batch 64", x, y)
    g = torch.Generator(device="cuda").manual_seed(3)
    x2 = torch.randn(64, 3, 224, 224, device="cuda", generator=g).to(memory_format=torch.channels_last)
    y2 = torch.randint(0, 1000, (64,), device="cuda", generator=g)
    compare("random 224x224 batch 64", x2, y2)
    x3 = torch.nn.functional.interpolate(x, size=(224, 224), mode="bilinear").contiguous(memory_format=torch.channels_last)
    compare("pattern upsampled 224x224 batch 64", x3, y)


if __name__ == "__main__":
    main()
