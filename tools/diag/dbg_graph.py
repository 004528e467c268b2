"""Which part of a ResNet step breaks under hipGraph capture?  For each variant, compare the
gradients of ONE fwd+bwd (same weights, same input) computed eagerly and by graph replay."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import kungfu_amd as kf  # noqa: E402
from kungfu_amd.models import resnet18  # noqa: E402
from kungfu_amd.ops import conv as conv_ops  # noqa: E402

kf.init()
conv_ops.set_enabled(False)
x = torch.randn(8, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (8,), device="cuda")


def grads(m):
    return torch.cat([p.grad.detach().float().flatten() for p in m.parameters() if p.grad is not None])


def run(name, fused_bn, autocast, cl=True, bn_train=True):
    torch.manual_seed(0)
    m = resnet18(fused_bn=fused_bn).cuda()
    if cl:
        m = m.to(memory_format=torch.channels_last)
    m.train(bn_train)
    xx = x if cl else x.contiguous()

    def fb():
        for p in m.parameters():
            p.grad = None if False else p.grad
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            loss = F.cross_entropy(m(xx).float(), y)
        loss.backward()
        return loss

    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    fb()
    torch.cuda.synchronize()
    ge = grads(m)
    for p in m.parameters():
        p.grad.zero_()
    m.load_state_dict(sd)
    fb()
    torch.cuda.synchronize()
    noise = ((grads(m) - ge).norm() / ge.norm()).item()
    # warm + capture
    for p in m.parameters():
        p.grad.zero_()
    m.load_state_dict(sd)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            for p in m.parameters():
                p.grad.zero_()
            m.load_state_dict(sd)
            fb()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    for p in m.parameters():
        p.grad.zero_()
    m.load_state_dict(sd)
    try:
        with torch.cuda.graph(g):
            out = fb()
    except Exception as e:  # noqa: BLE001
        print("%-28s CAPTURE FAILED: %s" % (name, str(e)[:200]), flush=True)
        return
    for p in m.parameters():
        p.grad.zero_()
    m.load_state_dict(sd)
    g.replay()
    torch.cuda.synchronize()
    gg = grads(m)
    rel = ((gg - ge).norm() / ge.norm()).item()
    worst = []
    for (n, p), in zip([(n, p) for n, p in m.named_parameters() if p.grad is not None]):
        pass
    off = 0
    for n, p in m.named_parameters():
        k = p.numel()
        a, b = gg[off:off + k], ge[off:off + k]
        worst.append((((a - b).norm() / (b.norm() + 1e-20)).item(), n))
        off += k
    worst.sort(reverse=True)
    # second replay (grads accumulate: expect 2x)
    g.replay()
    torch.cuda.synchronize()
    rel2 = ((grads(m) - 2 * ge).norm() / (2 * ge).norm()).item()
    print("%-28s eager noise %.3e | grad rel diff replay1 %.3e replay2 %.3e loss %.4f" % (name, noise, rel, rel2, out.item()), flush=True)
    print("    worst:", ", ".join("%s %.2e" % (n, r) for r, n in worst[:6]), flush=True)


run("stock fp32 nchw", False, False, cl=False)
run("stock fp32 cl", False, False)
run("stock autocast cl", False, True)
run("fusedbn autocast cl", True, True)
conv_ops.set_enabled(True)
run("fusedbn autocast cl conv3x3", True, True)
