"""Per-layer gradient numerics of the fused ResNet-50 engine against a stock f32 reference
(VERDICT r4 "Next round" #1b), and which engine component moves the lr-0.1 trajectory.

Two phases, one process each (the component knobs are read at import time):

  python tools/diag/engine_numerics.py ref  DIR
      Stock modules.  Seeds the model, saves state S0; runs 3 stock-bf16 SGD steps at lr 0.1 on the
      fixed batch and saves state S3.  At each state: the stock-f32 gradient (autocast off) and two
      stock-bf16 (autocast) gradients; saves the f32 gradient and the per-layer bf16-vs-f32 error
      envelope (relative L2 error, cosine) to DIR.  Prints the stock lr-0.1 trajectory.

  python tools/diag/engine_numerics.py chaos DIR
      How much the lr-0.1 trajectory amplifies a minimal perturbation, with stock modules only: the
      stock-f32 trajectory, and stock-bf16 trajectories from S0 with 1 % of the conv / fc weights
      moved by one bf16 ulp (three draws).

  python tools/diag/engine_numerics.py var  DIR TAG [--no-shadow] [--stock-modules]
      The engine (fused_bn model + S-SGD + bf16 shadow unless told otherwise) under whatever
      KUNGFU_* environment the caller set, loaded from S0 / S3: per-layer relative error and cosine
      of its gradient vs the f32 reference, as a multiple of the stock-bf16 envelope; the worst
      layers; then its own lr-0.1 trajectory from S0.

Batch: 64 x 3 x 224 x 224, the seed-99 batch of tests/test_gpu_engine.py."""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import kungfu_amd as kf  # noqa: E402
from kungfu_amd.models import resnet50  # noqa: E402

BATCH = 64


def batch():
    g = torch.Generator(device="cuda").manual_seed(99)
    x = torch.randn(BATCH, 3, 224, 224, device="cuda", generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (BATCH,), device="cuda", generator=g)
    return x, y


def stock_model(state=None):
    torch.manual_seed(1234)
    m = resnet50(fused_bn=False).cuda().to(memory_format=torch.channels_last)
    if state is not None:
        m.load_state_dict(state)
    return m


def stock_grads(state, x, y, amp):
    m = stock_model(state)
    m.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    return loss.item(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}


def layer_err(ref, got):
    """name -> (relative L2 error, cosine) of got vs ref."""
    out = {}
    for n, a in ref.items():
        b = got[n].reshape(a.shape)
        rel = ((b - a).norm() / a.norm().clamp_min(1e-30)).item()
        cos = F.cosine_similarity(a.flatten().double(), b.flatten().double(), 0).item()
        out[n] = (rel, cos)
    return out


def overall(ref, got):
    a = torch.cat([v.flatten() for v in ref.values()])
    b = torch.cat([got[n].flatten() for n in ref])
    return ((b - a).norm() / a.norm()).item(), F.cosine_similarity(a.double(), b.double(), 0).item()


def trajectory(make, steps=5, lr=0.1):
    """(model, optimizer) from make(); losses of `steps` SGD steps on the fixed batch."""
    x, y = batch()
    m, opt = make(lr)
    out = []
    for _ in range(steps):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        opt.step()
        out.append(round(loss.item(), 4))
    return out


def phase_ref(d):
    os.makedirs(d, exist_ok=True)
    x, y = batch()
    m = stock_model()
    s0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    torch.save(s0, os.path.join(d, "S0.pt"))
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    for _ in range(3):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            F.cross_entropy(m(x).float(), y).backward()
        opt.step()
    torch.save({k: v.detach().clone() for k, v in m.state_dict().items()}, os.path.join(d, "S3.pt"))
    env = {}
    for tag in ("S0", "S3"):
        st = torch.load(os.path.join(d, tag + ".pt"), weights_only=True)
        lf, gf = stock_grads(st, x, y, amp=False)
        la, ga = stock_grads(st, x, y, amp=True)
        lb, gb = stock_grads(st, x, y, amp=True)
        torch.save(gf, os.path.join(d, "gref_%s.pt" % tag))
        ea, eb = layer_err(gf, ga), layer_err(gf, gb)
        env[tag] = {"loss_f32": lf, "loss_bf16": [la, lb],
                    "layers": {n: [max(ea[n][0], eb[n][0]), min(ea[n][1], eb[n][1])] for n in gf},
                    "overall_bf16": [overall(gf, ga), overall(gf, gb)],
                    "bf16_vs_bf16": overall(ga, gb)}
        print("%s loss f32 %.5f bf16 %.5f / %.5f; overall bf16 vs f32 %s; bf16 vs bf16 %s" % (
            tag, lf, la, lb, env[tag]["overall_bf16"], env[tag]["bf16_vs_bf16"]), flush=True)
    with open(os.path.join(d, "envelope.json"), "w") as f:
        json.dump(env, f)

    def make_stock(lr):
        mm = stock_model(s0)
        return mm, torch.optim.SGD(mm.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)

    print("TRAJ stock   ", trajectory(make_stock), flush=True)
    print("TRAJ stock   ", trajectory(make_stock), flush=True)


def phase_chaos(d):
    s0 = torch.load(os.path.join(d, "S0.pt"), weights_only=True)

    def make(lr, state=s0):
        mm = stock_model(state)
        return mm, torch.optim.SGD(mm.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)

    x, y = batch()
    m, opt = make(0.1)
    out = []
    for _ in range(5):  # f32: no autocast
        opt.zero_grad()
        loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        opt.step()
        out.append(round(loss.item(), 4))
    print("TRAJ stock-f32  ", out, flush=True)
    for draw in range(3):
        g = torch.Generator().manual_seed(1000 + draw)
        st = {}
        for k, v in s0.items():
            if v.dim() in (2, 4) and v.is_floating_point():  # conv / fc weights
                pick = (torch.rand(v.shape, generator=g) < 0.01).to(v.device)
                ulp = v.abs().clamp_min(1e-30) * 2.0 ** -7  # one bf16 ulp (8 significant bits)
                sign = torch.where(torch.rand(v.shape, generator=g) < 0.5, -1.0, 1.0).to(v.device)
                st[k] = torch.where(pick, v + sign * ulp, v)
            else:
                st[k] = v
        print("TRAJ stock-ulp%d  " % draw, trajectory(lambda lr: make(lr, st)), flush=True)


def phase_var(d, tag, shadow=True, fused=True):
    from kungfu_amd.parallel.mixed import enable_bf16_shadow

    x, y = batch()
    env = json.load(open(os.path.join(d, "envelope.json")))

    def make(state, lr):
        torch.manual_seed(1234)
        m = resnet50(fused_bn=fused).cuda().to(memory_format=torch.channels_last)
        m.load_state_dict(state)
        opt = kf.optimizers.SynchronousSGDOptimizer(
            torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4),
            named_parameters=m.named_parameters())
        if shadow:
            enable_bf16_shadow(m, opt)
        return m, opt

    res = {"tag": tag, "env": {k: v for k, v in os.environ.items() if k.startswith("KUNGFU_")}}
    for st in ("S0", "S3"):
        state = torch.load(os.path.join(d, st + ".pt"), weights_only=True)
        gref = torch.load(os.path.join(d, "gref_%s.pt" % st), weights_only=True)
        m, opt = make(state, 0.0)
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        opt.reducer.synchronize()
        g = {n: opt.space.grad_view(i).detach().float().clone() for i, n in enumerate(opt.space.names)}
        e = layer_err(gref, g)
        envl = env[st]["layers"]
        rows = []
        for n, (rel, cos) in e.items():
            erel, ecos = envl[n]
            rows.append((rel / max(erel, 1e-12), n, rel, erel, cos, ecos))
        rows.sort(key=lambda r: -r[0])
        orel, ocos = overall(gref, g)
        print("== %s %s loss %.5f (f32 %.5f, bf16 %s)  overall rel %.4f cos %.6f  (bf16 envelope %s)" % (
            tag, st, loss.item(), env[st]["loss_f32"], env[st]["loss_bf16"], orel, ocos,
            env[st]["overall_bf16"]), flush=True)
        for ratio, n, rel, erel, cos, ecos in rows[:12]:
            print("  %-34s rel %.4f  env %.4f  x%.2f   cos %.5f env %.5f" % (n, rel, erel, ratio, cos, ecos))
        over = [r for r in rows if r[0] > 2.0]
        print("  layers > 2x envelope: %d of %d; > 4x: %d" % (len(over), len(rows), sum(r[0] > 4 for r in rows)))
        res[st] = {"loss": loss.item(), "overall": [orel, ocos], "worst": rows[:12],
                   "n_over2": len(over), "n_over4": sum(r[0] > 4 for r in rows)}
        del m, opt
    s0 = torch.load(os.path.join(d, "S0.pt"), weights_only=True)
    res["traj"] = trajectory(lambda lr: make(s0, lr))
    print("TRAJ %-8s" % tag, res["traj"], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "numerics_%s.json" % tag), "w") as f:
        json.dump(res, f)


def main():
    kf.init()
    if sys.argv[1] == "ref":
        phase_ref(sys.argv[2])
    elif sys.argv[1] == "chaos":
        phase_chaos(sys.argv[2])
    else:
        phase_var(sys.argv[2], sys.argv[3], shadow="--no-shadow" not in sys.argv,
                  fused="--stock-modules" not in sys.argv)


if __name__ == "__main__":
    main()
