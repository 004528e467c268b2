"""Which part of the fused engine changes learning on the convergence task of
tests/test_gpu_convergence.py?  Trains ResNet-50 on the 96x96 pattern task for 150 steps in
several configurations and prints the last-50-step mean loss and the eval accuracy of each:
  stock      torch modules + torch.optim.SGD
  ssgd       torch modules + SynchronousSGDOptimizer (flat space, fused SGD)
  shadow     torch modules + SSGD + bf16 shadow weights
  fusedbn    fused_bn model + torch.optim.SGD (HIP BN / fused blocks, no flat space)
  fused_ssgd fused_bn model + SSGD (no shadow)
  engine     fused_bn model + SSGD + bf16 shadow (the bench path)
argv: configurations to run (default all)."""
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
from test_gpu_convergence import _lr, _pattern_dataset  # noqa: E402


def train(cfg, steps=150, batch=64, seed=1234, peak=0.2):
    dev = torch.device("cuda")
    x_all, y_all = _pattern_dataset()
    x_all = x_all.to(dev).to(memory_format=torch.channels_last)
    y_all = y_all.to(dev)
    torch.manual_seed(seed)
    fused = cfg in ("fusedbn", "fused_ssgd", "engine")
    model = resnet50(fused_bn=fused).to(dev).to(memory_format=torch.channels_last)
    base = torch.optim.SGD(model.parameters(), lr=0.0, momentum=0.9, weight_decay=5e-5)
    opt = base
    if cfg in ("ssgd", "shadow", "fused_ssgd", "engine"):
        opt = kf.optimizers.SynchronousSGDOptimizer(base, named_parameters=model.named_parameters())
        if cfg in ("shadow", "engine"):
            from kungfu_amd.parallel.mixed import enable_bf16_shadow

            enable_bf16_shadow(model, opt)
    order = torch.randperm(len(y_all), generator=torch.Generator().manual_seed(77 + seed)).to(dev)
    losses = []
    nb = len(y_all) // batch
    for s in range(steps):
        for gr in opt.param_groups:
            gr["lr"] = _lr(s, steps, peak=peak)
        idx = order[(s % nb) * batch:(s % nb + 1) * batch]
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x_all[idx]).float(), y_all[idx])
        loss.backward()
        opt.step()
        losses.append(loss.item())
    model.eval()
    correct = 0
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for i in range(0, len(y_all), 256):
            correct += int((model(x_all[i:i + 256]).float().argmax(1) == y_all[i:i + 256]).sum())
    return sum(losses[-50:]) / 50, correct / len(y_all), losses


def main():
    kf.init()
    cfgs = sys.argv[1:] or ["stock", "ssgd", "shadow", "fusedbn", "fused_ssgd", "engine"]
    seeds = [int(v) for v in os.environ.get("SEEDS", "1234").split(",")]
    peaks = [float(v) for v in os.environ.get("PEAKS", "0.2").split(",")]
    for peak in peaks:
        for c in cfgs:
            res = []
            for sd in seeds:
                m, acc, ls = train(c, seed=sd, peak=peak)
                res.append((m, acc))
                print("peak %.2f %-11s seed %d last-50 loss %.4f  eval acc %.3f  trajectory %s" % (
                    peak, c, sd, m, acc, [round(v, 2) for v in ls[::15]]), flush=True)
            print("peak %.2f %-11s MEAN last-50 loss %.4f  eval acc %.3f" % (
                peak, c, sum(r[0] for r in res) / len(res), sum(r[1] for r in res) / len(res)), flush=True)


if __name__ == "__main__":
    main()
