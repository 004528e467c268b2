"""ops.linear on gemm.hip (set_gemm_enabled) vs hipBLASLt on a 2-layer BERT: per-step loss and the
flat-gradient relative difference per parameter (the largest ones), to tell a broken GEMM path from
trajectory sensitivity.  Usage: python tools/diag/linear_gemm_ab.py [--lr 1e-4] [--steps 2]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import kungfu_amd as kf  # noqa: E402
from kungfu_amd.models.bert import BertForPreTraining, pretraining_loss, synthetic_pretraining_batch  # noqa: E402
from kungfu_amd.ops import linear as lin  # noqa: E402
from kungfu_amd.parallel.mixed import enable_bf16_shadow  # noqa: E402


def run(on, lr, steps):
    old = lin.set_gemm_enabled(on)
    try:
        torch.manual_seed(0)
        m = BertForPreTraining(layers=2).cuda()
        for l in m.layers:
            l.dropout = 0.0
        opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.AdamW(m.parameters(), lr=lr),
                                                    named_parameters=m.named_parameters())
        enable_bf16_shadow(m, opt)
        g = torch.Generator(device="cuda").manual_seed(1)
        batch = synthetic_pretraining_batch(16, 128, device="cuda", generator=g)
        out = []
        for _ in range(steps):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = pretraining_loss(m, batch)
            loss.backward()
            opt.reducer.synchronize()
            out.append((loss.item(), {n: opt.space.grad_view(i).clone() for i, n in enumerate(opt.space.names)}
                        if hasattr(opt.space, "names") else opt.space.flat_grad.clone()))
            opt.step()
        torch.cuda.synchronize()
        return out, opt
    finally:
        lin.set_gemm_enabled(old)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    kf.init()
    ra, opt = run(False, a.lr, a.steps)
    rb, _ = run(True, a.lr, a.steps)
    names = [n for n, _ in opt.named_parameters] if hasattr(opt, "named_parameters") else None
    for s, ((la, ga), (lb, gb)) in enumerate(zip(ra, rb)):
        if isinstance(ga, dict):
            rel = {n: ((gb[n] - ga[n]).norm() / ga[n].norm().clamp_min(1e-30)).item() for n in ga}
            tot = sum((gb[n] - ga[n]).double().norm() ** 2 for n in ga) ** 0.5 / sum(ga[n].double().norm() ** 2 for n in ga) ** 0.5
        else:
            rel, tot = {}, ((gb - ga).norm() / ga.norm()).item()
        print("step %d: loss %.6f vs %.6f  flat grad rel %.4f" % (s, la, lb, float(tot)))
        for n, v in sorted(rel.items(), key=lambda kv: -kv[1])[:8]:
            print("    %-50s %.4f" % (n, v))
    print("names available:", names is not None)


if __name__ == "__main__":
    main()
