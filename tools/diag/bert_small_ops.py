"""Where do the BERT-base step's small torch ops come from?  (copies, fills, adds, casts: ~35 D2D
copyBuffer + ~43 memsets + ~30 one-block elementwise launches per step in the r5t26 profile.)

Runs the bench.py BERT-base + GNS step (bf16 shadow, AdamW) eagerly under torch.profiler with Python
stacks and prints, per aten op of interest, the count per step grouped by the innermost kungfu_amd /
bench frame that issued it."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import kungfu_amd as kf  # noqa: E402
from kungfu_amd.models import get_model  # noqa: E402
from kungfu_amd.models.bert import pretraining_loss, synthetic_pretraining_batch  # noqa: E402
from kungfu_amd.parallel.mixed import enable_bf16_shadow  # noqa: E402

OPS = {"aten::copy_", "aten::zero_", "aten::fill_", "aten::add_", "aten::add", "aten::clone", "aten::zeros",
       "aten::_to_copy", "aten::sum", "aten::mul", "aten::div", "aten::mul_", "aten::div_", "aten::sub",
       "aten::sqrt", "aten::cat", "aten::stack", "aten::index", "aten::gather", "aten::empty_strided"}


def main():
    kf.init()
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    model = get_model("bert_base").to(dev)
    base = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01)
    opt = kf.optimizers.MonitorGradientNoiseScaleOptimizer(base, device_batch_size=128,
                                                           named_parameters=model.named_parameters())
    kf.broadcast_parameters(model.state_dict())
    enable_bf16_shadow(model, opt)
    data = synthetic_pretraining_batch(128, 128, device=dev)

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = pretraining_loss(model, data)
        loss.backward()
        opt.step()

    for _ in range(4):
        step()
    torch.cuda.synchronize()
    steps = 2
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    tab = collections.Counter()
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        frames = [f for f in (ev.stack or []) if ("kungfu_amd" in f or "bench" in f or "tools/diag" in f)]
        where = frames[0] if frames else "(no python frame)"
        shape = ""
        tab[(ev.name, where.replace(os.getcwd() + "/", ""))] += 1
    rows = sorted(tab.items(), key=lambda kv: -kv[1])
    print("per step: op, count, innermost frame")
    for (name, where), n in rows[:60]:
        print("%-20s %6.1f  %s" % (name, n / steps, where))


if __name__ == "__main__":
    main()
