"""Is a model's S-SGD step reproducible, eager and under whole-step capture?  Runs the bench engine
(fused kernels, bf16 shadow weights, 1-rank RCCL buckets) for STEPS steps from one seed, twice eagerly
and twice through GraphedStep, and prints the losses and the first step at which two runs differ.

  python tools/diag/capture_repro.py MODEL [BATCH] [SIZE]
  env: STEPS (8), LR (0.01), DETERMINISTIC=1 (torch.backends.cudnn.deterministic: MIOpen's
       deterministic solvers), NODROP=1 (dropout p = 0)."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(ROOT, "kungfu_amd", "tuning", "miopen"))
import kungfu_amd as kf  # noqa: E402
from kungfu_amd.models import get_model  # noqa: E402
from kungfu_amd.parallel.graphs import GraphedStep  # noqa: E402
from kungfu_amd.parallel.mixed import enable_bf16_shadow  # noqa: E402


def run(name, batch, size, graph, steps, lr):
    torch.manual_seed(1234)
    m = get_model(name, fused_bn=True).cuda().to(memory_format=torch.channels_last)
    if os.environ.get("NODROP") == "1":
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
    opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9,
                                                                weight_decay=1e-4),
                                                named_parameters=m.named_parameters(), force_comm=True)
    enable_bf16_shadow(m, opt)
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(batch, 3, size, size, device="cuda", generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device="cuda", generator=g)

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        opt.step()
        return loss

    fn = GraphedStep(step, opt, warmup=3) if graph else step
    out = [float(fn().detach()) for _ in range(steps)]
    torch.cuda.synchronize()
    return out, opt.space.flat_param.clone()


def first_diff(a, b):
    for i, (u, v) in enumerate(zip(a, b)):
        if u != v:
            return i
    return None


def main():
    name = sys.argv[1]
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 224
    steps, lr = int(os.environ.get("STEPS", "8")), float(os.environ.get("LR", "0.01"))
    kf.init()
    if os.environ.get("DETERMINISTIC") == "1":
        torch.backends.cudnn.deterministic = True
    runs = {}
    for tag, graph in (("eager1", False), ("eager2", False), ("graph1", True), ("graph2", True)):
        runs[tag] = run(name, batch, size, graph, steps, lr)
        print("%-7s %s" % (tag, runs[tag][0]), flush=True)
    base = runs["eager1"]
    for tag in ("eager2", "graph1", "graph2"):
        d = first_diff(base[0], runs[tag][0])
        print("%s vs eager1: first differing loss at step %s; weights identical: %s" % (
            tag, d, torch.equal(base[1], runs[tag][1])), flush=True)
    kf.finalize()


if __name__ == "__main__":
    main()
