"""Elastic training worker: the flat-buffer engines (bucketed S-SGD, gradient-noise-scale
monitor, SMA, AdaSGD) through a resize schedule under ``kungfu-run -w``.

Every rank prints, after every step, the step index, the cluster size it trained
with and a hash of its flat parameter buffer; the test checks that all replicas agree
(and, for S-SGD on CPU, that they equal a single-process simulation of the same
sharded global batch, ``tests/test_elastic_engine.py``).

Data: a fixed global batch per step (seeded by the step), sharded contiguously over
the current peers, so averaged gradients equal the global-batch gradient whatever np is
(parity: tests/python/integration/test_mnist_slp.py's invariance argument).
"""
import argparse
import hashlib
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import kungfu_amd as kf  # noqa: E402
from kungfu_amd.elastic import ElasticTrainer  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--schedule", default="1:3,2:3,1:3")
p.add_argument("--max-step", type=int, default=9)
p.add_argument("--optimizer", default="ssgd", choices=["ssgd", "gns", "sma", "ada"])
p.add_argument("--device", default="cpu")
p.add_argument("--model", default="mlp", choices=["mlp", "resnet18"])
p.add_argument("--global-batch", type=int, default=8)
p.add_argument("--simulate", action="store_true",
               help="single process: replay the schedule, averaging the shards' gradients like the host all-reduce")
a = p.parse_args()


def make_model(kind, device):
    torch.manual_seed(0)
    if kind == "mlp":
        m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    else:
        from kungfu_amd.models import resnet18

        m = resnet18(num_classes=10, fused_bn=True)
    m = m.to(device)
    if device.type == "cuda":
        m = m.to(memory_format=torch.channels_last)
    return m


def batch(kind, step, device):
    g = torch.Generator().manual_seed(1000 + step)
    if kind == "mlp":
        x = torch.randn(a.global_batch, 16, generator=g)
        y = torch.randint(0, 4, (a.global_batch,), generator=g)
    else:
        x = torch.randn(a.global_batch, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (a.global_batch,), generator=g)
    return x.to(device), y.to(device)


def make_optimizer(model, kind, flat):
    base = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    if kind == "ssgd":
        return kf.optimizers.SynchronousSGDOptimizer(base, flat=flat)
    if kind == "gns":
        return kf.optimizers.MonitorGradientNoiseScaleOptimizer(base, device_batch_size=a.global_batch // 2,
                                                                flat=flat)
    if kind == "sma":
        return kf.optimizers.SynchronousAveragingOptimizer(base, flat=flat)
    return kf.optimizers.AdaptiveSGDOptimizer(base, change_step=4, flat=flat)


def digest(t):
    return hashlib.sha1(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()[:16]


def simulate():
    """Single-process reference of the sharded S-SGD run: per step, every shard's gradient
    is computed separately and averaged as the host runtime does (sum, then divide by np)."""
    from kungfu_amd.ops import StepBasedSchedule

    kf.init()
    dev = torch.device(a.device)
    sched = StepBasedSchedule(a.schedule)
    model = make_model(a.model, dev)
    opt = make_optimizer(model, "ssgd", flat=True)
    space = opt.space
    for step in range(a.max_step):
        np_ = sched(step)
        x, y = batch(a.model, step, dev)
        k = a.global_batch // np_
        shards = []
        with opt.reducer.no_sync():
            for r in range(np_):
                opt.zero_grad()
                F.cross_entropy(model(x[r * k:(r + 1) * k]).float(), y[r * k:(r + 1) * k]).backward()
                shards.append(space.flat_grad.clone())
        tot = shards[0]
        for g in shards[1:]:
            tot = tot + g
        space.flat_grad.copy_(tot / np_ if np_ > 1 else tot)
        opt.inner.step()
        print("SIM %d np=%d h=%s" % (step, np_, digest(space.flat_param)), flush=True)


def main():
    if a.simulate:
        return simulate()
    kf.init()
    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(kf.get_hip_index())
    model = make_model(a.model, dev)
    with torch.no_grad():  # only rank 0's initial model may survive the first broadcast
        for q in model.parameters():
            q.add_(0.01 * kf.current_rank())
    opt = make_optimizer(model, a.optimizer, flat=True)
    tr = ElasticTrainer(model, opt, schedule=a.schedule, local_batch_size=1)
    while True:
        tr.before_step()
        if tr.step >= a.max_step:
            break
        np_, r = kf.current_cluster_size(), kf.current_rank()
        x, y = batch(a.model, tr.step, dev)
        k = a.global_batch // np_
        xs, ys = x[r * k:(r + 1) * k], y[r * k:(r + 1) * k]
        if dev.type == "cuda":
            xs = xs.contiguous(memory_format=torch.channels_last) if xs.dim() == 4 else xs
        opt.zero_grad()
        with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=dev.type == "cuda"):
            loss = F.cross_entropy(model(xs).float(), ys)
        loss.backward()
        opt.step()
        extra = ""
        if a.optimizer == "gns" and np_ > 1:
            extra = " gns=%s" % opt.noise_scale
        red = getattr(opt, "reducer", None)
        if red is not None and np_ > 1:
            extra += " plane=%s" % red.describe()["comm_plane"]
        print("STEP %d np=%d rank=%d loss=%.6f h=%s%s" % (tr.step, np_, r, loss.item(), digest(opt.space.flat_param),
                                                         extra), flush=True)
        if tr.after_step():
            break
    if not kf.detached():
        print("ELASTIC_TRAIN_DONE rank=%d np=%d step=%d v=%d rebinds=%d" % (
            kf.current_rank(), kf.current_cluster_size(), tr.step, kf.cluster_version(),
            getattr(getattr(opt, "reducer", None), "rebinds", -1)), flush=True)
    else:
        print("ELASTIC_TRAIN_DETACHED step=%d" % tr.step, flush=True)


if __name__ == "__main__":
    main()
