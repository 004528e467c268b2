"""Worker: save on 2 peers, then resume on 1 or 3 peers from the same checkpoint (a restart with
a different cluster size) and continue S-SGD identically on every replica."""
import argparse
import hashlib

import torch
import torch.nn.functional as F

import kungfu_amd as kf
from kungfu_amd import checkpoint

p = argparse.ArgumentParser()
p.add_argument("--dir", required=True)
p.add_argument("--phase", choices=["save", "resume"], required=True)
p.add_argument("--kind", choices=["flat", "torch_sgd", "torch_adam"], default="flat",
               help="flat: fused flat-buffer SGD; torch_*: per-tensor torch optimizers (lazily created state)")
a = p.parse_args()

kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
torch.manual_seed(100 + r)  # different initial models on purpose
m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))
if a.kind == "torch_adam":
    base = torch.optim.Adam(m.parameters(), lr=0.01, amsgrad=True)  # amsgrad: never fused
else:
    base = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
opt = kf.optimizers.SynchronousSGDOptimizer(base, flat=a.kind == "flat")


def train(steps, start):
    for s in range(start, start + steps):
        g = torch.Generator().manual_seed(s * 10 + r)
        x, y = torch.randn(4, 8, generator=g), torch.randint(0, 3, (4,), generator=g)
        opt.zero_grad()
        F.cross_entropy(m(x), y).backward()
        opt.step()


def digest():
    if opt.space is not None:
        return hashlib.sha1(opt.space.flat_param.numpy().tobytes()).hexdigest()[:16]
    return hashlib.sha1(torch.cat([q.detach().reshape(-1) for q in m.parameters()]).numpy().tobytes()).hexdigest()[:16]


if a.phase == "save":
    kf.broadcast_parameters(m.state_dict())
    train(3, 0)
    path = checkpoint.save(a.dir + "/ckpt-3.pt", m, opt, step=3, trained_samples=3 * 4 * n,
                           extra={"loader_pos": 17, "sched": torch.arange(3)})
    print("SAVED rank=%d h=%s path=%s" % (r, digest(), path), flush=True)
else:
    path = checkpoint.latest(a.dir)
    meta = checkpoint.load(path, m, opt)
    assert meta["step"] == 3 and meta["cluster_size"] == 2, meta
    if a.kind == "flat":
        assert opt.inner._first is False  # momentum continues, not re-initialised
    else:
        inner = getattr(opt, "inner", opt)
        # every peer (not only rank 0) holds the per-parameter state after the load
        assert len(inner.state) == len(list(m.parameters())), len(inner.state)
    assert meta["extra"]["loader_pos"] == 17 and torch.equal(meta["extra"]["sched"], torch.arange(3)), meta["extra"]
    print("RESUMED rank=%d h=%s" % (r, digest()), flush=True)
    train(2, meta["step"])
    print("AFTER rank=%d h=%s" % (r, digest()), flush=True)
