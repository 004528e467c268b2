"""Worker: SLP convergence regression under S-SGD (parity:
tests/python/integration/test_mnist_slp.py).  Contiguous sharding + gradient
averaging must reproduce single-process training on the global batch, so the
final test accuracy and weights are independent of np.  Uses real MNIST when
KUNGFU_MNIST_DIR holds the idx files, else the deterministic synthetic set."""
import argparse
import hashlib
import sys

import torch
import torch.nn.functional as F

import kungfu_amd as kf
from kungfu_amd.datasets import load_mnist, shard_range, synthetic_mnist
from kungfu_amd.models.slp import SLP

p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, default=500)
p.add_argument("--epochs", type=int, default=2)
p.add_argument("--opt", default="ssgd")
a = p.parse_args()

kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
torch.set_num_threads(1)
data = load_mnist() or synthetic_mnist()
tx, ty = data["train_x"].reshape(-1, 784), data["train_y"]
model = SLP()
base = torch.optim.SGD(model.parameters(), lr=0.1)
if a.opt == "ssgd":
    opt = kf.optimizers.SynchronousSGDOptimizer(base, named_parameters=model.named_parameters())
elif a.opt == "sma":
    opt = kf.optimizers.SynchronousAveragingOptimizer(base, alpha=0.1)
elif a.opt == "pair":
    opt = kf.optimizers.PairAveragingOptimizer(base)
elif a.opt == "pair_rr":
    opt = kf.optimizers.PairAveragingOptimizer(base, peer_selection="roundrobin")
elif a.opt == "ada":
    opt = kf.optimizers.AdaptiveSGDOptimizer(base, change_step=5)
elif a.opt == "gns":
    opt = kf.optimizers.MonitorGradientNoiseScaleOptimizer(base, device_batch_size=a.batch // n)
elif a.opt == "var":
    opt = kf.optimizers.MonitorGradientVarianceOptimizer(base, verbose=False)
kf.broadcast_parameters(model.state_dict())
steps = tx.shape[0] // a.batch
for ep in range(a.epochs):
    for s in range(steps):
        b, e = shard_range(a.batch, r, n)
        xb = tx[s * a.batch + b: s * a.batch + e]
        yb = ty[s * a.batch + b: s * a.batch + e]
        opt.zero_grad()
        loss = F.cross_entropy(model(xb), yb)
        loss.backward()
        opt.step()
# async optimizers (pair averaging) pull from peers' stores at any time: do not let a
# fast peer exit (closing its store) while a slower one may still request from it
kf.run_barrier()
with torch.no_grad():
    acc = (model(data["test_x"].reshape(-1, 784)).argmax(1) == data["test_y"]).float().mean().item()
digest = "%.6e" % model.fc.weight.detach().double().norm().item()
extra = ""
if a.opt == "gns":
    extra = " gns=%s" % opt.noise_scale
if a.opt == "var":
    extra = " var=%s" % opt.variance
print("SLP_RESULT rank=%d np=%d acc=%.4f w=%s%s" % (r, n, acc, digest, extra), flush=True)
kf.finalize()
