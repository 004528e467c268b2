"""Bucket engine with a parameter used twice per step, the buckets one parameter each
(ADVICE r1): the overlapped engine must equal the non-overlapped all-reduce, also when
the parameter's use count changes between steps.  (The autograd engine sums every use
of a leaf before its AccumulateGrad node runs, so the post-accumulate hook fires once
per backward; only the direct-gradient sink sees one delivery per use, and there a
delivery after the bucket launched raises LateGradientError -- see test_gpu.py.)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import kungfu_amd as kf  # noqa: E402


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(8, 8)
        self.b = torch.nn.Linear(8, 8)
        self.c = torch.nn.Linear(8, 3)

    def forward(self, x, reuse=True):
        h = torch.relu(self.a(x))
        h = torch.relu(self.b(h))
        if reuse:
            h = torch.relu(self.a(h))  # `a` again: its gradient accumulates twice
        return self.c(h)


def run(overlap, steps=4, reuse_from=0):
    torch.manual_seed(0)
    m = Net()
    opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9), flat=True,
                                                overlap=overlap, bucket_mb=1e-4, first_bucket_mb=1e-4)
    if opt.reducer is not None:
        assert len(opt.reducer.buckets) >= 3, len(opt.reducer.buckets)
    g = torch.Generator().manual_seed(kf.current_rank())
    for s in range(steps):
        x = torch.randn(4, 8, generator=g)
        opt.zero_grad()
        m(x, reuse=s >= reuse_from).pow(2).mean().backward()
        opt.step()
    return opt.space.flat_param.clone()


kf.init()
w_ov = run(True)
w_ref = run(False)
assert torch.equal(w_ov, w_ref), (w_ov - w_ref).abs().max()
w_ov = run(True, reuse_from=2)  # learned with one use of `a`, then two
w_ref = run(False, reuse_from=2)
assert torch.equal(w_ov, w_ref), (w_ov - w_ref).abs().max()
print("SHARED_OK rank=%d" % kf.current_rank(), flush=True)
