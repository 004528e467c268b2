"""Worker: skewed pair averaging over the HIP-IPC store (SURVEY §5.2 race).  Every model
version is a uniform vector (uniform init, uniform gradient), so any torn read -- part of
one snapshot, part of the next -- leaves a non-uniform model after averaging.  Rank 1
sleeps a random time between steps; rank 0 runs flat out and keeps rewriting its ring."""
import random
import time

import torch

import kungfu_amd as kf

kf.init()
r = kf.current_rank()
dev = torch.device("cuda", kf.get_hip_index())
torch.cuda.set_device(dev)
w = torch.nn.Parameter(torch.full((8 << 20,), float(r + 1), device=dev))
opt = kf.optimizers.PairAveragingOptimizer(torch.optim.SGD([w], lr=1e-3))
rng = random.Random(7 + r)
pulls = 0
for step in range(60):
    opt.zero_grad()
    w.sum().backward()
    opt.step()
    torch.cuda.synchronize()
    lo, hi = float(w.min()), float(w.max())
    assert lo == hi, "torn snapshot at step %d: [%r, %r]" % (step, lo, hi)
    pulls += opt.store.last_pulled is not None
    if r == 1:
        time.sleep(rng.uniform(0, 0.02))
kf.run_barrier()
print("PAIR_STRESS_OK rank=%d dropped=%d value=%.6f" % (r, opt.store.dropped, float(w[0])), flush=True)
kf.finalize()
