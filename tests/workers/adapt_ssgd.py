"""Worker: S-SGD with monitor + adapt on the bucket engine: the bucket
all-reduces feed the strategy statistics (non-zero throughput), then an injected slowdown
(each rank delays alternate buckets, so BOTH peers see their windows stretch) makes the
cluster vote for interference and switch to the alternative star tree, on the same step
everywhere.  argv: cpu | cuda (cuda: run with KUNGFU_GPU_DATAPLANE=host or the RCCL plane)."""
import sys
import time

import torch
import torch.nn.functional as F

import kungfu_amd as kf
from kungfu_amd._lib import runtime

kind = sys.argv[1] if len(sys.argv) > 1 else "cpu"
kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
dev = torch.device("cuda", kf.get_hip_index()) if kind == "cuda" else torch.device("cpu")
if kind == "cuda":
    torch.cuda.set_device(dev)
torch.manual_seed(0)
m = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.ReLU(), torch.nn.Linear(512, 512), torch.nn.ReLU(),
                        torch.nn.Linear(512, 10)).to(dev)
opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.01), flat=True, bucket_mb=0.5,
                                            adapt=True, adapt_warmup=3)
kf.broadcast_parameters(m.state_dict())
assert opt.reducer is not None and opt.reducer.monitored and len(opt.reducer.buckets) >= 2
before = runtime.global_strategy_pairs()
slow = [False]
count = [0]
patched = [False]
for step in range(12):
    if step == 7:
        slow[0] = True
    x = torch.randn(64, 256, device=dev)
    y = torch.randint(0, 10, (64,), device=dev)
    opt.zero_grad()
    F.cross_entropy(m(x), y).backward()
    opt.step()
    if not patched[0]:  # the communicator is bound at the first backward
        comm = opt.reducer.comm
        orig = comm.monitored_all_reduce

        def delayed(t, *a, **k):
            count[0] += 1
            if slow[0] and count[0] % 2 == r:
                time.sleep(0.08)
            return orig(t, *a, **k)

        comm.monitored_all_reduce = delayed
        patched[0] = True
if kind == "cuda":
    torch.cuda.synchronize()
ad = opt.adapter
tps = [t for t in ad.throughputs if t]
assert len(tps) >= 5 and all(t > 0 for t in tps[:6]), ad.throughputs
rccl = opt.reducer.describe()["comm_plane"] == "rccl"
# the vote is collective: every peer switches (or not) at the same step
sw = kf.ops.all_gather(torch.tensor([ad.switched_at or -1], dtype=torch.int64))
assert torch.all(sw == sw[0]), sw
slowed = kf.ops.all_gather(torch.tensor([float(tps[-1] < 0.5 * max(tps[2:6]))]))
if rccl:
    # device-timed windows of ranks that share one GPU: the injected host delay shows
    # on at least one rank (the one whose kernel waits); a majority is not guaranteed
    assert slowed.sum() >= 1, (slowed, ad.throughputs)
else:
    assert ad.changed and ad.switched_at is not None and ad.switched_at > 3, (ad.switched_at, ad.throughputs)
    if kind == "cpu" and ad.switched_at < 8:
        # switched before the injected slowdown: only acceptable when the statistics really showed
        # a slowdown then (a loaded CI machine stalls the host transport too); the vote must have
        # had the evidence it acted on (the vote's own rule: a window below 0.8 x the reference,
        # adaptiveStrategies.go)
        early = [t for t in ad.throughputs[3:ad.switched_at] if t]
        assert early and min(early) < 0.8 * max(tps[:6]), (ad.switched_at, ad.throughputs)
    # the slowdown is visible in the statistics (in some window after it starts: on a loaded CI
    # machine single windows of the slowed phase can be as fast as the noisy warm-up ones)
    late = [t for t in ad.throughputs[7:] if t]
    assert late and min(late) < 0.5 * max(tps[2:6]), ad.throughputs
    after = runtime.global_strategy_pairs()
    assert after != before, (before, after)
print("ADAPT_OK rank=%d switched_at=%s tp_before=%.3g tp_after=%.3g" % (r, ad.switched_at, tps[4], tps[-1]), flush=True)
kf.finalize()
