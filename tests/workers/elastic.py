"""Worker for elastic resize tests (parity: tests/python/integration/test_tensorflow_resize.py):
schedule step -> size; after a change sync the step (all-reduce max) and the model."""
import argparse

import torch

import kungfu_amd as kf
from kungfu_amd import ops
from kungfu_amd.elastic import ElasticTrainer

p = argparse.ArgumentParser()
p.add_argument("--schedule", default="1:3,2:3,3:3,1:3")
p.add_argument("--max-step", type=int, default=12)
a = p.parse_args()

kf.init()
model = torch.nn.Linear(4, 1, bias=False)
with torch.no_grad():
    model.weight.fill_(float(kf.current_rank() + 100))  # only rank 0's value may survive the broadcasts
tr = ElasticTrainer(model, None, schedule=a.schedule)
while True:
    tr.before_step()
    if tr.step >= a.max_step:
        break
    x = ops.all_reduce(torch.ones(3), op="sum")  # the "training" collective
    assert int(x[0]) == kf.current_cluster_size(), (x, kf.current_cluster_size())
    if tr.after_step():
        break
if not kf.detached():
    print("ELASTIC_DONE rank=%d np=%d step=%d w=%.1f v=%d" % (kf.current_rank(), kf.current_cluster_size(), tr.step,
          model.weight[0, 0].item(), kf.cluster_version()), flush=True)
else:
    print("ELASTIC_DETACHED step=%d" % tr.step, flush=True)
