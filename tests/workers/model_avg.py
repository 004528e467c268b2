"""Worker: legacy fused-model pair averaging ops (save / request / sync + prefetching average).

Parity: srcs/cpp/src/tensorflow/ops/cpu/peer_to_peer.cpp (ModelAveraging, AsyncModelAveraging,
SaveModel, RequestModel) with random / roundrobin peer selection.
"""
import torch

import kungfu_amd as kf
from kungfu_amd import ops

kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
ts = [torch.full((1000,), float(r)), torch.full((3, 7), float(r))]
for sel in ["random", "roundrobin"]:
    m = ops.ModelAveraging(ts, peer_selection=sel, name="m-" + sel)
    m.save()
    kf.run_barrier()
    got = m.request()
    assert got is not None and m.last_peer != r
    assert torch.equal(got[0], torch.full((1000,), float(m.last_peer)))
    assert got[1].shape == (3, 7)
    before = [t.clone() for t in ts]
    p = m()
    assert p >= 0 and p != r
    for t, b in zip(ts, before):
        assert torch.equal(t, (b + float(p)) / 2)
    kf.run_barrier()
    for t in ts:
        t.fill_(float(r))

# prefetching variant: the first call pulls synchronously, later ones use the last pull
a = ops.async_model_averaging(ts, "roundrobin", name="m-async")
a.save()
kf.run_barrier()
for _ in range(3):
    p = a()
    assert p >= 0 and p != r
a.wait()
assert a.engine.pulls() >= 2  # one synchronous pull + >= 1 background prefetch
kf.run_barrier()
print("MODEL_AVG_OK", r)
