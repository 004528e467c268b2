"""SynchronousSGDOptimizer (S-SGD): average gradients across all peers, then apply.

Parity: ``srcs/python/kungfu/tensorflow/optimizers/sync_sgd.py:15-109``
(``nccl``, ``nccl_fusion``, ``hierarchical_nccl``, ``monitor`` options) and
the torch wrapper ``srcs/python/kungfu/torch/optimizers/sync_sgd.py:6-32``.

Data planes:
* GPU (default): bucketed in-place RCCL all-reduce of the flat gradient
  buffer, launched from backward hooks on a comm stream (overlapped with
  backward), op ``avg``.  ``hierarchical=True`` uses local-reduce ->
  cross-host host all-reduce -> local-broadcast instead (reference's
  hierarchical NCCL path, ``ops/gpu/collective.cpp:105-156``).
* CPU tensors: the C++ host runtime's graph all-reduce (TCP/UDS) with the
  chosen strategy; async per tensor, then wait all.

Unlike the reference torch wrapper (which sums, ``torch/optimizers/sync_sgd.py:29-32``),
gradients are averaged unless ``op='sum'``.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import ops
from ..parallel.ddp import GradReducer
from .core import KungFuOptimizer


class _SynchronousSGD(KungFuOptimizer):
    def __init__(self, optimizer, named_parameters=None, op: str = "avg", fused: bool = True,
                 bucket_mb: Optional[float] = None, comm_dtype: Optional[torch.dtype] = None,
                 hierarchical: bool = False, monitor: bool = False, overlap: bool = True,
                 force_comm: bool = False, flat=None, first_bucket_mb: float = 1.0):
        super().__init__(optimizer, named_parameters, fused=fused, flat=flat)
        self.op = op
        self.monitor = monitor
        self.hierarchical = hierarchical
        self.reducer: Optional[GradReducer] = None
        if self.space is not None and not hierarchical and overlap:
            self.reducer = GradReducer(self.space, op="avg" if op == "avg" else "sum", bucket_mb=bucket_mb,
                                       comm_dtype=comm_dtype, skip_single=not force_comm,
                                       first_bucket_mb=first_bucket_mb)

    def _before_step(self):
        if self.reducer is not None:
            self.reducer.synchronize()
            return
        self.sync_gradients()

    def sync_gradients(self):
        if self.space is not None:
            g = self.space.flat_grad
            if self.hierarchical:
                ops.hierarchical_all_reduce_(g, op="sum")
                if self.op == "avg":
                    g.mul_(1.0 / ops.cluster_size())
            else:
                ops.inplace_all_reduce_op(g, op=self.op)
            return
        grads = [p.grad for p in self.params if p.grad is not None]
        names = [self.names.get(id(p), "grad%d" % i) for i, p in enumerate(self.params) if p.grad is not None]
        if self.monitor:
            for n, g in zip(names, grads):
                ops.monitored_all_reduce_(g, name=n)
            if self.op == "avg":
                for g in grads:
                    g.mul_(1.0 / ops.cluster_size())
            return
        ops.group_all_reduce_(grads, op=self.op, names=names)


def SynchronousSGDOptimizer(optimizer, named_parameters=None, op: str = "avg", fused: bool = True,
                            bucket_mb: Optional[float] = None, comm_dtype: Optional[torch.dtype] = None,
                            hierarchical: bool = False, monitor: bool = False, overlap: bool = True,
                            nccl=None, nccl_fusion=None, hierarchical_nccl=None, force_comm: bool = False,
                            flat=None, first_bucket_mb: float = 1.0):
    """Wrap ``optimizer`` so that ``step()`` applies globally averaged gradients.

    * ``comm_dtype=torch.bfloat16``: bf16 gradients on the wire (half the bytes).
    * ``force_comm=True``: issue the bucket collectives even with one peer
      (exercises the RCCL data plane at N=1; by default a single peer skips them).
    * ``flat=True``: use the flat-buffer bucket engine for CPU models too (over
      the host transport); the default is flat on GPU, per-tensor on CPU.
    * ``nccl``/``nccl_fusion`` are accepted for API parity with the reference and
      have no effect (documented no-ops): on GPU the RCCL data plane is always
      used and fusion is the flat bucketed buffer.  ``hierarchical_nccl`` maps
      to ``hierarchical``.
    """
    if hierarchical_nccl:
        hierarchical = True
    return _SynchronousSGD(optimizer, named_parameters, op=op, fused=fused, bucket_mb=bucket_mb,
                           comm_dtype=comm_dtype, hierarchical=hierarchical, monitor=monitor, overlap=overlap,
                           force_comm=force_comm, flat=flat, first_bucket_mb=first_bucket_mb)
