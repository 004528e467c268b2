"""SynchronousSGDOptimizer (S-SGD): average gradients across all peers, then apply.

Parity: ``srcs/python/kungfu/tensorflow/optimizers/sync_sgd.py:15-109``
(``nccl``, ``nccl_fusion``, ``hierarchical_nccl``, ``monitor`` options) and
the torch wrapper ``srcs/python/kungfu/torch/optimizers/sync_sgd.py:6-32``.

Data planes:
* GPU (default): bucketed in-place RCCL all-reduce of the flat gradient
  buffer, launched from backward hooks on a comm stream (overlapped with
  backward), op ``avg``.  ``hierarchical=True`` runs every bucket as local reduce ->
  cross-host host all-reduce among the local roots -> local broadcast, still
  overlapped with backward (reference's hierarchical NCCL path,
  ``ops/gpu/collective.cpp:105-156``; see ``ddp._CrossHostStage``).
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


class InterferenceAdapter:
    """Adaptive strategy switching driven by the monitored all-reduce statistics.

    Parity: ``experimental/adapt_strategy/adapt_strategy.py:188-213`` (after warm-up, every
    step: ``calc_stats``; ``check_interference``; on a cluster majority switch ONCE to an
    alternative star tree, ``get_alternative_star_strategy``) over
    ``srcs/go/kungfu/session/adaptiveStrategies.go:61-121`` (throughput < 0.8 x the
    reference window => vote).  Every peer calls :meth:`after_step` at the same steps, so
    the votes (a collective) match.  On the RCCL plane the statistics are device-timed
    bucket all-reduces; the switch re-routes the host plane and the device graph plane
    (``KUNGFU_GPU_ALLREDUCE=graph``) -- RCCL's own ring/tree choice is RCCL's."""

    def __init__(self, warmup: int = 5, interval: int = 1, alternative_root: int = 1):
        self.warmup, self.interval, self.alt_root = warmup, max(1, interval), alternative_root
        self.step = 0
        self.changed = False
        self.switched_at = None
        self.throughputs = []

    def after_step(self):
        from .. import ops
        from .._lib import runtime

        self.step += 1
        if self.step % self.interval:
            return
        ops.calc_stats()
        tp = runtime.strategy_throughputs()
        self.throughputs.append(tp[0] if len(tp) == 1 else None)
        if self.changed or self.step <= self.warmup:
            return
        if ops.check_interference():
            n = ops.cluster_size()
            ops.set_tree([self.alt_root % n] * n)
            self.changed = True
            self.switched_at = self.step


class _SynchronousSGD(KungFuOptimizer):
    def __init__(self, optimizer, named_parameters=None, op: str = "avg", fused: bool = True,
                 bucket_mb: Optional[float] = None, comm_dtype: Optional[torch.dtype] = None,
                 hierarchical: bool = False, monitor: bool = False, overlap: bool = True,
                 force_comm: bool = False, flat=None, first_bucket_mb: float = 1.0, adapt: bool = False,
                 adapt_warmup: int = 5):
        super().__init__(optimizer, named_parameters, fused=fused, flat=flat)
        self.op = op
        self.monitor = monitor or adapt
        self.hierarchical = hierarchical
        self.reducer: Optional[GradReducer] = None
        if self.space is not None and overlap:
            self.reducer = GradReducer(self.space, op="avg" if op == "avg" else "sum", bucket_mb=bucket_mb,
                                       comm_dtype=comm_dtype, skip_single=not force_comm,
                                       first_bucket_mb=first_bucket_mb, monitored=self.monitor and not hierarchical,
                                       hierarchical=hierarchical)
        self.adapter = InterferenceAdapter(warmup=adapt_warmup) if adapt else None

    def _before_step(self):
        if self.reducer is not None:
            self.reducer.synchronize()
            return
        self.sync_gradients()

    def _after_step(self):
        if self.adapter is not None and ops.cluster_size() > 1:
            self.adapter.after_step()

    def sync_gradients(self):
        if self.space is not None:
            g = self.space.flat_grad
            if self.hierarchical:
                ops.hierarchical_all_reduce_(g, op="sum")
                if self.op == "avg":
                    g.mul_(1.0 / ops.cluster_size())
            elif self.monitor:
                ops.monitored_all_reduce_(g)
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
                            flat=None, first_bucket_mb: float = 1.0, adapt: bool = False, adapt_warmup: int = 5):
    """Wrap ``optimizer`` so that ``step()`` applies globally averaged gradients.

    * ``comm_dtype=torch.bfloat16``: bf16 gradients on the wire (half the bytes).
    * ``force_comm=True``: issue the bucket collectives even with one peer
      (exercises the RCCL data plane at N=1; by default a single peer skips them).
    * ``flat=True``: use the flat-buffer bucket engine for CPU models too (over
      the host transport); the default is flat on GPU, per-tensor on CPU.
    * ``monitor=True``: every gradient all-reduce (each bucket on the GPU engine, timed
      with HIP events on the comm stream and anchored to the runtime clock) feeds the
      session's strategy statistics (``calc_stats`` / ``check_interference``).
    * ``adapt=True`` (implies ``monitor``): after ``adapt_warmup`` steps, check for
      interference every step and switch once to an alternative star tree on a cluster
      majority (:class:`InterferenceAdapter`).
    * ``nccl``/``nccl_fusion`` are accepted for API parity with the reference and
      have no effect (documented no-ops): on GPU the RCCL data plane is always
      used and fusion is the flat bucketed buffer.  ``hierarchical_nccl`` maps
      to ``hierarchical``.
    """
    if hierarchical_nccl:
        hierarchical = True
    return _SynchronousSGD(optimizer, named_parameters, op=op, fused=fused, bucket_mb=bucket_mb,
                           comm_dtype=comm_dtype, hierarchical=hierarchical, monitor=monitor, overlap=overlap,
                           force_comm=force_comm, flat=flat, first_bucket_mb=first_bucket_mb, adapt=adapt,
                           adapt_warmup=adapt_warmup)
