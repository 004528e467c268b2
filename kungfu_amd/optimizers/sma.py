"""SynchronousAveragingOptimizer (SMA / EA-SGD style model averaging).

Parity: ``srcs/python/kungfu/tensorflow/optimizers/sma_sgd.py:9-74``: every
step, all-reduce the *variables*, blend ``v <- (1-alpha) v + alpha avg(v)``,
then apply the local gradient (overlapped via control dependencies).

MI355X design (GPU): right after each update the flat parameter buffer is
snapshotted into a comm buffer on the comm stream and all-reduced (op avg)
there, so the model all-reduce overlaps the next iteration's forward and
backward.  At ``step()`` the compute stream waits for it and one fused HIP
kernel (K3 ``axpby``) blends the model, then the fused optimizer applies the
local gradient.

Elastic: the in-flight average is tagged with the (cluster version, comm
epoch) it was issued under.  After a resize (or on the very first step, so a
worker joining a running job issues no collective from its constructor) the
stale average is discarded and a fresh one is computed from the current
(just re-broadcast) parameters on the new communicator -- every member of the
new cluster does this at the same point of its step.

CPU models with a flat space run the same code over the host transport
(:class:`~kungfu_amd.parallel.comm.HostComm`); models without one use the
host runtime's grouped all-reduce per tensor.
"""
from __future__ import annotations

import torch

from .. import ops
from .._lib import runtime
from ..parallel.comm import comm_epoch, get_device_comm
from ..parallel.flat import axpby_
from .core import KungFuOptimizer


class ModelAverager:
    """Asynchronous all-reduce (op avg) of a flat parameter buffer, re-bound after resizes.
    Shared by SMA and AdaSGD."""

    def __init__(self, space, force_comm: bool = False):
        self.space = space
        # force_comm: with one peer still snapshot + all-reduce (1-rank RCCL) + blend, so the
        # overlap of the model all-reduce with the next forward is exercised / profiled at N=1
        self.force_comm = force_comm
        self.comm = None
        self.key = None  # (cluster version, comm epoch) of the pending average
        self._avg = torch.empty_like(space.flat_param)

    @staticmethod
    def current_key():
        return runtime.cluster_version(), comm_epoch()

    def launch(self):
        """Snapshot the parameters and start their average on the comm stream."""
        if runtime.size() == 1 and not self.force_comm:
            self.key = self.current_key()
            self.comm = None
            return
        self.comm = get_device_comm(device=self.space.device)
        self.key = self.current_key()
        self.comm.fence()
        with self.comm.on_stream():
            self._avg.copy_(self.space.flat_param, non_blocking=True)
        # one rank: the in-place sum IS the average (RCCL's one-rank avg is an extra scaled copy)
        self.comm.all_reduce(self._avg, op="avg" if self.comm.size > 1 else "sum", tag="sma model average")

    def blend(self, alpha: float):
        """v <- (1 - alpha) v + alpha avg(v), using the pending average if it is
        still valid for the current cluster, else a fresh one."""
        if self.key != self.current_key():
            self.launch()
        if self.comm is None:  # one peer: the average is the model itself
            return
        self.comm.join()
        axpby_(self.space.flat_param, self._avg, 1.0 - alpha, alpha)

    def wait(self):
        if self.comm is not None:
            self.comm.join()


class _SynchronousAveraging(KungFuOptimizer):
    def __init__(self, optimizer, named_parameters=None, alpha: float = 0.1, fused: bool = True,
                 flat=None, force_comm: bool = False):
        super().__init__(optimizer, named_parameters, fused=fused, flat=flat)
        self.alpha = alpha
        self.averager = ModelAverager(self.space, force_comm=force_comm) if self.space is not None else None

    def _before_step(self):
        if self.averager is not None:
            self.averager.blend(self.alpha)
            return
        vs = [p for p in self.params if p.grad is not None]
        avgs = [v.detach().clone() for v in vs]
        ops.group_all_reduce_(avgs, op="avg", names=["sma:%d" % i for i in range(len(avgs))])
        with torch.no_grad():
            for v, a in zip(vs, avgs):
                v.mul_(1.0 - self.alpha).add_(a, alpha=self.alpha)

    def _after_step(self):
        if self.averager is not None:
            self.averager.launch()


def SynchronousAveragingOptimizer(optimizer, named_parameters=None, alpha: float = 0.1, fused: bool = True,
                                  name=None, use_locking=False, with_keras=False, flat=None, force_comm: bool = False):
    """Wrap ``optimizer`` with synchronous model averaging (alpha = weight of
    the central model).  ``name``/``use_locking``/``with_keras`` are accepted
    for API parity with the reference and ignored.  ``force_comm``: run the model
    all-reduce even with one peer (see :class:`ModelAverager`)."""
    return _SynchronousAveraging(optimizer, named_parameters, alpha=alpha, fused=fused, flat=flat,
                                 force_comm=force_comm)
