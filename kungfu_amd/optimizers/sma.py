"""SynchronousAveragingOptimizer (SMA / EA-SGD style model averaging).

Parity: ``srcs/python/kungfu/tensorflow/optimizers/sma_sgd.py:9-74``: every
step, all-reduce the *variables*, blend ``v <- (1-alpha) v + alpha avg(v)``,
then apply the local gradient (overlapped via control dependencies).

MI355X design (GPU): right after each update the flat parameter buffer is
snapshotted into a comm buffer on the comm stream and all-reduced (op avg)
there, so the model all-reduce overlaps the next iteration's forward and
backward.  At ``step()`` the compute stream waits for it and one fused HIP
kernel (K3 ``axpby``) blends the model, then the fused optimizer applies the
local gradient.  CPU tensors use the host runtime's grouped all-reduce.
"""
from __future__ import annotations

import torch

from .. import ops
from .._lib import hip
from ..parallel.comm import get_device_comm
from .core import KungFuOptimizer


class _SynchronousAveraging(KungFuOptimizer):
    def __init__(self, optimizer, named_parameters=None, alpha: float = 0.1, fused: bool = True):
        super().__init__(optimizer, named_parameters, fused=fused)
        self.alpha = alpha
        self._avg = None
        if self.space is not None:
            self.comm = get_device_comm()
            self._avg = torch.empty_like(self.space.flat_param)
            self._launch_average()

    def _launch_average(self):
        comm = self.comm
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(comm.device))
        comm.stream.wait_event(ev)
        with torch.cuda.stream(comm.stream):
            self._avg.copy_(self.space.flat_param, non_blocking=True)
        comm.all_reduce(self._avg, op="avg")

    def _before_step(self):
        if self.space is not None:
            torch.cuda.current_stream(self.comm.device).wait_stream(self.comm.stream)
            # v <- (1 - a) v + a avg(v)
            hip().axpby(self.space.flat_param, self._avg, None, 1.0 - self.alpha, self.alpha)
            return
        vs = [p for p in self.params if p.grad is not None]
        avgs = [v.detach().clone() for v in vs]
        ops.group_all_reduce_(avgs, op="avg", names=["sma:%d" % i for i in range(len(avgs))])
        with torch.no_grad():
            for v, a in zip(vs, avgs):
                v.mul_(1.0 - self.alpha).add_(a, alpha=self.alpha)

    def _after_step(self):
        if self.space is not None:
            self._launch_average()


def SynchronousAveragingOptimizer(optimizer, named_parameters=None, alpha: float = 0.1, fused: bool = True,
                                  name=None, use_locking=False, with_keras=False):
    """Wrap ``optimizer`` with synchronous model averaging (alpha = weight of
    the central model).  ``name``/``use_locking``/``with_keras`` are accepted
    for API parity with the reference and ignored."""
    return _SynchronousAveraging(optimizer, named_parameters, alpha=alpha, fused=fused)
