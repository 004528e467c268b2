"""AdaptiveSGDOptimizer (AdaSGD): synchronous model averaging until
``change_step``, synchronous SGD afterwards; the models are re-synchronised by
a broadcast from rank 0 at the switch.

Parity: ``srcs/python/kungfu/tensorflow/optimizers/ada_sgd.py:12-83``
(``tf.cond(global_step < change_step, sma, ssgd)`` + ``AdaSGDHook`` broadcasting
all variables at ``change_step``).

GPU: both phases share one flat parameter space; the S-SGD gradient reducer
is registered from the start but disabled (``no_sync``) during the SMA phase,
so the switch costs one broadcast and no re-allocation.
"""
from __future__ import annotations

import torch

from .. import ops
from .._lib import hip
from ..parallel.comm import get_device_comm
from ..parallel.ddp import GradReducer
from .core import KungFuOptimizer


class _AdaptiveSGD(KungFuOptimizer):
    def __init__(self, optimizer, named_parameters=None, change_step: int = 1000, alpha: float = 0.1,
                 fused: bool = True):
        super().__init__(optimizer, named_parameters, fused=fused)
        self.change_step = change_step
        self.alpha = alpha
        self.global_step = 0
        self.reducer = None
        if self.space is not None:
            self.comm = get_device_comm()
            self._avg = torch.empty_like(self.space.flat_param)
            self.reducer = GradReducer(self.space, op="avg")
            self.reducer._enabled = change_step <= 0
            if change_step > 0:
                self._launch_average()

    @property
    def phase(self) -> str:
        return "sma" if self.global_step < self.change_step else "ssgd"

    def _launch_average(self):
        comm = self.comm
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(comm.device))
        comm.stream.wait_event(ev)
        with torch.cuda.stream(comm.stream):
            self._avg.copy_(self.space.flat_param, non_blocking=True)
        comm.all_reduce(self._avg, op="avg")

    def _before_step(self):
        if self.phase == "sma":
            if self.space is not None:
                torch.cuda.current_stream(self.comm.device).wait_stream(self.comm.stream)
                hip().axpby(self.space.flat_param, self._avg, None, 1.0 - self.alpha, self.alpha)
            else:
                vs = [p for p in self.params if p.grad is not None]
                avgs = [v.detach().clone() for v in vs]
                ops.group_all_reduce_(avgs, op="avg")
                with torch.no_grad():
                    for v, a in zip(vs, avgs):
                        v.mul_(1.0 - self.alpha).add_(a, alpha=self.alpha)
        else:
            if self.reducer is not None:
                self.reducer.synchronize()
            else:
                grads = [p.grad for p in self.params if p.grad is not None]
                ops.group_all_reduce_(grads, op="avg")

    def _after_step(self):
        self.global_step += 1
        if self.global_step == self.change_step:
            # AdaSGDHook: broadcast every variable when switching to S-SGD
            if self.space is not None:
                torch.cuda.current_stream(self.comm.device).wait_stream(self.comm.stream)
                ops.inplace_broadcast_(self.space.flat_param)
                self.reducer._enabled = True
            else:
                for p in self.params:
                    ops.inplace_broadcast_(p.data)
        elif self.phase == "sma" and self.space is not None:
            self._launch_average()


def AdaptiveSGDOptimizer(optimizer, change_step: int, named_parameters=None, alpha: float = 0.1,
                         fused: bool = True, name=None, use_locking=False, with_keras=False):
    return _AdaptiveSGD(optimizer, named_parameters, change_step=change_step, alpha=alpha, fused=fused)
