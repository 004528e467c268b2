"""AdaptiveSGDOptimizer (AdaSGD): synchronous model averaging until
``change_step``, synchronous SGD afterwards; the models are re-synchronised by
a broadcast from rank 0 at the switch.

Parity: ``srcs/python/kungfu/tensorflow/optimizers/ada_sgd.py:12-83``
(``tf.cond(global_step < change_step, sma, ssgd)`` + ``AdaSGDHook`` broadcasting
all variables at ``change_step``).

Flat-space models (GPU, or CPU with ``flat=True``): both phases share one flat
parameter space; the S-SGD gradient reducer is registered from the start but
disabled during the SMA phase, so the switch costs one broadcast and no
re-allocation.  Both the averager and the reducer re-bind to the current
communicator after an elastic resize (see ``sma.ModelAverager`` and
``ddp.GradReducer._bind``).
"""
from __future__ import annotations

import torch

from .. import ops
from ..parallel.ddp import GradReducer
from .core import KungFuOptimizer
from .sma import ModelAverager


class _AdaptiveSGD(KungFuOptimizer):
    def __init__(self, optimizer, named_parameters=None, change_step: int = 1000, alpha: float = 0.1,
                 fused: bool = True, flat=None):
        super().__init__(optimizer, named_parameters, fused=fused, flat=flat)
        self.change_step = change_step
        self.alpha = alpha
        self.global_step = 0
        self.reducer = None
        self.averager = None
        if self.space is not None:
            self.averager = ModelAverager(self.space)
            self.reducer = GradReducer(self.space, op="avg")
            self.reducer._enabled = change_step <= 0

    @property
    def phase(self) -> str:
        return "sma" if self.global_step < self.change_step else "ssgd"

    def _before_step(self):
        if self.phase == "sma":
            if self.averager is not None:
                self.averager.blend(self.alpha)
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
            # AdaSGDHook: broadcast every global variable when switching to S-SGD -- in
            # TF that includes the optimizer slots (momentum), so replicas continue
            # identically
            if self.space is not None:
                from ..initializer import broadcast_optimizer_state

                self.averager.wait()
                ops.inplace_broadcast_(self.space.flat_param)
                broadcast_optimizer_state(self)
                self.reducer._enabled = True
            else:
                for p in self.params:
                    ops.inplace_broadcast_(p.data)
        elif self.phase == "sma" and self.averager is not None:
            self.averager.launch()

    def _kf_scalars(self):
        return [self.global_step]

    def _kf_load_scalars(self, vals):
        self.global_step = int(vals[0])
        if self.reducer is not None:
            self.reducer._enabled = self.phase == "ssgd"


def AdaptiveSGDOptimizer(optimizer, change_step: int, named_parameters=None, alpha: float = 0.1,
                         fused: bool = True, name=None, use_locking=False, with_keras=False, flat=None):
    return _AdaptiveSGD(optimizer, named_parameters, change_step=change_step, alpha=alpha, fused=fused, flat=flat)
