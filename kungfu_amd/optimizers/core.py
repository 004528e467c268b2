"""Base class of the distributed optimizer wrappers.

Parity: ``srcs/python/kungfu/tensorflow/optimizers/core.py:6-72``
(``KungFuTFOptimizer``: wraps a framework optimizer and intercepts
``apply_gradients``) and the torch wrapper
``srcs/python/kungfu/torch/optimizers/sync_sgd.py:6-32``.

A wrapper is itself a ``torch.optim.Optimizer`` whose ``param_groups`` and
``state`` ARE the wrapped optimizer's, so LR schedulers, ``zero_grad`` and
``state_dict`` behave as with the inner optimizer.

On GPU the wrapper re-homes the parameters into a :class:`FlatParamSpace`
(one flat f32 param buffer + one flat grad buffer); plain ``torch.optim.SGD``
/ ``Adam`` / ``AdamW`` with a single param group are replaced by the fused
flat-buffer HIP optimizers unless ``fused=False``.
"""
from __future__ import annotations

from typing import Iterable, Optional, Tuple

import torch

from ..parallel.flat import FlatParamSpace
from ..utils import trace
from .fused import FusedAdam, FusedSGD


def _named(named_parameters, optimizer) -> dict:
    names = {}
    if named_parameters is not None:
        for n, p in named_parameters:
            names[id(p)] = n
    return names


def make_fused(optimizer: torch.optim.Optimizer, space: FlatParamSpace) -> Optional[torch.optim.Optimizer]:
    """Build a fused flat optimizer equivalent to ``optimizer`` if possible."""
    if len(optimizer.param_groups) != 1:
        return None
    g = optimizer.param_groups[0]
    t = type(optimizer)
    if t is torch.optim.SGD:
        if g.get("maximize", False):
            return None
        return FusedSGD(space, lr=g["lr"], momentum=g["momentum"], dampening=g["dampening"],
                        weight_decay=g["weight_decay"], nesterov=g["nesterov"])
    if t in (torch.optim.Adam, torch.optim.AdamW):
        if g.get("amsgrad", False) or g.get("maximize", False):
            return None
        return FusedAdam(space, lr=g["lr"], betas=g["betas"], eps=g["eps"], weight_decay=g["weight_decay"],
                         adamw=(t is torch.optim.AdamW))
    return None


class KungFuOptimizer(torch.optim.Optimizer):
    """Wraps ``optimizer``; subclasses implement :meth:`_before_step` /
    :meth:`_after_step` (the distributed part)."""

    def __init__(self, optimizer: torch.optim.Optimizer, named_parameters: Optional[Iterable[Tuple[str, torch.nn.Parameter]]] = None,
                 fused: bool = True, flat: Optional[bool] = None):
        params = [p for g in optimizer.param_groups for p in g["params"]]
        gpu = len(params) > 0 and params[0].is_cuda
        use_flat = gpu if flat is None else flat
        names = _named(named_parameters, optimizer)
        self.space: Optional[FlatParamSpace] = None
        inner = optimizer
        if use_flat:
            self.space = FlatParamSpace(params, names=names)
            if fused:
                f = make_fused(optimizer, self.space)
                if f is not None:
                    inner = f
        self.inner = inner
        super().__init__(inner.param_groups, inner.defaults)
        self.param_groups = inner.param_groups
        self.state = inner.state
        self.names = names
        self._wrapped = True

    # -- torch.optim.Optimizer surface ---------------------------------------
    def zero_grad(self, set_to_none: bool = False):
        if self.space is not None:
            self.space.zero_grad()
        else:
            self.inner.zero_grad(set_to_none=set_to_none)

    def state_dict(self):
        return self.inner.state_dict()

    def load_state_dict(self, sd):
        self.inner.load_state_dict(sd)

    def add_param_group(self, group):
        if not getattr(self, "_wrapped", False):
            return super().add_param_group(group)
        raise RuntimeError("kungfu_amd optimizers do not support adding param groups after wrapping")

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        with trace.scope("optimizer::before_step"):
            self._before_step()
        with trace.scope("optimizer::apply"):
            self.inner.step()
        with trace.scope("optimizer::after_step"):
            self._after_step()
        return loss

    # -- hooks for subclasses ------------------------------------------------
    def _before_step(self):
        pass

    def _after_step(self):
        pass

    @property
    def params(self):
        return [p for g in self.param_groups for p in g["params"]]
