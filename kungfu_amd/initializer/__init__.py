"""Initial (and post-resize) state synchronisation.

Parity: ``srcs/python/kungfu/tensorflow/initializer/__init__.py:13-99``
(``broadcast_variables``, ``BroadcastGlobalVariablesOp``,
``BroadcastGlobalVariablesHook``, ``BroadcastGlobalVariablesCallback`` which
broadcasts after the first batch so optimizer slots exist) and
``srcs/python/kungfu/torch/ops/collective.py:40-45`` (``broadcast_parameters``).

Engine-aware: when the optimizer re-homed the parameters into a flat buffer,
the whole model is ONE broadcast of that buffer (plus one per optimizer state
buffer) instead of one per tensor.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import ops


def broadcast_parameters(state) -> None:
    ops.broadcast_parameters(state)


broadcast_variables = broadcast_parameters


def _scalar_holders(optimizer):
    """Objects (the wrapper and the wrapped optimizer) exposing ``_kf_scalars`` /
    ``_kf_load_scalars``: host-side state such as FusedSGD's first-step flag or
    a monitor's step counter, which must match rank 0 after a (re)join."""
    out = []
    for o in (optimizer, getattr(optimizer, "inner", None)):
        if o is not None and hasattr(o, "_kf_scalars") and all(o is not x for x in out):
            out.append(o)
    return out


def broadcast_optimizer_state(optimizer) -> None:
    """Broadcast optimizer state from rank 0: flat buffers (momentum, Adam moments
    and step), per-parameter state tensors, and host-side scalars."""
    inner = getattr(optimizer, "inner", optimizer)
    flat_bufs = [getattr(inner, n, None) for n in ("momentum_buffer", "exp_avg", "exp_avg_sq", "_step_t")]
    for b in flat_bufs:
        if isinstance(b, torch.Tensor):
            ops.inplace_broadcast_(b)
    holders = _scalar_holders(optimizer)
    if holders:
        vals = [list(map(float, h._kf_scalars())) for h in holders]
        t = torch.tensor([v for vs in vals for v in vs], dtype=torch.float64)
        ops.inplace_broadcast_(t)
        k = 0
        for h, vs in zip(holders, vals):
            h._kf_load_scalars(t[k:k + len(vs)].tolist())
            k += len(vs)
    for p, st in inner.state.items():
        for k in sorted(st.keys()):
            v = st[k]
            if isinstance(v, torch.Tensor):
                ops.inplace_broadcast_(v)


def broadcast_model(model: torch.nn.Module, optimizer=None) -> None:
    """Make every peer hold rank 0's model (and optimizer state)."""
    space = getattr(optimizer, "space", None) if optimizer is not None else None
    if space is not None:
        ops.inplace_broadcast_(space.flat_param)
        bufs = {k: v for k, v in model.state_dict().items()
                if isinstance(v, torch.Tensor) and not any(v.data_ptr() == p.data_ptr() for p in space.params)}
        ops.broadcast_parameters(bufs)
    else:
        ops.broadcast_parameters(model.state_dict())
    if optimizer is not None:
        broadcast_optimizer_state(optimizer)


class BroadcastGlobalVariablesCallback:
    """Training-loop callback: broadcast model + optimizer state once, after
    the first batch (so lazily created optimizer state exists)."""

    def __init__(self, model: torch.nn.Module, optimizer=None):
        self.model, self.optimizer, self.done = model, optimizer, False

    def on_batch_end(self, *_):
        if not self.done:
            broadcast_model(self.model, self.optimizer)
            self.done = True

    after_step = on_batch_end


BroadcastGlobalVariablesHook = BroadcastGlobalVariablesCallback


def BroadcastGlobalVariablesOp(model: torch.nn.Module, optimizer: Optional[object] = None):
    """Eager equivalent of the TF op: performs the broadcast now."""
    broadcast_model(model, optimizer)
