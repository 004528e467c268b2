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


def broadcast_bytes(data: Optional[bytes]) -> bytes:
    """Rank 0's ``data`` on every peer (other ranks may pass None)."""
    from ..python import current_rank

    root = current_rank() == 0
    n = torch.tensor([len(data) if root and data is not None else 0], dtype=torch.int64)
    ops.inplace_broadcast_(n)
    buf = torch.zeros(int(n[0]), dtype=torch.uint8)
    if root and int(n[0]):
        buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    if int(n[0]):
        ops.inplace_broadcast_(buf)
    return bytes(buf.numpy().tobytes())


def _agree_state_layout(inner) -> None:
    """Make every peer's per-parameter optimizer state match rank 0's LAYOUT (which
    parameters have state, which keys, shapes, dtypes) and its non-tensor values, before
    the per-tensor broadcasts: a freshly started (or re-joined) peer has no lazily
    created state while rank 0 -- e.g. after a checkpoint load -- has one entry per
    parameter, and mismatched broadcast counts would hang (RCCL) or silently pair the
    wrong tensors (host plane).  Param-group hyper-parameters follow rank 0 too."""
    import json

    from ..python import current_rank

    params = [p for g in inner.param_groups for p in g["params"]]
    if current_rank() == 0:
        index = {id(p): i for i, p in enumerate(params)}
        layout = []
        for p, st in inner.state.items():
            if id(p) not in index:
                continue
            ent = {}
            for k, v in st.items():
                if isinstance(v, torch.Tensor):
                    ent[k] = ["t", list(v.shape), str(v.dtype).replace("torch.", ""), v.device.type == "cpu"]
                elif isinstance(v, (bool, int, float)) or v is None:
                    ent[k] = ["v", v]
            layout.append([index[id(p)], ent])
        groups = [{k: v for k, v in g.items() if k != "params" and (isinstance(v, (bool, int, float)) or v is None)}
                  for g in inner.param_groups]
        data = json.dumps({"state": layout, "groups": groups}).encode()
    else:
        data = None
    spec = json.loads(broadcast_bytes(data).decode())
    for g, gv in zip(inner.param_groups, spec["groups"]):
        g.update(gv)
    want = {i: ent for i, ent in spec["state"]}
    for i, p in enumerate(params):
        ent = want.get(i)
        if ent is None:
            inner.state.pop(p, None)
            continue
        st = inner.state.setdefault(p, {})
        for k in [k for k in st if k not in ent]:
            del st[k]
        for k, e in ent.items():
            if e[0] == "v":
                st[k] = e[1]
                continue
            shape, dt, on_cpu = tuple(e[1]), getattr(torch, e[2]), e[3]
            dev = torch.device("cpu") if on_cpu else p.device
            v = st.get(k)
            if not (isinstance(v, torch.Tensor) and tuple(v.shape) == shape and v.dtype == dt and v.device == dev):
                st[k] = torch.zeros(shape, dtype=dt, device=dev)


def broadcast_optimizer_state(optimizer) -> None:
    """Broadcast optimizer state from rank 0: flat buffers (momentum, Adam moments
    and step), per-parameter state tensors (after agreeing on their layout), and
    host-side scalars."""
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
    if not hasattr(inner, "param_groups"):
        return
    _agree_state_layout(inner)
    params = [p for g in inner.param_groups for p in g["params"]]
    for p in params:  # parameter order, identical on every peer
        st = inner.state.get(p)
        if not st:
            continue
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
