"""Whole-step hipGraph capture: one training step (zero_grad + forward + backward with the
bucketed RCCL all-reduces + the fused optimizer) recorded once and replayed as ONE graph launch.

Why: the eager step is a few hundred kernel launches issued from Python (autograd, the fused
blocks' bookkeeping, the bucket hooks); the host needs ~16 ms to enqueue a ResNet-50 step whose
GPU time is ~21 ms (``tools/diag/cpu_overhead.py``), so any extra host work per step -- more
ranks' RCCL enqueues, slower host CPUs -- would make the step host-bound.  A replay costs the
host one ``hipGraphLaunch``.

What makes a step capturable here:
* every kernel of the engine is launched on the current / comm stream with device-resident
  arguments; host-side decisions (bucket order, BN links, tile choices) are made at capture time
  and stay valid because the replayed step has the same shapes and pointers (static inputs);
* per-step scalars that change between replays live in device tensors refreshed before each
  replay (:meth:`GraphedStep.pre_replay`: the fused optimizers' learning rate);
* the RCCL bucket collectives are captured on the comm stream, which joins the capture through
  the engine's event fence / join; the native watchdog skips registrations made while a stream
  is capturing (graph replays are not watched -- ``rccl_comm.hip`` ``watch``);
* capture happens after ``warmup`` eager steps, once the bucket engine has learned its
  collective order (rank 0's order is adopted on the second step) and every lazily allocated
  workspace (BN statistics slots, flip caches, comm buffers) exists.

Limits: inputs must be static tensors the caller refills in place; the step's Python code runs
only at capture (counters it keeps stop advancing).  Dropout: the attention / add+LayerNorm
kernels hash a host seed recorded at capture with a device word that :meth:`pre_replay`
advances (``ops.dropout_seed``), so every replay draws fresh masks.  Parity: none in the reference (TF
graphs are its equivalent); MI355X-first replacement for a tracing compiler.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import torch


def _lr_holders(opt) -> List[object]:
    """Objects with a device ``_lr_t`` scalar mirroring ``param_groups[0]['lr']``."""
    out, seen = [], set()
    stack = [opt]
    while stack:
        o = stack.pop()
        if o is None or id(o) in seen:
            continue
        seen.add(id(o))
        if hasattr(o, "_lr_t") and hasattr(o, "param_groups"):
            out.append(o)
        for attr in ("inner", "optimizer", "_opt"):
            stack.append(getattr(o, attr, None))
    return out


class GraphedStep:
    """``step = GraphedStep(fn, optimizer)``; ``loss = step()`` runs ``fn`` eagerly for ``warmup``
    calls, then captures it and replays the graph on every later call (returning the captured
    output tensor, refreshed by each replay)."""

    def __init__(self, fn: Callable[[], torch.Tensor], optimizer=None, warmup: int = 3,
                 capture_error_mode: str = "thread_local"):
        self.fn = fn
        self.opt = optimizer
        self.warmup = warmup
        self.mode = capture_error_mode
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out = None
        self.calls = 0
        self.replays = 0
        self._lr = _lr_holders(optimizer) if optimizer is not None else []

    def pre_replay(self):
        from ..ops import dropout_seed

        for o in self._lr:
            o._lr_t.fill_(o.param_groups[0]["lr"])
        dropout_seed.advance()  # fresh hashed dropout masks for this replay

    def capture(self):
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode=self.mode):
            self.out = self.fn()
        torch.cuda.synchronize()
        self.graph = g

    def __call__(self):
        self.calls += 1
        if self.graph is None:
            if self.calls <= self.warmup:
                return self.fn()
            self.capture()  # records without executing: replay now so this call did a step
        self.pre_replay()
        self.graph.replay()
        self.replays += 1
        return self.out
