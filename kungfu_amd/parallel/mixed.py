"""bf16 compute weights over f32 master weights, with gradients landed directly
in the flat f32 gradient buffer ("direct gradients").

Under ``torch.autocast(dtype=bfloat16)`` a stock model pays, per conv/linear
weight and per step: one f32->bf16 cast in forward, one bf16->f32 cast of the
weight gradient in backward and one ``AccumulateGrad`` add into ``.grad`` --
~3 x 53 small launches for ResNet-50 (profiles/r5_*.md: ~1.7 ms of a 29 ms
step).  The MI355X-native arrangement instead:

* keeps a bf16 *shadow* of the whole flat master buffer, refreshed by ONE
  cast kernel at the start of every forward (a model forward pre-hook), and
  hands conv/linear modules a bf16 view of it -- numerically identical to
  autocast's own round-to-nearest-even weight cast;
* routes the bf16 weight gradient (and the fused BN's f32 gamma/beta
  gradients) to the space's *gradient sink* instead of ``AccumulateGrad``.
  The default sink adds immediately; the S-SGD engine's
  :class:`~kungfu_amd.parallel.ddp.GradReducer` stages them per bucket and
  lands a whole bucket with ONE multi-tensor kernel
  (``_hip.grad_accumulate``: flat += bf16/f32 sources) right before the
  bucket's all-reduce.

No reference counterpart: the reference trains in f32 TensorFlow and leaves
precision to the framework; this is the MI355X data path for its S-SGD
(``srcs/python/kungfu/tensorflow/optimizers/sync_sgd.py:78-109``).

Usage::

    opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(model.parameters(), ...))
    kf.parallel.mixed.enable_bf16_shadow(model, opt)
"""
from __future__ import annotations

import os
import types
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .flat import FlatParamSpace

# id(param) -> (space, index) for parameters whose gradients go to space.sink
_DIRECT: Dict[int, Tuple[FlatParamSpace, int]] = {}


def direct_target(p: Optional[torch.Tensor]) -> Optional[Tuple[FlatParamSpace, int]]:
    """(space, index) if ``p``'s gradient should be handed to ``space.sink``."""
    if p is None:
        return None
    return _DIRECT.get(id(p))


def deliver(target: Tuple[FlatParamSpace, int], g: torch.Tensor) -> None:
    space, i = target
    space.sink.put(i, g)


# Parameters with SEVERAL direct producers in one backward (a tied embedding: the lookup's scatter-add
# and the vocabulary projection's weight gradient, ops/embedding.py + ops/vocab.py).  Every forward use
# calls use_direct; each producer adds its share into the flat f32 slot itself and calls landed_direct,
# and the LAST one hands the parameter to the sink's bucket accounting (put_direct) -- so the bucket
# launches once, after the whole gradient is in the slot, whatever order the producers run in.
_PENDING: Dict[Tuple[int, int], int] = {}
_EMBED_DIRECT = True  # module switch (tests / A/B)


def reset_pending() -> None:
    """Forget every outstanding forward use (called at the end of each backward): a forward that
    never got a backward (grad-enabled eval, a skipped step) would otherwise keep its table's count
    above zero and its bucket would only launch at the end-of-backward flush from then on."""
    _PENDING.clear()


def use_direct(target: Tuple[FlatParamSpace, int]) -> None:
    k = (id(target[0]), target[1])
    _PENDING[k] = _PENDING.get(k, 0) + 1


def landed_direct(target: Tuple[FlatParamSpace, int]) -> None:
    space, i = target
    k = (id(space), i)
    n = _PENDING.get(k, 1) - 1
    if n > 0:
        _PENDING[k] = n
        return
    _PENDING.pop(k, None)
    space.sink.put_direct(i)


def embedding_target(p: Optional[torch.Tensor]) -> Optional[Tuple[FlatParamSpace, int]]:
    """(space, index) of a registered embedding table whose direct producers land in its flat slot
    (needs a sink with ``put_direct``); None otherwise."""
    t = _DIRECT.get(id(p)) if p is not None and _EMBED_DIRECT else None
    if t is None or not hasattr(t[0].sink, "put_direct") or not p.is_cuda:
        return None
    return t


def _bf16_autocast(dev: str) -> bool:
    return torch.is_autocast_enabled(dev) and torch.get_autocast_dtype(dev) == torch.bfloat16


class _ShadowWeight(torch.autograd.Function):
    """Forward: the bf16 shadow view of a master weight (no kernel).
    Backward: the bf16 weight gradient goes to the space's sink."""

    @staticmethod
    def forward(ctx, w, space, i):
        ctx.target = (space, i)
        # a consumer that reduced the weight gradient straight into the flat slot (ops/linear.py
        # put_direct) returns None: no zero-filled gradient to materialise and land (49 weight-sized
        # fills + landing adds per BERT-base step)
        ctx.set_materialize_grads(False)
        return space.shadow_view(i)

    @staticmethod
    def backward(ctx, g):
        if g is not None:
            deliver(ctx.target, g)
        return None, None, None


def shadow(p: torch.Tensor) -> torch.Tensor:
    """bf16 compute copy of a registered master weight under bf16 autocast; ``p`` otherwise."""
    t = _DIRECT.get(id(p)) if p is not None else None
    if t is None or t[0].flat_shadow is None or not _bf16_autocast(p.device.type):
        return p
    return _ShadowWeight.apply(p, t[0], t[1])


def _conv_forward(self, x):
    w = shadow(self.weight)
    b = shadow(self.bias) if self.bias is not None else None
    if isinstance(self, nn.Conv2d) and self.padding_mode == "zeros" and x.dtype == torch.bfloat16:
        # 3x3 convolutions take the hand-written MFMA implicit-GEMM kernel (ops/conv.py)
        from ..ops import conv as _conv

        return _conv.conv2d(x, w, b, self.stride, self.padding, self.dilation, self.groups)
    return self._conv_forward(x, w, b)


def _linear_forward(self, x):
    from ..ops.linear import linear

    # bf16 shadow weights: the weight gradient takes the split-K MFMA kernel (ops/linear.py), which
    # reduces its splits straight into the weight's flat f32 gradient slot
    w = shadow(self.weight)
    return linear(x, w, shadow(self.bias) if self.bias is not None else None,
                  grad_target=direct_target(self.weight) if w is not self.weight else None)


class SideStream:
    """Weight gradients on a side stream, overlapping the backward data-gradient chain: the linear
    layers' direct split-K weight gradients (ops/linear.py ``_WGRAD_SIDE``; the fused bottleneck's
    conv weight gradients measured slower there, r3 / r6t4).  A weight gradient
    depends only on its layer's output gradient and input, and nothing on the critical path of
    backward reads it, so it can
    run beside the next layers' data gradients and the memory-bound BN passes (filling the
    CUs an under-sized grid leaves idle).  Its results reach the flat gradient buffer only
    through a gradient sink, which makes the landing stream wait for every side-stream
    event recorded so far (:meth:`join`) -- the join is deferred to the bucket launch / the
    end of backward instead of the end of each layer."""

    _streams: Dict[int, torch.cuda.Stream] = {}
    _pending: list = []
    # storage base pointer -> the event after the last side-stream kernel reading it: an in-place write
    # on the main stream into such a storage (ops.linear's ``g.addmm_``: with no dropout the
    # AddLayerNorm's skip gradient IS the gradient the side-stream weight gradient of FC2 reads) must
    # wait for that event first (:meth:`before_write`)
    _reads: Dict[int, torch.cuda.Event] = {}

    @classmethod
    def note_reads(cls, ev: torch.cuda.Event, *ts: torch.Tensor) -> None:
        for t in ts:
            cls._reads[t.untyped_storage().data_ptr()] = ev

    @classmethod
    def before_write(cls, t: torch.Tensor) -> None:
        """Make the current stream wait for side-stream kernels still reading ``t``'s storage."""
        if cls._reads:
            ev = cls._reads.pop(t.untyped_storage().data_ptr(), None)
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)

    @classmethod
    def stream(cls, dev: torch.device) -> torch.cuda.Stream:
        k = dev.index if dev.index is not None else torch.cuda.current_device()
        s = cls._streams.get(k)
        if s is None:
            s = cls._streams[k] = torch.cuda.Stream(device=k)
        return s

    @classmethod
    def run(cls, fn, *inputs: torch.Tensor) -> torch.Tensor:
        """``fn(*inputs)`` on the side stream after the work issued so far on the current
        stream; the result is registered for a deferred :meth:`join`."""
        main = torch.cuda.current_stream()
        side = cls.stream(inputs[0].device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            out = fn(*inputs)
            ev = torch.cuda.Event()
            ev.record(side)
        for t in inputs:
            t.record_stream(side)  # main may free them while the side stream still reads
        out.record_stream(main)  # consumed on the main stream after the join
        cls._pending.append(ev)
        cls.note_reads(ev, *inputs)
        return out

    @classmethod
    def join(cls, stream=None) -> None:
        if not cls._pending:
            return
        s = stream if stream is not None else torch.cuda.current_stream()
        for ev in cls._pending:
            s.wait_event(ev)
        cls._pending = []
        cls._reads = {}


class ImmediateSink:
    """Add the gradient into the flat slot now (one torch kernel per gradient)."""

    def __init__(self, space: FlatParamSpace):
        self.space = space
        self._join_armed = False

    def put(self, i: int, g: torch.Tensor) -> None:
        SideStream.join()
        with torch.no_grad():
            self.space.grad_view(i).add_(g)

    def _end_of_backward(self) -> None:
        self._join_armed = False
        SideStream.join()
        reset_pending()  # a use whose producer never ran (forward without this backward) is stale

    def _arm(self, fn) -> bool:
        """Queue ``fn`` for the end of the running backward; False (nothing queued) outside one."""
        try:
            torch.autograd.Variable._execution_engine.queue_callback(fn)
            return True
        except RuntimeError:
            return False

    def put_direct(self, i: int) -> None:
        """Parameter ``i``'s gradient was already added into its flat f32 slot by its producer.  The
        producer may still be running on :class:`SideStream` (ops/linear.py): the end of backward
        joins it, so the optimizer step on the main stream never reads a slot still being written."""
        if not self._join_armed:
            self._join_armed = self._arm(self._end_of_backward)
            if not self._join_armed:
                self._end_of_backward()


class BatchedSink(ImmediateSink):
    """Default sink for optimizers without a bucket engine (SMA, pair averaging, AdaSGD,
    local): stages the direct gradients of a backward and lands them ALL with one
    multi-tensor ``grad_accumulate`` kernel when the backward ends (an autograd engine
    callback) -- instead of one ``AccumulateGrad``-style add per weight (ResNet-50: 161
    adds, ~1.1 ms/step in profiles/r3o_sma_summary.md)."""

    def __init__(self, space: FlatParamSpace):
        super().__init__(space)
        self._staged, self._offs = [], []
        self._armed = False

    def put(self, i: int, g: torch.Tensor) -> None:
        if (g.dtype not in (torch.bfloat16, torch.float32) or not g.is_cuda
                or g.stride() != self.space.strides[i]):
            return super().put(i, g)
        self._staged.append(g)
        self._offs.append(self.space.offsets[i][0])
        self._arm_flush()

    def put_direct(self, i: int) -> None:
        self._arm_flush()  # the flush joins the side stream even when nothing is staged

    def _arm_flush(self) -> None:
        if not self._armed:
            self._armed = self._arm(self.flush)
            if not self._armed:  # not inside a backward pass: land now
                self.flush()

    def flush(self) -> None:
        self._armed = False
        SideStream.join()
        reset_pending()
        if self._staged:
            from .._lib import hip

            hip().grad_accumulate(self.space.flat_grad, self._staged, self._offs, 1.0)
            self._staged, self._offs = [], []


def enable_bf16_shadow(model: nn.Module, optimizer, bn_direct: bool = True) -> int:
    """Switch ``model``'s conv/linear weights to bf16 shadow compute and direct
    gradients (and, with ``bn_direct``, the fused BN's / AddLayerNorm's gamma/beta gradients).

    ``optimizer`` is a kungfu_amd optimizer with a flat space (or the space
    itself).  Returns the number of parameters switched to direct gradients.
    Modules outside the space keep the stock path.
    """
    space: FlatParamSpace = optimizer if isinstance(optimizer, FlatParamSpace) else optimizer.space
    if space is None:
        raise ValueError("enable_bf16_shadow: optimizer has no flat parameter space (CPU model?)")
    space.enable_shadow()
    if getattr(space, "sink", None) is None:
        space.sink = BatchedSink(space)
    n = 0

    def register(p):
        nonlocal n
        if p is None or not p.requires_grad:
            return False
        try:
            i = space.index(p)
        except KeyError:
            return False
        _DIRECT[id(p)] = (space, i)
        n += 1
        return True

    from ..ops.fused_bn import BatchNormAct2d
    from ..ops.layernorm import AddLayerNorm

    for m in model.modules():
        if getattr(type(m), "kf_shadow_forward", False):  # takes shadow() in its own forward
            if register(m.weight) and getattr(m, "bias", None) is not None:
                register(m.bias)
        elif type(m).forward in (nn.Conv1d.forward, nn.Conv2d.forward, nn.Conv3d.forward):
            if register(m.weight):
                if m.bias is not None:
                    register(m.bias)
                m.forward = types.MethodType(_conv_forward, m)
        elif type(m).forward is nn.Linear.forward:
            if register(m.weight):
                if m.bias is not None:
                    register(m.bias)
                m.forward = types.MethodType(_linear_forward, m)
        elif type(m).forward is nn.Embedding.forward and m.weight.dtype == torch.float32:
            # looked up by ops/embedding.py (f32 master) and, when tied, projected onto by ops/vocab.py
            # (bf16 shadow): both add their gradients straight into the flat slot (use_direct)
            register(m.weight)
        elif bn_direct and isinstance(m, (BatchNormAct2d, AddLayerNorm)):
            # the fused BN / residual+LayerNorm kernels hand their f32 gamma/beta gradients to the sink
            register(m.weight)
            register(m.bias)
    if getattr(model, "_kf_shadow_hook", None) is None:
        model._kf_shadow_hook = model.register_forward_pre_hook(lambda mod, args: space.refresh_shadow())
    return n


def disable(model: nn.Module) -> None:
    """Undo :func:`enable_bf16_shadow` for ``model`` (stock forwards, AccumulateGrad)."""
    h = getattr(model, "_kf_shadow_hook", None)
    if h is not None:
        h.remove()
        model._kf_shadow_hook = None
    for m in model.modules():
        if "forward" in m.__dict__:
            del m.forward
        for p in m.parameters(recurse=False):
            _DIRECT.pop(id(p), None)
