"""Flat parameter / gradient storage.

Every trainable parameter of a model is re-homed into ONE contiguous f32
buffer (``param.data`` becomes a view) and its gradient into a second one
(``param.grad`` is a persistent view).  This is the MI355X-native replacement
for the reference's per-tensor collectives and fuse/defuse concat
(``srcs/python/kungfu/tensorflow/ops/__init__.py:29-46``):

* gradient buckets are plain slices of the flat gradient buffer, so the RCCL
  all-reduce runs in place with no pack/unpack copies;
* the optimizer step is a single fused HIP kernel over the flat buffers
  (K8) instead of one launch per tensor;
* model averaging (SMA, pair averaging) moves/blends one buffer.

Parameters are laid out in *reverse* registration order (the order autograd
produces their gradients), each slot aligned to 64 elements (256 B) so every
bucket boundary is 16-byte aligned for the vectorised kernels.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Tuple

import torch

ALIGN = 64


def _align(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


class FlatParamSpace:
    def __init__(self, params: Iterable[torch.nn.Parameter], dtype: torch.dtype = torch.float32,
                 reverse: bool = True, names: Optional[Dict[int, str]] = None):
        ps: List[torch.nn.Parameter] = []
        seen = set()
        for p in params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                ps.append(p)
        if not ps:
            raise ValueError("FlatParamSpace: no trainable parameters")
        if reverse:
            ps = ps[::-1]
        dev = ps[0].device
        for p in ps:
            if p.device != dev:
                raise ValueError("FlatParamSpace: parameters on several devices")
        self.params = ps
        self.names = [names.get(id(p), "param%d" % i) if names else "param%d" % i for i, p in enumerate(ps)]
        self.device = dev
        self.dtype = dtype
        self.offsets: List[Tuple[int, int]] = []
        off = 0
        for p in ps:
            n = p.numel()
            self.offsets.append((off, n))
            off = _align(off + n)
        self.numel = off
        self.flat_param = torch.zeros(self.numel, dtype=dtype, device=dev)
        self.flat_grad = torch.zeros(self.numel, dtype=dtype, device=dev)
        # Keep each parameter's memory layout (e.g. channels_last conv weights):
        # the flat slot holds the parameter's dense storage order and the view
        # re-applies its strides, so MIOpen sees the same NHWC weights.
        self.strides = []
        for p in ps:
            st = p.stride() if self._dense(p) else torch.empty(p.shape).stride()
            self.strides.append(st)
        with torch.no_grad():
            for i, (p, (o, n)) in enumerate(zip(ps, self.offsets)):
                v = self._view(self.flat_param, i)
                v.copy_(p.detach())
                p.data = v
                p.grad = self._view(self.flat_grad, i)
        self._index = {id(p): i for i, p in enumerate(ps)}
        # bf16 compute copy of flat_param (see parallel/mixed.py) and the
        # gradient sink that direct-gradient autograd functions deliver to.
        self.flat_shadow: Optional[torch.Tensor] = None
        self.shadow_gen = 0  # bumped by every refresh_shadow (caches derived from the shadow key on it)
        self._shadow_token = None  # set when an optimizer step wrote the shadow with the weights (mark_shadow_fresh)
        self.sink = None

    @staticmethod
    def _dense(p) -> bool:
        """True if p's strides are a permutation of a contiguous layout."""
        if p.numel() <= 1:
            return True
        dims = sorted((s, d) for d, s in zip(p.shape, p.stride()) if d != 1)
        expect = 1
        for s, d in dims:
            if s != expect:
                return False
            expect *= d
        return True

    def _view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        o, n = self.offsets[i]
        p = self.params[i]
        return torch.as_strided(flat, p.shape, self.strides[i], o)

    def index(self, p) -> int:
        return self._index[id(p)]

    def grad_view(self, i: int) -> torch.Tensor:
        return self._view(self.flat_grad, i)

    def param_view(self, i: int) -> torch.Tensor:
        return self._view(self.flat_param, i)

    def enable_shadow(self):
        if self.flat_shadow is None:
            self.flat_shadow = torch.empty(self.numel, dtype=torch.bfloat16, device=self.device)
            self.refresh_shadow()

    def _param_token(self):
        # what a later in-place weight update would change: the parameters' and the flat buffer's
        # version counters, and the epoch of the non-autograd writers (note_param_write)
        return (sum(p._version for p in self.params), self.flat_param._version, _PARAM_EPOCH[0])

    def mark_shadow_fresh(self):
        """The optimizer step that just ran also wrote flat_shadow = bf16(new flat_param) (ops.adam_step's
        shadow output): the next refresh_shadow skips its cast kernel unless the weights changed since."""
        self._shadow_token = self._param_token()

    @torch.no_grad()
    def refresh_shadow(self):
        """flat_shadow = bf16(flat_param): one cast kernel for the whole model (none when the optimizer
        step already wrote it and nothing touched the weights since, see mark_shadow_fresh)."""
        tok, self._shadow_token = self._shadow_token, None
        if (self.flat_shadow is not None and tok is not None and tok == self._param_token()
                and not (self.flat_param.is_cuda and torch.cuda.is_current_stream_capturing())):
            self.shadow_gen += 1
            return
        if self.flat_shadow is not None:
            # Version counter preserved: shadow views saved by a still-pending
            # backward (gradient accumulation over several forwards) stay valid;
            # the master does not change between micro-batches, so the values
            # they see are unchanged.
            with torch.autograd._unsafe_preserve_version_counter(self.flat_shadow):
                self.flat_shadow.copy_(self.flat_param)
            self.shadow_gen += 1

    def shadow_view(self, i: int) -> torch.Tensor:
        return self._view(self.flat_shadow, i)

    def zero_grad(self):
        self.flat_grad.zero_()
        self.rebind_grads()

    def rebind_grads(self):
        """Restore ``p.grad`` views if user code replaced or dropped them."""
        for i, p in enumerate(self.params):
            g = p.grad
            v = self.grad_view(i)
            if g is None or g.data_ptr() != v.data_ptr():
                if g is not None:
                    with torch.no_grad():
                        v.copy_(g)
                p.grad = v

    def check_params(self):
        """Re-home parameters whose ``.data`` was replaced (e.g. by load_state_dict copy semantics keep
        views, but ``p.data = t`` does not)."""
        with torch.no_grad():
            for i, p in enumerate(self.params):
                v = self.param_view(i)
                if p.data.data_ptr() != v.data_ptr():
                    v.copy_(p.data)
                    p.data = v

    def state_slices(self):
        return list(zip(self.params, self.offsets))


_PARAM_EPOCH = [0]


def note_param_write() -> None:
    """A weight buffer was (or may have been) written outside autograd's version counters (a HIP kernel,
    a collective): optimizer-written bf16 shadows are stale (FlatParamSpace.refresh_shadow recasts)."""
    _PARAM_EPOCH[0] += 1


def axpby_(y: torch.Tensor, x: torch.Tensor, a: float, b: float) -> torch.Tensor:
    """y <- a*y + b*x: one fused HIP kernel (K3/K4) on GPU, torch ops on CPU."""
    note_param_write()
    if y.is_cuda:
        from .._lib import hip

        hip().axpby(y, x, None, a, b)
    else:
        y.mul_(a).add_(x, alpha=b)
    return y


def sumsq(t: torch.Tensor, other: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[sum(t^2), sum(other^2)] (f32, on t's device): one-pass K5 kernel on GPU."""
    if t.is_cuda:
        from .._lib import hip

        return hip().sumsq2(t, other)
    a = t.double().square().sum()
    b = other.double().square().sum() if other is not None else torch.zeros((), dtype=torch.float64)
    return torch.stack([a, b]).float()
