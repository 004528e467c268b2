"""``F.linear`` whose weight gradient runs on the split-K MFMA kernel of conv_wgrad.hip.

A linear layer's weight gradient ``dW[o][i] = sum_t dy[t][o] x[t][i]`` over T = batch*seq tokens
is exactly the 1x1-convolution weight gradient over T "pixels" (both operands token-major,
the "NT" layout that kernel stages unchanged).  hipBLASLt's choices for these long-K, small
M x N products are poor on BERT-base at 16 K tokens (r8 profile: 768x768 out-projection 147 us
= 130 TF/s, 3072x768 FFN 185 us = 417 TF/s); the split-K kernel runs them as a 1x1 conv wgrad.
Forward and data gradient stay on hipBLASLt (``F.linear`` / ``mm``).

Eligible: CUDA bf16 activations and weight, in/out features multiples of 64, < 2^23 tokens;
anything else is plain ``F.linear``.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .._lib import hip, hip_available

_MAX_TOKENS = 1 << 23
_ENABLED = os.environ.get("KUNGFU_LINEAR_WGRAD", "1") != "0"


def _as_nhwc(t2: torch.Tensor) -> torch.Tensor:
    """[T, C] row-major -> [1, C, 1, T] channels_last view of the same memory."""
    T, C = t2.shape
    return t2.as_strided((1, C, 1, T), (T * C, 1, T * C, C))


class BiasLink:
    """Link from a linear layer's output to the ONE consumer that can produce the layer's bias
    gradient in its own backward pass (an AddLayerNorm with ``bias_link=True``: the column sums of
    the residual gradient it writes).  ``ptr`` lets the linear's backward check that the gradient it
    receives is exactly that tensor; otherwise it sums the columns itself."""
    __slots__ = ("dtype", "value", "ptr")

    def __init__(self, dtype):
        self.dtype, self.value, self.ptr = dtype, None, 0


class ResidualLink:
    """Link between the two consumers of a residual-stream tensor ``x`` in a transformer layer: a
    linear layer ``linear(x)`` and the AddLayerNorm that adds ``x`` back as its skip input.  The
    LayerNorm's backward runs first (it consumes the linear's descendants) and hands its gradient of
    ``x`` over instead of returning it; the linear's backward then forms the whole gradient of ``x``
    in ONE GEMM, ``g_skip.addmm_(dy, W)`` (hipBLASLt beta = 1 epilogue, in place) -- no separate residual add
    pass over the [tokens, d] gradient (25 launches per BERT-base step).  ``armed``: the linear's
    forward took the path that consumes the link (set before the LayerNorm's forward checks it)."""
    __slots__ = ("armed", "value")

    def __init__(self):
        self.armed, self.value = False, None


class GeluLink:
    """Link from ``gelu(u)`` to the ONE linear layer that consumes it (BERT's FC2): that layer's
    backward forms ``du = gelu'(u) * (dy W)`` inside its data-gradient GEMM (gemm.hip's GELU-gradient
    epilogue) together with the column sums of ``du`` -- the bias gradient of the layer that produced
    ``u``, handed on through its :class:`BiasLink` -- and returns ``du`` in place of the gradient of
    ``gelu(u)``; the GELU node then passes it through (``ptr`` checks that it receives exactly that
    tensor).  Replaces hipBLASLt's data-gradient GEMM plus the separate GELU-backward + column-sum pass."""
    __slots__ = ("u", "blink", "ptr")

    def __init__(self, u, blink):
        self.u, self.blink, self.ptr = u, blink, 0


_RES_LINK = True  # module switch (tests / A/B)
_GELU_GEMM = True  # module switch (tests / A/B): FC2's data gradient + GELU backward on gemm.hip
# (round 6: FC1's forward + GELU on one gemm.hip launch is gone -- measured slower end to end, BERT-base +
# GNS 15.58-15.69 -> 15.90-15.94 ms/step on one box, r5t34: the 256 x 256 NT GEMM stays behind hipBLASLt's
# stream-K kernel at that shape by more than the GELU pass it saves)


def residual_link(x: torch.Tensor):
    """Attach a fresh :class:`ResidualLink` to ``x`` (its two consumers pick it up) and return it."""
    if not (_RES_LINK and x.is_cuda and x.requires_grad and torch.is_grad_enabled()):
        return None
    rl = ResidualLink()
    x._kf_rlink = rl
    return rl


_DIRECT_WGRAD = True  # module switch (tests)
# direct weight gradients on the side stream (module switch): BERT-base + GNS 16.57-16.61 -> 16.45 ms/step
# on one box, two interleaved rounds (r5t30); the conv weight gradients measured the other way (mixed.SideStream)
_WGRAD_SIDE = True
# set_gemm_enabled(True): forward (x W^T + b) and data gradient (dy W, with W^T from the flat space's
# per-step multi-tensor transpose) on gemm.hip's pipelined NT GEMM instead of hipBLASLt -- measured
# slower (profiles/r4_gemm_nt.md), so off and not an environment knob any more (round 5)
_GEMM = False


def set_gemm_enabled(on: bool) -> bool:
    global _GEMM
    old, _GEMM = _GEMM, bool(on)
    return old


def _gemm_ok(M: int, K: int, N: int) -> bool:
    return _GEMM and hip().gemm_nt_supported(M, N, K)


def _wt_cache(target, w):
    """(flip cache, index) giving W^T [in, out] for the shadow weight ``w`` of flat-space parameter
    ``target`` -- the 1x1-conv "flip" of [out, in, 1, 1] is exactly the transpose -- refreshed by ONE
    multi-tensor kernel per optimizer step (ops.fused_block._FlipCache)."""
    from .fused_block import _flip_cache

    fc = _flip_cache(target[0])
    out_f, in_f = w.shape
    fc.register(target[1], w.view(out_f, in_f, 1, 1))
    return fc, target[1]


def _gelu_gemm_ok(M: int, in_f: int, out_f: int) -> bool:
    return _GELU_GEMM and in_f % 256 == 0 and hip().gemm_nt_supported(M, in_f, out_f)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, target=None, rlink=None, glink=None):
        ctx.save_for_backward(x, w)
        ctx.target = target
        ctx.rlink = rlink
        ctx.glink = ctx.wt_g = None
        if glink is not None and target is not None and rlink is None:
            out_f, in_f = w.shape
            if _gelu_gemm_ok(x.numel() // in_f, in_f, out_f):
                ctx.glink, ctx.wt_g = glink, _wt_cache(target, w)
        if rlink is not None:
            rlink.armed = True
        ctx.has_b = b is not None
        ctx.b_dtype = b.dtype if b is not None else None
        ctx.blink = BiasLink(b.dtype) if b is not None and b.dtype in (torch.bfloat16, torch.float32) else None
        out_f, in_f = w.shape
        M = x.numel() // in_f
        ctx.wt = None
        if _gemm_ok(M, in_f, out_f) and x.is_contiguous() and (b is None or b.dtype == torch.bfloat16):
            if target is not None and _gemm_ok(M, out_f, in_f):
                ctx.wt = _wt_cache(target, w)
            return hip().gemm_nt(x.view(M, in_f), w, b).view(*x.shape[:-1], out_f)
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        out_f, in_f = w.shape
        dy2 = dy.reshape(-1, out_f)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        x2 = x.reshape(-1, in_f)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            rl, g = ctx.rlink, None
            if rl is not None and rl.value is not None:  # the consuming AddLayerNorm's skip gradient
                g, rl.value = rl.value.reshape(-1, in_f), None
            gl = ctx.glink
            if gl is not None:
                # x = gelu(u): du = gelu'(u) * (dy . W) and u's layer's bias gradient in one GEMM (W^T from
                # the flat space's per-step transpose); the GELU node passes du through
                fc, i = ctx.wt_g
                bl = gl.blink
                du, dbu = hip().gemm_nt_gelu_grad(dy2, fc.get(i).view(in_f, out_f), gl.u.reshape(-1, in_f),
                                                  bl.dtype if bl is not None else torch.float32)
                gl.ptr = du.data_ptr()
                if bl is not None:
                    bl.value, bl.ptr = dbu, du.data_ptr()
                dx = du.view(x.shape)
            elif ctx.wt is not None:  # dx = dy . W = dy . (W^T)^T on the NT GEMM
                fc, i = ctx.wt
                dx = hip().gemm_nt(dy2, fc.get(i).view(in_f, out_f))
                if g is not None:
                    dx += g
                dx = dx.view(x.shape)
            elif g is not None:
                # added by the GEMM itself (beta = 1), IN PLACE: torch.addmm into a new tensor copies
                # g first (a 25 MB D2D copy per BERT-base product, measured slower than the add it
                # replaces).  g is the AddLayerNorm's own backward output; when it also went out as
                # the residual branch's gradient (no dropout) that branch's backward consumed it
                # earlier on this stream -- but its weight gradient may still be reading it on the side
                # stream: wait for that first
                from ..parallel.mixed import SideStream

                SideStream.before_write(g)
                dx = g.addmm_(dy2, w).view(x.shape)
            else:
                dx = torch.mm(dy2, w).view(x.shape)
        tgt = ctx.target
        if ctx.needs_input_grad[1] and tgt is not None and _DIRECT_WGRAD and hasattr(tgt[0].sink, "put_direct"):
            # the split-K partials are reduced straight into the weight's flat f32 gradient slot
            # (deterministic, accumulating): no bf16 weight gradient, no landing pass
            space, i = tgt
            gv = space.grad_view(i)

            def wg():
                hip().conv_wgrad(_as_nhwc(dy2), _as_nhwc(x2), 1, 1,
                                 out=gv.as_strided((out_f, in_f, 1, 1), (in_f, 1, in_f, in_f)),
                                 accumulate=True, atomics=False)  # deterministic partials + reduce (atomics: -3 %, r4t29)

            if _WGRAD_SIDE and dy2.is_cuda and not torch.cuda.is_current_stream_capturing():
                # on the side stream: the split-K kernel and its (memory-bound) reduce overlap the next
                # layers' data-gradient GEMMs; the bucket launch / end of backward joins it
                from ..parallel.mixed import SideStream

                main = torch.cuda.current_stream()
                side = SideStream.stream(dy2.device)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    wg()
                    ev = torch.cuda.Event()
                    ev.record(side)
                dy2.record_stream(side)
                x2.record_stream(side)
                SideStream._pending.append(ev)
                SideStream.note_reads(ev, dy2, x2)
            else:
                wg()
            space.sink.put_direct(i)
        elif ctx.needs_input_grad[1]:
            dw = hip().conv_wgrad(_as_nhwc(dy2), _as_nhwc(x2), 1, 1).view(out_f, in_f)
        bl = ctx.blink
        if bl is not None and bl.value is not None and bl.ptr == dy2.data_ptr() and ctx.needs_input_grad[2]:
            db = bl.value  # produced by the consuming LayerNorm's backward pass
            bl.value, bl.ptr = None, 0
        elif ctx.has_b and ctx.needs_input_grad[2]:
            # bias gradient: deterministic two-stage column sum (norms.hip; torch's reduce took
            # 26 us per BERT-base layer product at 16 K tokens)
            if dy2.dtype == torch.bfloat16:
                db = hip().colsum(dy2, ctx.b_dtype)
            else:
                db = dy2.sum(0, dtype=torch.float32).to(ctx.b_dtype)
        return dx, dw, db, None, None, None


def eligible(x: torch.Tensor, w: torch.Tensor) -> bool:
    if not (_ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.dim() == 2):
        return False
    out_f, in_f = w.shape
    if out_f % 64 or in_f % 64 or x.shape[-1] != in_f or x.numel() // in_f >= _MAX_TOKENS:
        return False
    return hip_available() and hip().conv_wgrad_supported(int(in_f), int(out_f), 1, 1)


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor = None, grad_target=None) -> torch.Tensor:
    """``F.linear(x, w, b)`` with the MFMA split-K weight gradient when eligible.  ``grad_target``
    ``(space, index)``: ``w`` is the bf16 shadow of that flat-space parameter -- its gradient is
    reduced straight into the parameter's f32 gradient slot (``space.sink.put_direct``)."""
    if eligible(x, w) and (b is None or b.dtype in (torch.bfloat16, torch.float32)):
        rl = getattr(x, "_kf_rlink", None)
        if rl is not None and (rl.armed or x.dtype != torch.bfloat16):
            rl = None  # one linear consumer per link
        gl = getattr(x, "_kf_glink", None)
        y = _LinearFn.apply(x, w, b, grad_target, rl, gl)
        if y.grad_fn is not None and getattr(y.grad_fn, "blink", None) is not None:
            y._kf_blink = y.grad_fn.blink
        return y
    return F.linear(x, w, b)


class _GeluFn(torch.autograd.Function):
    """``F.gelu(u)`` whose backward is ONE HIP pass (norms.hip gelu_bwd_colsum): du and its column
    sums -- the bias gradient of the linear layer that produced ``u`` (handed to that layer's
    backward through its :class:`BiasLink`, which then skips its own column-sum pass)."""

    @staticmethod
    def forward(ctx, u, blink, glink):
        ctx.save_for_backward(u)
        ctx.blink = blink
        ctx.glink = glink
        return F.gelu(u)  # a HIP erf-GELU forward measured 0.6 % slower end to end (r4t20): torch's

    @staticmethod
    def backward(ctx, dy):
        gl = ctx.glink
        if gl is not None and gl.ptr:
            # the consuming linear already formed du (and u's layer's bias gradient) in its GEMM
            if dy.data_ptr() != gl.ptr:
                raise RuntimeError("gelu: the gradient received is not the consuming linear's fused GELU gradient "
                                   "(gelu(u) must have that linear as its only consumer)")
            gl.ptr = 0
            return dy, None, None
        (u,) = ctx.saved_tensors
        bl = ctx.blink
        du, db = hip().gelu_backward_colsum(dy.contiguous(), u, bl.dtype if bl is not None else torch.float32)
        if bl is not None:
            bl.value, bl.ptr = db, du.data_ptr()
        return du, None, None


_GELU_LINK = True  # module switch (tests)


def gelu(u: torch.Tensor, bias_link: bool = False) -> torch.Tensor:
    """``F.gelu(u)``; with ``bias_link`` (the caller guarantees ``u`` is a :func:`linear` output consumed
    only here) the backward also produces that layer's bias gradient in the same pass."""
    bl = getattr(u, "_kf_blink", None) if bias_link and _GELU_LINK else None
    if (u.is_cuda and u.dtype == torch.bfloat16 and u.is_contiguous() and u.shape[-1] % 8 == 0 and hip_available()
            and (bl is not None or not bias_link)):
        # bias_link also promises that gelu(u) has one consumer: a linear layer may fuse the GELU
        # backward into its data-gradient GEMM (GeluLink)
        gl = GeluLink(u, bl) if bias_link and _GELU_GEMM and torch.is_grad_enabled() else None
        h = _GeluFn.apply(u, bl, gl)
        if gl is not None:
            h._kf_glink = gl
        return h
    return F.gelu(u)

