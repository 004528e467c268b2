"""3x3 convolutions on the hand-written MFMA implicit-GEMM kernel (csrc/kernels/conv.hip).

``conv3x3(x, w, stride)`` computes ``F.conv2d(x, w, stride=stride, padding=1)`` for NHWC
(channels_last) bf16 tensors with Cin, Cout multiples of 64:

* forward: ``_hip.conv3x3`` (stride 1 or 2);
* data gradient, stride 1: the same kernel on the flipped/transposed weights
  (``dx = conv3x3(dy, w')``, ``w'[ci,co,kh,kw] = w[co,ci,2-kh,2-kw]``);
  stride 2: MIOpen (``aten.convolution_backward``);
* weight gradient: the split-K MFMA kernel (csrc/kernels/conv_wgrad.hip, ``wgrad`` below,
  also used by the fused bottleneck blocks) for 1x1 / 3x3, stride 1 / 2.

Measured per ResNet-50 shape against MIOpen in ``tools/bench_conv3x3.py`` and
``tools/bench_wgrad.py`` (profiles/README.md).  Set ``KUNGFU_CONV3X3=0`` to route the 3x3
forward / data gradient through MIOpen, ``KUNGFU_WGRAD=0`` the weight gradients.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._lib import buf_ok, hip, hip_available

_ENABLED = os.environ.get("KUNGFU_CONV3X3", "1") != "0"
_WGRAD = os.environ.get("KUNGFU_WGRAD", "1") != "0"
_WGRAD_MAX_PIXELS = 1 << 31  # test hook; the kernels' own cap: hip().conv_wgrad_max_pixels


def set_wgrad_enabled(on: bool) -> bool:
    """Turn the MFMA weight-gradient path on/off at run time; returns the previous setting."""
    global _WGRAD
    old, _WGRAD = _WGRAD, bool(on)
    return old


def _cl4(t: torch.Tensor) -> bool:
    return t.dim() == 4 and t.dtype == torch.bfloat16 and t.is_contiguous(memory_format=torch.channels_last)


def wgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> torch.Tensor:
    """Weight gradient of ``F.conv2d(x, w, stride=stride, padding=pad)`` (bf16, w's shape).

    The MFMA split-K kernel for NHWC bf16 1x1 / 3x3 (pad (ks-1)/2) convolutions with
    channel counts that are multiples of 64; MIOpen otherwise."""
    ks = int(w.shape[2])
    if (_WGRAD and x.is_cuda and _cl4(x) and _cl4(dy) and w.dim() == 4 and w.shape[3] == ks
            and pad == (ks - 1) // 2 and hip_available()
            and hip().conv_wgrad_supported(int(x.shape[1]), int(dy.shape[1]), ks, int(stride))):
        n = int(x.shape[0])
        per_img = int(dy.shape[2]) * int(dy.shape[3])
        cap = min(_WGRAD_MAX_PIXELS, hip().conv_wgrad_max_pixels(n, int(x.shape[2]), int(x.shape[3]), int(x.shape[1]),
                                                                 int(dy.shape[1]), ks, int(stride)))
        if n * per_img < cap:
            return hip().conv_wgrad(dy, x, ks, int(stride))
        # the tap-tiled kernel's pixel index math holds < 2^23 output pixels per launch: sum over
        # batch chunks into one f32 gradient (the row-image 3x3 kernel has no such cap)
        step = max(1, (cap - 1) // per_img)
        acc = torch.zeros(w.shape, dtype=torch.float32, device=x.device).contiguous(
            memory_format=torch.channels_last)
        for i in range(0, n, step):
            hip().conv_wgrad(dy[i:i + step], x[i:i + step], ks, int(stride), out=acc, accumulate=True,
                             atomics=False)  # deterministic (split-K partials + reduce)
        return acc.to(torch.bfloat16)
    return torch.ops.aten.convolution_backward(dy, x, w, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1,
                                               [False, True, False])[1]


def set_enabled(on: bool) -> bool:
    """Turn the MFMA 3x3 path on/off at run time; returns the previous setting."""
    global _ENABLED
    old, _ENABLED = _ENABLED, bool(on)
    return old


def eligible(x: torch.Tensor, w: torch.Tensor, stride, padding, dilation, groups) -> bool:
    if not _ENABLED or not x.is_cuda or groups != 1:
        return False
    st = stride if isinstance(stride, int) else (stride[0] if stride[0] == stride[1] else -1)
    pd = padding if isinstance(padding, int) else (padding[0] if padding[0] == padding[1] else -1)
    dl = dilation if isinstance(dilation, int) else (dilation[0] if dilation[0] == dilation[1] else -1)
    if st not in (1, 2) or pd != 1 or dl != 1:
        return False
    if w.dim() != 4 or w.shape[2] != 3 or w.shape[3] != 3 or x.dim() != 4:
        return False
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if not x.is_contiguous(memory_format=torch.channels_last):
        return False
    if not w.is_contiguous(memory_format=torch.channels_last):
        return False
    if not hip_available() or not buf_ok(x.numel(), w.numel()):
        return False
    return hip().conv3x3_supported(int(x.shape[1]), int(w.shape[0]), int(st))


class _Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride):
        ctx.save_for_backward(x, w)
        ctx.stride = stride
        return hip().conv3x3(x, w, stride)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        s = ctx.stride
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        need_dx, need_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dx = dw = None
        if need_dx and s == 1:
            dx = hip().conv3x3(dy, hip().conv3x3_flip_weight(w), 1)
            need_dx = False
        if need_dw:
            dw = wgrad(dy, x, w, s, 1)
        if need_dx:
            dx = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                     [True, False, False])[0]
        return dx, dw, None


def conv3x3(x: torch.Tensor, w: torch.Tensor, stride: int = 1) -> torch.Tensor:
    """3x3, padding 1 convolution (MFMA kernel when eligible, else F.conv2d)."""
    if eligible(x, w, stride, 1, 1, 1):
        return _Conv3x3Fn.apply(x, w, int(stride if isinstance(stride, int) else stride[0]))
    return F.conv2d(x, w, stride=stride, padding=1)


class _BiasActFn(torch.autograd.Function):
    """y = relu(y + b) in place on a conv output (csrc/kernels/bias_act.hip); backward is one
    pass producing dy * (y > 0) and its per-channel sum (the bias gradient).

    Determinism: the per-channel bias-gradient sum is per-block partials plus a fixed-order
    column sum -- bitwise reproducible, no zero-fill of the output (round 5: the previous f32
    atomics into a hipMemsetAsync-zeroed buffer made VGG-16's per-layer step vary, and go NaN,
    under whole-step capture; tests/test_gpu_engine.py captured-vs-eager VGG test).  The
    ReLU keeps NaN (``!(v <= 0)``), as ``torch.relu`` does."""

    @staticmethod
    def forward(ctx, y, b, relu):
        hip().bias_act_forward_(y, b, relu)
        ctx.mark_dirty(y)
        ctx.save_for_backward(y)
        ctx.relu = relu
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dz, db = hip().bias_act_backward(dy.contiguous(memory_format=torch.channels_last), y, ctx.relu)
        return dz, db, None


def _pair(v):
    return (int(v), int(v)) if isinstance(v, int) else (int(v[0]), int(v[1]))


def rect_eligible(x: torch.Tensor, w: torch.Tensor, stride, padding, dilation, groups) -> bool:
    """KH x KW windows the MFMA kernel takes (1x1, 3x3, 1x7, 7x1, 1x3, 3x1, 5x5; Cin, Cout
    multiples of 64, equal strides 1|2, padding < window): Inception-v3's convolutions."""
    if not (_ENABLED and _RECT) or not x.is_cuda or groups != 1 or w.dim() != 4 or x.dim() != 4:
        return False
    st, pd, dl = _pair(stride), _pair(padding), _pair(dilation)
    if st[0] != st[1] or dl != (1, 1) or pd[0] >= w.shape[2] or pd[1] >= w.shape[3]:
        return False
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or not hip_available():
        return False
    if not x.is_contiguous(memory_format=torch.channels_last) or not w.is_contiguous(memory_format=torch.channels_last):
        return False
    if not buf_ok(x.numel(), w.numel()):
        return False
    return hip().conv_rect_supported(int(x.shape[1]), int(w.shape[0]), int(w.shape[2]), int(w.shape[3]), st[0])


class _ConvRectFn(torch.autograd.Function):
    """KH x KW convolution on the MFMA kernel (``_hip.conv_rect``).  Backward: stride 1 data
    gradient = the same kernel on the flipped weights with padding (KH-1-ph, KW-1-pw); stride 2
    via MIOpen; weight gradient on the split-K MFMA kernel (:func:`wgrad` for the ResNet-shaped
    1x1 / 3x3-pad-1 ones, ``_hip.conv_wgrad_rect`` for any other window / channel count).
    ``stats``: the BN statistics workspace of a following BN (epilogue sums, see ``bn_act``)."""

    @staticmethod
    def forward(ctx, x, w, stride, ph, pw, stats, flip=None):
        ctx.save_for_backward(x, w)
        ctx.geo = (stride, ph, pw)
        ctx.flip = flip
        ctx.link = getattr(x, "_kf_link", None)  # x = a BN+ReLU output with this conv its only consumer
        return hip().conv_rect(x, w, stride, ph, pw, stats)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        s, ph, pw = ctx.geo
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        kh, kw = int(w.shape[2]), int(w.shape[3])
        if ctx.needs_input_grad[0]:
            if s == 1:
                # flipped weights: from the flat space's per-step multi-tensor flip when registered
                wt = ctx.flip[0].get(ctx.flip[1]) if ctx.flip is not None else hip().conv_flip_weight(w)
                dx = _dgrad_link(dy, wt, kh - 1 - ph, kw - 1 - pw, None, ctx.link)
            elif s == 2 and kh == kw == 3 and ph == pw and ph in (0, 1) and min(x.shape[1], dy.shape[1]) >= 16:
                # parity-phase GEMMs for any input size (Inception's 3x3/s2/p0 on 25x25 / 12x12 maps)
                wt = ctx.flip[0].get(ctx.flip[1]) if ctx.flip is not None else hip().conv_flip_weight(w)
                H = hip()
                lk = ctx.link
                if lk is not None and lk.y is not None:
                    dx = H.conv_dgrad_s2(dy, wt, 3, lk.ws, lk.y, lk.coef, None, -1, int(x.shape[2]), int(x.shape[3]), ph)
                    lk.ready, lk.dx_ptr = True, dx.data_ptr()
                else:
                    dx = H.conv_dgrad_s2(dy, wt, 3, dh=int(x.shape[2]), dw=int(x.shape[3]), pad=ph)
            else:
                dx = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [ph, pw], [1, 1], False, [0, 0], 1,
                                                         [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            dw = _rect_wgrad(dy, x, w, s, ph, pw)
        return dx, dw, None, None, None, None, None


def _dgrad_link(dy, wt, ph, pw, out, link):
    """Stride-1 data gradient ``conv_rect(dy, wt)`` (accumulated into ``out`` if given); with a
    :class:`~kungfu_amd.ops.fused_bn.BNLink` its epilogue also produces the backward sums of
    the BN that made the conv input (that BN's backward then skips its reduction)."""
    if link is None or link.y is None:
        return hip().conv_rect(dy, wt, 1, ph, pw, None, out)
    dx = hip().conv_rect(dy, wt, 1, ph, pw, link.ws, out, link.y, link.coef)
    link.ready, link.dx_ptr = True, dx.data_ptr()
    return dx


def _rect_wgrad(dy, x, w, s, ph, pw):
    """Weight gradient of a KH x KW convolution: the ResNet-tuned planner for 1x1 / 3x3-pad-1 with
    channels % 64, the runtime-window split-K kernel for other wide layers, MIOpen for narrow ones."""
    kh, kw = int(w.shape[2]), int(w.shape[3])
    cin, cout = int(x.shape[1]), int(dy.shape[1])
    if kh == kw and ph == pw == (kh - 1) // 2 and cin % 64 == 0 and cout % 64 == 0:
        return wgrad(dy, x, w, s, ph)  # ResNet-tuned planner (row-image 3x3 kernel etc.)
    # measured per Inception-v3 shape (tools/bench_inception_wgrad.py, profiles/r3q_inception_wgrad.txt):
    # the split-K kernel wins every 1x1 (2-3x) and the multi-tap windows over >= 256 input
    # channels; the narrow stride-1 multi-tap ones (32..192 inputs) take the row-image kernel
    # (all taps of a workgroup share one staged input image: 54x54 80->192 3x3 992 -> 405 us,
    # 111x111 32->32 3x3 438 -> 167 us on 32-channel tiles, 12x12 160->160 1x7 79 -> 55 us vs
    # MIOpen, profiles/r5_inception_wgrad.md)
    if (_WGRAD and _WGRAD_RECT and s == 1 and kh * kw > 1 and cin <= 192
            and hip().conv_wgrad_rows_rect_supported(int(x.shape[0]), int(x.shape[2]), int(x.shape[3]), cin, cout,
                                                     kh, kw, ph, pw, 1)):
        return hip().conv_wgrad_rect(dy, x, kh, kw, 1, ph, pw, 13)  # 13: the per-shape row-image variant
    if (_WGRAD and _WGRAD_RECT and s == 2 and kh * kw > 1
            and hip().conv_wgrad_rows_rect_supported(int(x.shape[0]), int(x.shape[2]), int(x.shape[3]), cin, cout,
                                                     kh, kw, ph, pw, 2)):
        # the stride-2 windows (Mixed_6a / 7a reductions) on the row-image ring variants: 96->96 on
        # 25x25 34 vs MIOpen 50 us, 288->384 241 vs 266 tap-tiled (profiles/r5_inception_wgrad.md)
        return hip().conv_wgrad_rect(dy, x, kh, kw, 2, ph, pw, 13)
    wide = kh * kw == 1 or cin % 128 == 0 or cin >= 256
    if (_WGRAD and _WGRAD_RECT and wide and min(cin, cout) >= 32 and hip().conv_wgrad_rect_supported(cin, cout, kh, kw, s)
            and int(dy.shape[0]) * int(dy.shape[2]) * int(dy.shape[3]) < (1 << 23)):
        return hip().conv_wgrad_rect(dy, x, kh, kw, s, ph, pw)
    return torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [ph, pw], [1, 1], False, [0, 0], 1,
                                               [False, True, False])[1]


class _SiblingConvFn(torch.autograd.Function):
    """Stride-1 convolutions that all read the same input (the branch heads of an Inception
    block) as ONE autograd node: forward = one MFMA conv per sibling (BN statistics in each
    epilogue when a workspace is given); backward = their data gradients chained into one dx by
    the kernel's accumulate epilogue (no autograd adds of the branch gradients: one pass each
    fewer), weight gradients per sibling."""

    @staticmethod
    def forward(ctx, x, pads, stats, flips, *ws):
        ys = tuple(hip().conv_rect(x, w, 1, ph, pw, st) for w, (ph, pw), st in zip(ws, pads, stats))
        ctx.save_for_backward(x, *ws)
        ctx.pads, ctx.flips = pads, flips
        ctx.link = getattr(x, "_kf_link", None)
        return ys

    @staticmethod
    def backward(ctx, *dys):
        x, *ws = ctx.saved_tensors
        dx = None
        dws = []
        last = max((i for i, d in enumerate(dys) if d is not None), default=-1)
        for i, (w, dy, (ph, pw), fl) in enumerate(zip(ws, dys, ctx.pads, ctx.flips)):
            if dy is None:
                dws.append(None)
                continue
            if not dy.is_contiguous(memory_format=torch.channels_last):
                dy = dy.contiguous(memory_format=torch.channels_last)
            if ctx.needs_input_grad[0]:
                wt = fl[0].get(fl[1]) if fl is not None else hip().conv_flip_weight(w)
                kh, kw = int(w.shape[2]), int(w.shape[3])
                # dx += (first: =); the last one completes dx, so its epilogue may take the BN sums
                dx = _dgrad_link(dy, wt, kh - 1 - ph, kw - 1 - pw, dx, ctx.link if i == last else None)
            dws.append(_rect_wgrad(dy, x, w, 1, ph, pw))
        return (dx, None, None, None, *dws)


def sibling_convs(x, convs, stats):
    """``[conv(x) for conv in convs]`` for nn.Conv2d modules (no bias, stride 1) on the MFMA
    kernel as one autograd node (:class:`_SiblingConvFn`); ``stats[i]``: BN statistics workspace
    for conv i's output or None.  Takes the bf16 shadow weights.  Returns None when any conv is
    not eligible (the caller runs the modules one by one)."""
    from ..parallel.mixed import direct_target, shadow

    ws, pads, flips = [], [], []
    for c in convs:
        if c.bias is not None or _pair(c.stride) != (1, 1):
            return None
        w = shadow(c.weight)
        if not rect_eligible(x, w, 1, c.padding, c.dilation, c.groups):
            return None
        ws.append(w)
        pads.append(_pair(c.padding))
        tc = direct_target(c.weight)
        if tc is not None and w is not c.weight:
            from .fused_block import _flip_cache

            fc = _flip_cache(tc[0])
            fc.register(tc[1], w)
            flips.append((fc, tc[1]))
        else:
            flips.append(None)
    return _SiblingConvFn.apply(x, tuple(pads), tuple(stats), tuple(flips), *ws)


_RECT = os.environ.get("KUNGFU_CONV_RECT", "1") != "0"
_WGRAD_RECT = os.environ.get("KUNGFU_WGRAD_RECT", "1") != "0"


def conv2d_stats(x, w, stride, padding, stats: torch.Tensor, master: torch.Tensor = None):
    """conv2d whose MFMA epilogue also accumulates the per-channel batch statistics of its bf16
    output into ``stats`` (a following BN's workspace, ``BatchNormAct2d.stats_workspace``).
    ``master``: the f32 parameter ``w`` shadows -- its flipped copy for the data gradient then
    comes from the flat space's one-launch-per-step multi-tensor flip.
    Returns None when the shape is not on the MFMA kernel (the caller runs the plain path)."""
    if not rect_eligible(x, w, stride, padding, 1, 1):
        return None
    st, pd = _pair(stride), _pair(padding)
    flip = None
    if master is not None:
        from ..parallel.mixed import direct_target
        from .fused_block import _flip_cache

        tc = direct_target(master)
        if tc is not None and w is not master:
            fc = _flip_cache(tc[0])
            fc.register(tc[1], w)
            flip = (fc, tc[1])
    return _ConvRectFn.apply(x, w, st[0], pd[0], pd[1], stats, flip)


def conv2d(x, w, bias, stride, padding, dilation, groups, relu: bool = False):
    """F.conv2d (+ ReLU) with the MFMA fast paths: 3x3/pad 1 (there the bias (+ ReLU) is one
    in-place HIP pass over the conv output, ``_BiasActFn``, when the channel count allows) and
    the other KH x KW windows of :func:`rect_eligible` (no bias)."""
    if bias is None and not eligible(x, w, stride, padding, dilation, groups) and \
            rect_eligible(x, w, stride, padding, dilation, groups):
        st, pd = _pair(stride), _pair(padding)
        y = _ConvRectFn.apply(x, w, st[0], pd[0], pd[1], None)
        return F.relu(y) if relu else y
    if eligible(x, w, stride, padding, dilation, groups):
        y = _Conv3x3Fn.apply(x, w, int(stride if isinstance(stride, int) else stride[0]))
        if bias is not None and hip().bias_act_supported(int(y.shape[1])):
            return _BiasActFn.apply(y, bias.float().contiguous(), bool(relu))
        if bias is not None:
            y = y + bias.view(1, -1, 1, 1).to(y.dtype)
        return F.relu(y) if relu else y
    y = F.conv2d(x, w, bias, stride, padding, dilation, groups)
    return F.relu(y) if relu else y


class Conv2dReLU(nn.Conv2d):
    """relu(conv2d(x) + bias) as one module (VGG's conv -> ReLU pairs): on the MFMA path the
    bias and ReLU are fused into one pass.  Takes the bf16 shadow weights itself
    (``kf_shadow_forward``: parallel/mixed.py registers its parameters, keeps this forward)."""

    kf_shadow_forward = True

    def forward(self, x):
        from ..parallel.mixed import shadow

        w = shadow(self.weight)
        b = shadow(self.bias) if self.bias is not None else None
        if self.padding_mode == "zeros" and x.dtype == torch.bfloat16:
            return conv2d(x, w, b, self.stride, self.padding, self.dilation, self.groups, relu=True)
        if b is not None and x.is_cuda and hip_available() and hip().bias_act_supported(self.out_channels):
            # e.g. the f32-image first layer under autocast: library conv, then the fused pass
            y = self._conv_forward(x, w, None)
            if y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last):
                return _BiasActFn.apply(y, b.float().contiguous(), True)
            return F.relu(y + b.view(1, -1, 1, 1).to(y.dtype))
        return F.relu(self._conv_forward(x, w, b))
