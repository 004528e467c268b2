"""ResNet stem convolution (7x7, stride 2, pad 3, 3 -> 64) on the hand-written MFMA kernels
of ``csrc/kernels/stem.hip``.

``stem_conv(x, w, stats)`` computes ``F.conv2d(x, w, stride=2, padding=3)`` for an NHWC
image batch (f32 or bf16, channels_last) and bf16 weights, and -- when ``stats`` (the
following BN's f64 slotted sums workspace, ``fused_block._sums``) is given -- accumulates
the BN batch statistics in the conv epilogue, so ``bn_pool_forward(..., sums=stats)`` skips
its statistics pass.  The image is cast to bf16 and padded to 4 channels in one pass; the
weight gradient is the split-K MFMA kernel; the image gets no gradient.

Set ``KUNGFU_STEM=0`` to use MIOpen.  No reference counterpart (the reference trains
``tf.keras.applications`` ResNet-50, ``benchmarks/system/benchmark_kungfu.py:96``).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from .._lib import hip, hip_available

_ENABLED = os.environ.get("KUNGFU_STEM", "1") != "0"
# Stem conv + BN + ReLU + MaxPool as one autograd node whose weight gradient forms the BN input
# gradient while staging (``_StemBlockFn``) instead of the layered BN-pool backward + weight gradient.
FUSED_BACKWARD = True


def set_enabled(on: bool) -> bool:
    global _ENABLED
    old, _ENABLED = _ENABLED, bool(on)
    return old


def eligible(conv: torch.nn.Conv2d, x: torch.Tensor) -> bool:
    if not (_ENABLED and x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and not x.requires_grad):
        return False
    if x.dtype not in (torch.float32, torch.bfloat16) or not x.is_contiguous(memory_format=torch.channels_last):
        return False
    # the output is bf16: only where the conv would compute in bf16 anyway (bf16 input or autocast)
    if x.dtype != torch.bfloat16 and not (torch.is_autocast_enabled("cuda") and
                                          torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    if not (conv.in_channels == 3 and conv.out_channels == 64 and conv.kernel_size == (7, 7)
            and conv.stride == (2, 2) and conv.padding == (3, 3) and conv.dilation == (1, 1)
            and conv.groups == 1 and conv.bias is None and conv.padding_mode == "zeros"):
        return False
    return x.shape[2] >= 4 and x.shape[3] >= 4 and hip_available()


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stats):
        H = hip()
        x4 = H.stem_pad4(x)
        wb = w if w.dtype == torch.bfloat16 else w.to(torch.bfloat16)
        if not wb.is_contiguous(memory_format=torch.channels_last):
            wb = wb.contiguous(memory_format=torch.channels_last)
        y = H.stem_forward(x4, H.stem_pack_weight(wb), stats)
        ctx.save_for_backward(x4)
        ctx.wdtype = w.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        (x4,) = ctx.saved_tensors
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        dw = hip().stem_wgrad(dy, x4) if ctx.needs_input_grad[1] else None
        if dw is not None and dw.dtype != ctx.wdtype:
            dw = dw.to(ctx.wdtype)
        return None, dw, None


def stem_conv(x: torch.Tensor, w: torch.Tensor, stats: Optional[torch.Tensor] = None) -> torch.Tensor:
    """conv7x7/2 pad 3 of an NHWC image (f32/bf16) -> bf16 [N, 64, OH, OW] channels_last."""
    return _StemFn.apply(x, w, stats)


class _StemBlockFn(torch.autograd.Function):
    """maxpool3x3s2p1(relu(bn(conv7x7s2p3(x)))) as ONE autograd node.  Backward: the BN+ReLU+pool
    backward runs only its statistics + finalize (``bn_pool_backward(apply=False)``: the BN
    gamma/beta gradients and the coefficients k1, k2, k3 of ``dx = k1 dz + k2 y + k3``), then the
    stem weight-gradient kernel FORMS dx while staging its dy operand (``stem_wgrad_bnp``: pool
    gather + ReLU gate + BN backward from dyp, the argmax bytes and y) -- the BN input gradient
    (411 MB at batch 256) is never written nor read back."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, running_mean, running_var, momentum, eps, training, nbt, sums):
        from .fused_bn import _direct

        H = hip()
        x4 = H.stem_pad4(x)
        wb = w if w.dtype == torch.bfloat16 else w.to(torch.bfloat16)
        if not wb.is_contiguous(memory_format=torch.channels_last):
            wb = wb.contiguous(memory_format=torch.channels_last)
        st = sums if training else None
        y = H.stem_forward(x4, H.stem_pack_weight(wb), st)
        yp, mean, invstd, coef, arg, xarg = H.bn_pool_forward(y, gamma, beta, running_mean, running_var, momentum,
                                                              eps, training, nbt, st)
        ctx.save_for_backward(x4, y, mean, invstd, gamma, coef, arg, xarg)
        ctx.training = training
        ctx.wdtype = w.dtype
        ctx.direct = _direct(gamma, beta)
        return yp

    @staticmethod
    def backward(ctx, dyp):
        from .fused_bn import _param_grads

        x4, y, mean, invstd, gamma, coef, arg, xarg = ctx.saved_tensors
        H = hip()
        if not dyp.is_contiguous(memory_format=torch.channels_last):
            dyp = dyp.contiguous(memory_format=torch.channels_last)
        _, dg, db, bcoef = H.bn_pool_backward(dyp, arg, y, mean, invstd, gamma, coef, ctx.training, xarg,
                                              apply=False)
        dw = H.stem_wgrad_bnp(y, x4, dyp, arg, coef, bcoef)
        dg, db = _param_grads(ctx, dg, db)
        if dw.dtype != ctx.wdtype:
            dw = dw.to(ctx.wdtype)
        return None, dw, dg, db, None, None, None, None, None, None, None


def block_eligible(x: torch.Tensor, bn) -> bool:
    """The fused stem node applies: training with batch statistics and an image the row kernel
    takes (``stem_wgrad_bnp_supported``)."""
    return (FUSED_BACKWARD and bn.training and bn.track_running_stats and bn.momentum is not None
            and hip().stem_wgrad_bnp_supported(x.shape[0], x.shape[2], x.shape[3]))


def stem_block(x: torch.Tensor, w: torch.Tensor, bn, sums: Optional[torch.Tensor]) -> torch.Tensor:
    """ResNet stem ``maxpool(relu(bn(conv(x))))`` on the fused kernels; ``bn`` is the fused
    ``BatchNormAct2d`` (its parameters, running statistics and ``num_batches_tracked``)."""
    (gamma, beta, rm, rv, use_batch, momentum, eps), nbt = bn._args()
    return _StemBlockFn.apply(x, w, gamma, beta, rm, rv, momentum, eps, use_batch, nbt, sums)


# ---------------------------------------------------------------------------------------------
# Small image stems (csrc/kernels/stem3.hip): a <= 4x4 window over the 3-channel image, 32 output
# channels, any stride / zero padding -- Inception-v3's Conv2d_1a (3x3, stride 2, no padding).


def stem3_eligible(conv: torch.nn.Conv2d, x: torch.Tensor) -> bool:
    if not (_ENABLED and x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and not x.requires_grad):
        return False
    if x.dtype not in (torch.float32, torch.bfloat16) or not x.is_contiguous(memory_format=torch.channels_last):
        return False
    if x.dtype != torch.bfloat16 and not (torch.is_autocast_enabled("cuda") and
                                          torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    kh, kw = conv.kernel_size
    sh, sw = conv.stride
    ph, pw = conv.padding
    if not (conv.in_channels == 3 and conv.out_channels == 32 and kh <= 4 and kw <= 4 and sh == sw and sh >= 1
            and ph < kh and pw < kw and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.padding_mode == "zeros"):
        return False
    return (x.shape[2] + 2 * ph - kh) // sh + 1 >= 1 and (x.shape[3] + 2 * pw - kw) // sw + 1 >= 1 and hip_available()


class _Stem3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, geo, stats):
        H = hip()
        kh, kw, s, ph, pw = geo
        wb = w if w.dtype == torch.bfloat16 else w.to(torch.bfloat16)
        if not wb.is_contiguous(memory_format=torch.channels_last):
            wb = wb.contiguous(memory_format=torch.channels_last)
        # the f32 (or bf16) image is read as it is: no cast / pad pass
        y = H.stem3_forward(x, H.stem3_pack_weight(wb), kh, kw, s, ph, pw, stats)
        ctx.save_for_backward(x)
        ctx.geo = geo
        ctx.wdtype = w.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        if not ctx.needs_input_grad[1]:
            return None, None, None, None
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        kh, kw, s, ph, pw = ctx.geo
        dw = hip().stem3_wgrad(dy.to(torch.bfloat16), x, kh, kw, s, ph, pw, out_f32=ctx.wdtype == torch.float32)
        if dw.dtype != ctx.wdtype:
            dw = dw.to(ctx.wdtype)
        return None, dw, None, None


def stem3_conv(conv: torch.nn.Conv2d, x: torch.Tensor, w: torch.Tensor,
               stats: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``conv(x)`` with ``w`` (the bf16 shadow of ``conv.weight`` or the weight) on stem3.hip ->
    bf16 [N, 32, OH, OW] channels_last; ``stats``: the following BN's f64 slotted sums workspace."""
    geo = (conv.kernel_size[0], conv.kernel_size[1], conv.stride[0], conv.padding[0], conv.padding[1])
    return _Stem3Fn.apply(x, w, geo, stats)
