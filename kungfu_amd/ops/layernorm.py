"""Fused residual-add + LayerNorm on the HIP kernels of csrc/kernels/layernorm.hip.

``AddLayerNorm(D)`` is an ``nn.LayerNorm`` (same parameters and state_dict keys) whose
``forward(x, residual=None)`` computes ``layer_norm(x + residual)``.  For bf16 GPU inputs
(the transformer residual stream under bf16 autocast) it runs one HIP pass each way and
keeps the stream in bf16; torch's autocast LayerNorm instead produces f32 (which the next
GEMM casts back to bf16) and its backward is three kernels.  Anything else (CPU, f32,
unsupported D) uses the torch composition.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._lib import hip, hip_available
from . import dropout_seed

import os

_BIAS_LINK = True  # module switch of the linear bias-gradient link (tests)


class _AddLayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, gamma, beta, eps, p=0.0, seed=0, blink=None, rlink=None):
        from ..parallel.mixed import direct_target

        y, s, mean, rstd = hip().layernorm_forward(x, r, gamma, beta, eps, p, seed)
        ctx.save_for_backward(s, gamma, mean, rstd)
        ctx.has_r = r is not None
        ctx.p, ctx.seed = (p, seed) if r is not None else (0.0, 0)
        tg, tb = direct_target(gamma), direct_target(beta)
        ctx.direct = (tg, tb) if tg is not None and tb is not None else None
        ctx.blink = blink if r is not None else None
        ctx.rlink = rlink
        return y

    @staticmethod
    def backward(ctx, dy):
        s, gamma, mean, rstd = ctx.saved_tensors
        bl = ctx.blink
        if bl is not None:
            # the residual input is a linear layer's output whose only consumer is this LayerNorm:
            # the same pass also sums its gradient's columns = that layer's bias gradient
            ds, dg, db, dr, rb = hip().layernorm_backward(dy.contiguous(), s, gamma, mean, rstd, ctx.p, ctx.seed,
                                                          bl.dtype)
            bl.value, bl.ptr = rb, (dr if dr is not None else ds).data_ptr()
        else:
            ds, dg, db, dr = hip().layernorm_backward(dy.contiguous(), s, gamma, mean, rstd, ctx.p, ctx.seed)
        if ctx.direct is not None:
            # gamma / beta gradients to the flat space's sink (landed with their bucket by one
            # multi-tensor kernel instead of an AccumulateGrad add each: 48 launches in BERT-base)
            from ..parallel.mixed import deliver

            deliver(ctx.direct[0], dg)
            deliver(ctx.direct[1], db)
            dg = db = None
        # d(x + r)/dx = d(x + r)/dr = 1: both inputs receive ds (the dropped r: ds * keep / (1-p))
        if ctx.has_r and dr is None:
            dr = ds
        dx = ds
        if ctx.rlink is not None and ctx.needs_input_grad[0]:
            # the skip input's other consumer (a linear layer, ops.linear.ResidualLink) adds this
            # gradient inside its data-gradient GEMM
            ctx.rlink.value, dx = ds, None
        return dx, (dr if ctx.has_r else None), dg, db, None, None, None, None, None


def _eligible(x: torch.Tensor, r: Optional[torch.Tensor], w: torch.Tensor) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and hip_available()):
        return False
    if r is not None and (r.dtype != torch.bfloat16 or r.shape != x.shape or not r.is_contiguous()):
        return False
    return w is not None and w.dtype == torch.float32 and hip().layernorm_supported(int(x.shape[-1]))


def add_layer_norm(x: torch.Tensor, residual: Optional[torch.Tensor], weight: torch.Tensor, bias: torch.Tensor,
                   eps: float = 1e-5, dropout: float = 0.0, training: bool = False,
                   bias_link: bool = False) -> torch.Tensor:
    """``F.layer_norm(x + F.dropout(residual, dropout, training), (D,), weight, bias, eps)``; on the
    HIP kernels the dropout is fused (hashed keep mask, recomputed in the backward).

    ``bias_link``: the caller guarantees ``residual`` is the output of :func:`ops.linear.linear`
    consumed only here -- the backward pass then also produces that layer's bias gradient
    (:class:`~kungfu_amd.ops.linear.BiasLink`), which skips its own column-sum pass."""
    p = float(dropout) if training and residual is not None else 0.0
    if _eligible(x, residual, weight):
        seed = int(torch.randint(0, 2**31 - 1, (1,)).item()) if p > 0 else 0  # CPU generator: no device sync
        if p > 0:
            dropout_seed.base(x.device)  # registers the device seed word (graph replays advance it)
        bl = (getattr(residual, "_kf_blink", None) if bias_link and _BIAS_LINK and residual is not None
              and x.shape[-1] <= 2048 else None)
        rl = getattr(x, "_kf_rlink", None) if residual is not None else None
        if rl is not None and not rl.armed:
            rl = None  # the linear consumer did not take the linking path: plain gradient return
        return _AddLayerNormFn.apply(x, residual, weight.contiguous(), bias.contiguous(), float(eps), p, seed, bl, rl)
    if p > 0:
        residual = F.dropout(residual, p, True)
    s = x if residual is None else x + residual
    return F.layer_norm(s, s.shape[-1:], weight, bias, eps)


class AddLayerNorm(nn.LayerNorm):
    def forward(self, x, residual=None, dropout: float = 0.0, bias_link: bool = False):
        """``layer_norm(x + dropout(residual))`` (``dropout`` active in training mode only);
        ``bias_link``: see :func:`add_layer_norm`."""
        if residual is not None and residual.dtype != x.dtype and x.is_cuda:
            residual = residual.to(x.dtype)  # e.g. an f32 dropout output beside a bf16 stream
        return add_layer_norm(x, residual, self.weight, self.bias, self.eps, dropout, self.training, bias_link)
