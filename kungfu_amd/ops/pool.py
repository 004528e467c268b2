"""Pooling on the HIP kernels of csrc/kernels/pool.hip: VGG-16's 2x2/s2 max-pool,
Inception-v3's 3x3/s2 max-pool and 3x3/s1/p1 average pool (see the section below), and the
global average pool of the ResNet / Inception heads.

2x2 / stride-2 max-pool:

The windows do not overlap, so no argmax tensor is written: the backward re-reads the window
from x (kept alive as the pool's input anyway) and gathers, writing every dx element once.
Ties go to the first maximum in row-major window order, as torch's max-pool does.
Anything the kernel does not take (CPU, f32, odd H/W, C % 8 != 0) uses ``F.max_pool2d``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._lib import hip, hip_available


def _eligible(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0
            and x.is_contiguous(memory_format=torch.channels_last) and hip_available())


class _MaxPool2x2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return hip().maxpool2x2_forward(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return hip().maxpool2x2_backward(x, dy.contiguous(memory_format=torch.channels_last))


def max_pool2x2(x: torch.Tensor) -> torch.Tensor:
    """``F.max_pool2d(x, 2, 2)``."""
    if _eligible(x):
        return _MaxPool2x2Fn.apply(x)
    return F.max_pool2d(x, 2, 2)


class MaxPool2x2(nn.MaxPool2d):
    """``nn.MaxPool2d(2, 2)`` on the HIP kernels when eligible."""

    def __init__(self):
        super().__init__(2, 2)

    def forward(self, x):
        return max_pool2x2(x)


# ---------------------------------------------------------------- 3x3 pools (Inception-v3)

def _eligible3(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.shape[2] >= 3 and x.shape[3] >= 3
            and x.is_contiguous(memory_format=torch.channels_last) and hip_available())


class _MaxPool3s2Fn(torch.autograd.Function):
    """3x3/s2 max-pool: the forward also writes a byte argmax per element (1/2 of y, vs
    torch's int64 per element); the backward gathers through it (pool.hip)."""

    @staticmethod
    def forward(ctx, x, pad):
        y, arg = hip().maxpool3s2_forward(x, pad)
        ctx.save_for_backward(arg)
        ctx.hw = (x.shape[2], x.shape[3], pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        H, W, pad = ctx.hw
        return hip().maxpool3s2_backward(dy.contiguous(memory_format=torch.channels_last), arg, H, W, pad), None


def max_pool3x3s2(x: torch.Tensor, padding: int = 0) -> torch.Tensor:
    """``F.max_pool2d(x, 3, 2, padding)`` (padding 0 or 1)."""
    if padding in (0, 1) and _eligible3(x):
        return _MaxPool3s2Fn.apply(x, padding)
    return F.max_pool2d(x, 3, 2, padding)


class _AvgPool3s1Fn(torch.autograd.Function):
    """3x3/s1/p1 average pool with count_include_pad: the gradient is the same 9-tap
    stencil applied to dy, so forward and backward are one kernel."""

    @staticmethod
    def forward(ctx, x):
        return hip().avgpool3s1(x)

    @staticmethod
    def backward(ctx, dy):
        return hip().avgpool3s1(dy.contiguous(memory_format=torch.channels_last))


def avg_pool3x3s1(x: torch.Tensor) -> torch.Tensor:
    """``F.avg_pool2d(x, 3, 1, 1)`` (count_include_pad=True, torch's default)."""
    if _eligible3(x):
        return _AvgPool3s1Fn.apply(x)
    return F.avg_pool2d(x, 3, 1, 1)


class MaxPool3x3s2(nn.MaxPool2d):
    """``nn.MaxPool2d(3, 2)`` on the HIP kernels when eligible."""

    def __init__(self, padding: int = 0):
        super().__init__(3, 2, padding)

    def forward(self, x):
        return max_pool3x3s2(x, self.padding)


# ---------------------------------------------------------------- global average pool (heads)

class _GlobalAvgPoolFn(torch.autograd.Function):
    """mean over H, W of an NHWC bf16 tensor -> [N, C]; the backward writes dy / HW to every
    pixel with 16-byte stores (torch's expand + channels_last copy took ~100 us for ResNet-50's
    7x7x2048 head at batch 256)."""

    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return hip().global_avgpool_forward(x)

    @staticmethod
    def backward(ctx, dy):
        return hip().global_avgpool_backward(dy.to(torch.bfloat16), *ctx.hw)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)``."""
    if (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last) and hip_available()):
        return _GlobalAvgPoolFn.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
