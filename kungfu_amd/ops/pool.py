"""2x2 / stride-2 max-pool on the HIP kernels of csrc/kernels/pool.hip (VGG-16's pools).

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
