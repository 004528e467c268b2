"""Softmax cross-entropy straight from bf16 logits (csrc/kernels/xent.hip): ``F.cross_entropy(
logits.float(), labels)`` without the f32 copy of the logits, the f32 log-probabilities and the f32
gradient -- one read of the row forward, one read + one bf16 write backward.

BERT-base's masked-LM head produces 2,560 x 30,522 logits per step; the stock path moved ~2 GB for
its loss (cast, log_softmax, nll, their backwards, the cast back).  Labels outside [0, V) (PyTorch's
``ignore_index=-100``) are not counted, as in ``F.cross_entropy``'s mean reduction.

Parity: the reference trains BERT through TF's ``sparse_softmax_cross_entropy_with_logits``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._lib import hip, hip_available

_ENABLED = True  # module switch (tests)


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        R, V = logits.shape
        lse, rows = hip().xent_forward(logits, labels)
        valid = ((labels >= 0) & (labels < V)).sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(logits, labels, lse, valid)
        return rows.sum() / valid

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse, valid = ctx.saved_tensors
        scale = (g.to(torch.float32) / valid).reshape(1)
        return hip().xent_backward(logits, labels, lse, scale), None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Mean softmax cross-entropy of ``logits`` [..., V] against integer ``labels`` [...] (f32 loss)."""
    V = logits.shape[-1]
    if (_ENABLED and logits.is_cuda and logits.dtype == torch.bfloat16 and V % 2 == 0 and labels.dtype == torch.long
            and hip_available()):
        x2 = logits.reshape(-1, V)
        # rows padded to a multiple of 8 classes (ops/vocab.py's logits: a [R, V] view of [R, ld]) are read
        # in place by the 16-byte-load kernels; anything else is made contiguous
        if not (x2.stride(1) == 1 and x2.stride(0) >= V and x2.stride(0) % 8 == 0):
            x2 = x2.contiguous()
        return _XentFn.apply(x2, labels.reshape(-1).contiguous())
    return F.cross_entropy(logits.float().reshape(-1, V), labels.reshape(-1))
