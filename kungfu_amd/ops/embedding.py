"""``F.embedding`` whose backward is a fixed-shape HIP scatter-add (csrc/kernels/flat_ops.hip
``embedding_bwd_kernel``: one f32 atomic per gradient element).

torch's embedding backward sorts the ids and reduces segments whose number comes from the data
(a device-to-host count): its launches depend on the batch, so a whole-step hipGraph replay of a
BERT step faulted inside it (profiles/r4_host_overhead.md).  The scatter-add has one launch of a
fixed size per step, so the step can be captured; it also replaces torch's sort-based kernels
(0.36 ms per BERT-base step, profiles/r3y_bert_base_summary.md).  The f32 atomics make the
summation order -- not the value set -- run-dependent.

Parity: the reference trains TF's embedding (``tf.gather`` + ``UnsortedSegmentSum`` gradient).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._lib import hip, hip_available


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, target=None):
        ctx.save_for_backward(ids)
        ctx.shape = weight.shape
        ctx.target = target
        if target is not None:
            from ..parallel.mixed import use_direct

            use_direct(target)
        return F.embedding(ids, weight)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        if not ctx.needs_input_grad[1]:
            return None, None, None
        tgt = ctx.target
        if tgt is not None:
            # scatter-add straight into the table's flat f32 gradient slot (zeroed at the step start): no
            # zero-filled table-sized gradient, no autograd sum with a tied use, no AccumulateGrad add
            from ..parallel.mixed import landed_direct

            space, i = tgt
            hip().embedding_backward(space.grad_view(i), ids.reshape(-1).contiguous(), dy.contiguous())
            landed_direct(tgt)
            return None, None, None
        grad = torch.zeros(ctx.shape, dtype=torch.float32, device=dy.device)
        hip().embedding_backward(grad, ids.reshape(-1).contiguous(), dy.contiguous())
        return None, grad, None


def embedding(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """``F.embedding(ids, weight)`` with the scatter-add backward on GPU (f32 weights, D % 4 == 0).
    A table registered with a flat space (parallel.mixed.enable_bf16_shadow) is scattered straight
    into its flat gradient slot."""
    if (weight.is_cuda and weight.dtype == torch.float32 and weight.dim() == 2 and weight.shape[1] % 4 == 0
            and ids.dtype == torch.long and hip_available()):
        from ..parallel.mixed import embedding_target

        tgt = embedding_target(weight) if torch.is_grad_enabled() and weight.requires_grad else None
        return _EmbeddingFn.apply(ids, weight, tgt)
    return F.embedding(ids, weight)
