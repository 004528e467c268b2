"""Vocabulary projection ``logits = h W^T + b`` (BERT's tied masked-LM decoder) with padded logits rows.

BERT-base's decoder is 2,560 predicted tokens x 30,522 classes x 768.  The odd-by-2 vocabulary made
every logits row 4-byte aligned only: the fused cross-entropy read it 4 bytes at a time (xent forward
72.5 us, backward 89.1 us per step, r5t23 profile), the decoder bias gradient was torch's column
reduction (77 us), and the tied table's gradient took an autocast cast each way, a zero-filled
table-sized embedding gradient, an autograd sum and an AccumulateGrad add (~140 us).  Here:

* forward: the logits GEMM writes rows padded to ``ld`` = V rounded up to 8 (16-byte aligned) --
  ``_FWD = "ours"``: gemm.hip's ``gemm_nt_ld`` (ragged N: rows of W past the vocabulary read zeros;
  150 us vs hipBLASLt's 135-154 us into the same padded rows, tools/bench_mlm_head.py, r5t26), or
  ``"blas"``: hipBLASLt through its leading dimension; the op returns the [..., V] view, which
  ops/xent.py reads in place with 16-byte loads (forward 28.5 us, backward 52.2 us);
* backward: the cross-entropy gradient arrives with the same padded row stride; the data gradient
  is hipBLASLt reading it through its leading dimension (no copy) as a split-K batched product
  (``_data_grad``: 242 -> 166 us); the bias gradient is the
  deterministic two-stage column sum (norms.hip) over the padded buffer (padding columns zero);
* a table registered with a flat space (parallel.mixed.enable_bf16_shadow) is projected from its
  bf16 shadow (the step's one cast kernel) and its weight gradient is accumulated by hipBLASLt in
  f32 straight into the table's flat slot, where ops/embedding.py's lookup scatter-adds too
  (parallel.mixed.use_direct: the last producer hands the table to the bucket accounting).

Falls back to ``F.linear`` off the GPU path.  Parity: the reference's BERT pre-training head
(TF ``tf.matmul(..., transpose_b=True)`` + ``bias_add`` against the embedding table).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._lib import hip, hip_available

_ENABLED = True  # module switch (tests / A/B)
_FWD = "ours"  # logits GEMM: "blas" (hipBLASLt into the padded rows) | "ours" (gemm_nt_ld)


def _padded_base(t2: torch.Tensor, ld: int):
    """The [R, ld] buffer ``t2`` ([R, V] view with row stride ld) was cut from, or None."""
    R = t2.shape[0]
    if t2.stride() != (ld, 1) or t2.storage_offset() != 0:
        return None
    if t2.untyped_storage().nbytes() < R * ld * t2.element_size():
        return None
    return t2.as_strided((R, ld), (ld, 1))


def _logits(h2, wb, bb, V, ld):
    if _FWD == "ours":
        return hip().gemm_nt_ld(h2, wb, bb, ld, 256)
    # hipBLASLt writing the padded rows through its leading dimension (stream-K kernel for the odd N)
    out = torch.empty(h2.shape[0], ld, device=h2.device, dtype=torch.bfloat16)
    view = out.narrow(1, 0, V)
    if bb is None:
        torch.mm(h2, wb.t(), out=view)
    else:
        torch.addmm(bb, h2, wb.t(), out=view)
    return out


class _VocabFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, w, b, target=None):
        V, D = w.shape
        ctx.target = target
        if target is not None:
            # a flat-space table: its bf16 shadow (the step's one cast kernel), and the weight gradient
            # goes straight into its f32 slot (parallel.mixed.use_direct: the tied lookup lands there too)
            from ..parallel.mixed import use_direct

            wb = target[0].shadow_view(target[1])
            use_direct(target)
        else:
            wb = w if w.dtype == torch.bfloat16 else w.to(torch.bfloat16)
        bb = None if b is None else (b if b.dtype == torch.bfloat16 else b.to(torch.bfloat16))
        h2 = h.reshape(-1, D)
        if not h2.is_contiguous():
            h2 = h2.contiguous()
        ld = (V + 7) // 8 * 8
        out = _logits(h2, wb, bb, V, ld)
        ctx.save_for_backward(h2, wb)
        ctx.hshape, ctx.ld = h.shape, ld
        ctx.w_dtype = w.dtype
        ctx.b_dtype = None if b is None else b.dtype
        return out.narrow(1, 0, V).view(*h.shape[:-1], V)

    @staticmethod
    def backward(ctx, dy):
        h2, wb = ctx.saved_tensors
        V, D = wb.shape
        dy2 = dy.reshape(-1, V)
        if dy2.stride(1) != 1:
            dy2 = dy2.contiguous()
        dh = dw = db = None
        if ctx.needs_input_grad[0]:
            dh = _data_grad(dy2, wb).view(ctx.hshape)
        tgt = ctx.target
        if tgt is not None:
            from ..parallel.mixed import landed_direct

            space, i = tgt
            _accumulate_wgrad(space, i, dy2, h2)
            landed_direct(tgt)
        elif ctx.needs_input_grad[1]:
            dw = torch.mm(dy2.t(), h2)
        if ctx.b_dtype is not None and ctx.needs_input_grad[2]:
            base = _padded_base(dy2, ctx.ld)
            if base is None and dy2.is_contiguous() and V % 8 == 0:
                base = dy2
            if base is not None and dy2.dtype == torch.bfloat16:
                db = hip().colsum(base, torch.float32).narrow(0, 0, V).to(ctx.b_dtype)
            else:
                db = dy2.sum(0, dtype=torch.float32).to(ctx.b_dtype)
        return dh, dw, db, None


_SPLIT_K = 6  # data-gradient K split (0: one product)


def _data_grad(dy2, wb):
    """dh = dy2 . W.  The output is only [rows, D] (2,560 x 768: 40 hipBLASLt tiles, one 95-workgroup
    launch, 242 us) while K is the vocabulary: split K into S equal slices as ONE batched product with
    f32 outputs (S x the tiles) and sum the slices in a fixed order -- 166 us (r5t28, S = 6)."""
    V, D = wb.shape
    S = _SPLIT_K
    if S > 1 and V % S == 0 and dy2.stride(1) == 1 and wb.stride() == (D, 1):
        Kc = V // S
        a = dy2.as_strided((S, dy2.shape[0], Kc), (Kc, dy2.stride(0), 1), dy2.storage_offset())
        b = wb.as_strided((S, Kc, D), (Kc * D, D, 1), wb.storage_offset())
        try:
            return torch.bmm(a, b, out_dtype=torch.float32).sum(0).to(wb.dtype)  # f32 slice sum, one rounding
        except (RuntimeError, TypeError):
            pass
    return torch.mm(dy2, wb)


_F32_ACC = [None]  # hipBLASLt bf16 x bf16 -> f32 accumulate (addmm out_dtype) usable: probed once


def _accumulate_wgrad(space, i, dy2, h2):
    """slot(i) += dy2^T h2 (f32): hipBLASLt accumulating in f32 straight into the flat slot when the build
    has ``addmm(..., out_dtype=float32)``; else the bf16 product landed by one grad_accumulate kernel."""
    g = space.grad_view(i)
    if _F32_ACC[0] is not False:
        try:
            torch.addmm(g, dy2.t(), h2, out_dtype=torch.float32, out=g)
            _F32_ACC[0] = True
            return
        except (RuntimeError, TypeError):
            if _F32_ACC[0]:
                raise
            _F32_ACC[0] = False
    hip().grad_accumulate(space.flat_grad, [torch.mm(dy2.t(), h2)], [space.offsets[i][0]], 1.0)


def vocab_projection(h: torch.Tensor, w: torch.Tensor, b: torch.Tensor = None) -> torch.Tensor:
    """``F.linear(h, w, b)`` for a vocabulary-sized output (any V); under bf16 autocast or with bf16
    operands the GEMM runs on gemm.hip with padded logits rows (see module docstring)."""
    bf16 = h.dtype == torch.bfloat16 or (h.is_cuda and torch.is_autocast_enabled("cuda")
                                         and torch.get_autocast_dtype("cuda") == torch.bfloat16)
    if (_ENABLED and h.is_cuda and w.is_cuda and bf16 and w.dim() == 2 and h.shape[-1] == w.shape[1]
            and w.shape[1] % 32 == 0 and hip_available()):
        M = h.numel() // w.shape[1]
        if M > 0 and hip().gemm_nt_ld_supported(M, w.shape[0], w.shape[1], (w.shape[0] + 7) // 8 * 8):
            from ..parallel.mixed import embedding_target

            tgt = embedding_target(w) if torch.is_grad_enabled() and w.requires_grad else None
            if tgt is not None and tgt[0].flat_shadow is None:
                tgt = None
            return _VocabFn.apply(h.to(torch.bfloat16), w, b, tgt)
    return F.linear(h, w, b)
