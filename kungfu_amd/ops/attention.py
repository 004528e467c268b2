"""Fused multi-head self-attention on the HIP kernels of csrc/kernels/attention.hip.

``self_attention(qkv, heads, p)`` takes the fused q/k/v projection output ``[B, S, 3*H*64]``
(the ``[B, S, 3, H, 64]`` layout of one ``nn.Linear(d, 3d)``) and returns the attention output
already in ``[B, S, H*64]`` (the layout the output projection consumes): no head permutes, no
transposed copies, and the backward writes dq/dk/dv straight into one ``[B, S, 3*H*64]``
gradient (no concatenation).  Dropout on the attention probabilities uses a counter hash of
(seed, b*H + h, query, key) -- the mask is recomputed in the backward, never stored;
:func:`dropout_keep` reproduces it in torch for the tests.

Covers BERT's shapes (S = 64 or 128 tokens, head dim 64, no attention mask); anything else
runs ``F.scaled_dot_product_attention``.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .._lib import hip, hip_available
from . import dropout_seed

# (round 6: the qkv bias gradient from column sums inside the attention backward is gone -- measured slower
# end to end than the projection's own two-stage column sum, BERT-base + GNS 15.70-15.76 -> 15.78-15.80
# ms/step on one box, r5t38)


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads, p, seed):
        scale = 1.0 / math.sqrt(64.0)
        out, lse = hip().attention_forward(qkv, heads, scale, seed, p)
        ctx.save_for_backward(qkv, out, lse)
        ctx.heads, ctx.p, ctx.seed, ctx.scale = heads, p, seed, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        dqkv = hip().attention_backward(qkv, out, lse, dout.contiguous(), ctx.heads, ctx.scale, ctx.seed, ctx.p)
        return dqkv, None, None, None


def eligible(qkv: torch.Tensor, heads: int) -> bool:
    return (qkv.is_cuda and qkv.dtype == torch.bfloat16 and qkv.dim() == 3 and qkv.is_contiguous()
            and qkv.shape[2] == 3 * heads * 64 and hip_available() and hip().attention_supported(int(qkv.shape[1]), 64))


def self_attention(qkv: torch.Tensor, heads: int, p: float = 0.0) -> torch.Tensor:
    """softmax(Q K^T / sqrt(64)) V with dropout ``p`` on the probabilities, per head;
    ``qkv``: [B, S, 3*H*dh] -> [B, S, H*dh]."""
    B, S, D3 = qkv.shape
    if eligible(qkv, heads):
        seed = int(torch.randint(0, 2**31 - 1, (1,)).item())  # CPU generator: no device sync
        dropout_seed.base(qkv.device)  # registers the device seed word (graph replays advance it)
        return _AttnFn.apply(qkv, heads, float(p), seed)
    dh = D3 // (3 * heads)
    q, k, v = qkv.view(B, S, 3, heads, dh).permute(2, 0, 3, 1, 4)
    a = F.scaled_dot_product_attention(q, k, v, dropout_p=p)
    return a.transpose(1, 2).reshape(B, S, heads * dh)


def dropout_keep(seed: int, B: int, H: int, S: int, p: float, device=None) -> torch.Tensor:
    """The kernels' keep mask [B, H, S(query), S(key)] (bool), computed with torch int64 ops."""
    m32 = 0xFFFFFFFF
    bh = torch.arange(B * H, device=device, dtype=torch.int64).view(B * H, 1, 1)
    q = torch.arange(S, device=device, dtype=torch.int64).view(1, S, 1)
    k = torch.arange(S, device=device, dtype=torch.int64).view(1, 1, S)
    x = ((q << 16) | k) ^ seed
    x = (x * 0x9E3779B1) & m32
    x = x ^ (((bh * 0x85EBCA77) & m32) + (x >> 15)) & m32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & m32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & m32
    x = x ^ (x >> 16)
    thresh = 0 if p <= 0 else min(int(p * 4294967296.0), 0xFFFFFFFF)
    return (x >= thresh).view(B, H, S, S)
