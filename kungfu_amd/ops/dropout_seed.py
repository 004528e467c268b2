"""Device seed base of the hashed dropout masks (attention and add+LayerNorm kernels).

Each dropout call draws its own 31-bit seed on the host (CPU generator: no device sync) and the
kernels hash it with the element coordinates; the mask is recomputed in the backward from the
same seed, so no mask tensor exists.  A hipGraph replay, however, re-uses the host seeds that
were recorded at capture -- every replayed step would drop the same elements.  So the kernels
also mix in one device word, this module's ``base``: :func:`advance` (called by
``parallel.graphs.GraphedStep`` before every replay) changes it on the device, which gives every
replayed step fresh masks while forward and backward of one step still agree.
"""
from __future__ import annotations

from typing import Optional

import torch

from .._lib import hip, hip_available

_base: Optional[torch.Tensor] = None


def base(device=None) -> Optional[torch.Tensor]:
    """The device seed word (created and registered with the kernels on first use)."""
    global _base
    if _base is None and hip_available() and torch.cuda.is_available():
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        seed = int(torch.randint(1, 2**31 - 1, (1,)).item())
        _base = torch.full((1,), seed, dtype=torch.int32, device=dev)
        hip().set_dropout_seed_base(_base)
    return _base


def effective(seed: int) -> int:
    """The seed the kernels hash for host seed ``seed`` (mixed with the current base; reads the
    base back from the device -- for tests and reference computations only)."""
    if _base is None:
        return seed
    b = int(_base.item()) & 0xFFFFFFFF
    return (seed ^ ((b * 0x85EBCA6B) & 0xFFFFFFFF)) & 0xFFFFFFFF


def advance() -> None:
    """New masks for the next (replayed) step: one tiny kernel, outside any graph."""
    b = base()
    if b is not None:
        b.add_(0x3C6EF372)
