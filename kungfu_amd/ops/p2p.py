"""One-sided pulls of named tensors from a peer's model store.

Parity: ``srcs/python/kungfu/tensorflow/ops/p2p.py:4-34`` /
``ops/cpu/p2p_new.cpp:5-60`` (KungfuRequestVariable: target rank, optional
version, name, shape, dtype).  Served by the owner's runtime thread without
the owner's participation (PeerToPeerEndpoint over TCP/UDS).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .._lib import runtime
from ..python import _ensure


def request_variable(target: int, name: str, shape: Sequence[int], dtype: torch.dtype,
                     version: Optional[int] = None, device=None) -> Optional[torch.Tensor]:
    """Returns the tensor, or None if the target does not have it."""
    _ensure()
    buf = torch.empty(tuple(shape), dtype=dtype)
    ok = runtime.request(int(target), "" if version is None else str(int(version)), name, buf.data_ptr(),
                         buf.numel() * buf.element_size())
    if not ok:
        return None
    return buf if device is None else buf.to(device)


def request_variable_with_template(target: int, template: torch.Tensor, name: str,
                                   version: Optional[int] = None) -> Optional[torch.Tensor]:
    return request_variable(target, name, template.shape, template.dtype, version=version, device=template.device)
