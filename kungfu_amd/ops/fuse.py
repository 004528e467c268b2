"""fuse / defuse: many tensors <-> one flat buffer.

Parity: ``srcs/python/kungfu/tensorflow/ops/__init__.py:29-46`` (``fuse`` =
concat of flattened tensors, ``defuse`` = split + reshape).  On GPU both are a
single K7 multi-tensor HIP kernel launch (with optional scale and dtype cast)
instead of one copy per tensor.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from .._lib import dtype_code, hip


def _desc(tensors: Sequence[torch.Tensor], device) -> torch.Tensor:
    rows = []
    off = 0
    for t in tensors:
        rows.append((t.data_ptr(), off, t.numel()))
        off += t.numel()
    return torch.tensor(rows, dtype=torch.int64).to(device, non_blocking=True)


def fuse(tensors: Sequence[torch.Tensor], dtype: Optional[torch.dtype] = None, scale: float = 1.0) -> torch.Tensor:
    tensors = [t if t.is_contiguous() else t.contiguous() for t in tensors]
    dtype = dtype or tensors[0].dtype
    total = sum(t.numel() for t in tensors)
    dev = tensors[0].device
    if dev.type == "cuda" and dtype in (torch.float32, torch.bfloat16, torch.float16) and \
            all(t.dtype == tensors[0].dtype for t in tensors) and tensors[0].dtype in (torch.float32, torch.bfloat16, torch.float16):
        flat = torch.empty(total, dtype=dtype, device=dev)
        d = _desc(tensors, dev)
        hip().pack(d, len(tensors), dtype_code(tensors[0]), flat, scale)
        d.record_stream(torch.cuda.current_stream(dev))
        return flat
    flat = torch.cat([t.reshape(-1).to(dtype) for t in tensors]) if tensors else torch.empty(0, dtype=dtype)
    if scale != 1.0:
        flat.mul_(scale)
    return flat


def defuse(flat: torch.Tensor, tensors: Sequence[torch.Tensor], scale: float = 1.0) -> List[torch.Tensor]:
    """Copy ``flat`` back into ``tensors`` (in place) and return them."""
    dev = flat.device
    if dev.type == "cuda" and flat.dtype in (torch.float32, torch.bfloat16, torch.float16) and \
            all(t.is_contiguous() and t.dtype in (torch.float32, torch.bfloat16, torch.float16) and
                t.dtype == tensors[0].dtype for t in tensors):
        d = _desc(tensors, dev)
        hip().unpack(d, len(tensors), dtype_code(tensors[0]), flat, scale)
        d.record_stream(torch.cuda.current_stream(dev))
        return list(tensors)
    off = 0
    with torch.no_grad():
        for t in tensors:
            n = t.numel()
            src = flat[off:off + n].view(t.shape)
            t.copy_(src * scale if scale != 1.0 else src)
            off += n
    return list(tensors)


def split_like(flat: torch.Tensor, shapes: Sequence[torch.Size]) -> List[torch.Tensor]:
    out, off = [], 0
    for s in shapes:
        n = 1
        for d in s:
            n *= d
        out.append(flat[off:off + n].view(s))
        off += n
    return out
