"""Save tensors into this peer's model store (for P2P pulls by other peers).

Parity: ``srcs/python/kungfu/tensorflow/ops/local.py:4-33`` /
``ops/cpu/local.cpp:5-81`` (KungfuSaveVariable with optional version,
KungfuSaveVariables).  The store is the C++ runtime's Store / VersionedStore
(window of 3 versions); blob writes take the blob's exclusive lock.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .._lib import runtime
from ..python import _ensure


def _host(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to("cpu").contiguous()


def save_variable(t: torch.Tensor, name: str, version: Optional[int] = None) -> None:
    _ensure()
    h = _host(t)
    nbytes = h.numel() * h.element_size()
    if version is None:
        runtime.save(name, h.data_ptr(), nbytes)
    else:
        runtime.save_version(str(int(version)), name, h.data_ptr(), nbytes)


def save_variables(variables: Sequence[torch.Tensor], names: Sequence[str], version: Optional[int] = None) -> None:
    for t, n in zip(variables, names):
        save_variable(t, n, version)
