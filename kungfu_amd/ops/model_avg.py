"""Fused-model pair averaging over the host P2P store (the reference's legacy ops).

Parity: ``ModelAveraging``, ``AsyncModelAveraging``, ``SaveModel``,
``RequestModel``, ``AsyncRequestModel`` with ``random`` / ``roundrobin`` peer
selection (``srcs/cpp/src/tensorflow/ops/cpu/peer_to_peer.cpp:8-523``).  The
engine is native (``csrc/runtime/model_avg.cpp``: selection, store, prefetch
thread, AVX averaging); this module stages the model as ONE contiguous f32
host buffer.  GPU training should prefer
:class:`kungfu_amd.optimizers.PairAveragingOptimizer`, whose store is
device-resident (HIP IPC pulls over xGMI); this path is the TCP/host one.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from .._lib import runtime
from ..python import _ensure


class ModelAveraging:
    """``v <- (v + v_peer) / 2`` for a list of f32 tensors, pulling a peer's saved model.

    ``prefetch=True`` is AsyncModelAveraging: average with the last completed pull
    while the next one runs in the background.
    """

    def __init__(self, tensors: Sequence[torch.Tensor], peer_selection: str = "random",
                 name: str = "kungfu-model", prefetch: bool = False):
        _ensure()
        self.tensors: List[torch.Tensor] = list(tensors)
        for t in self.tensors:
            if t.dtype != torch.float32:
                raise TypeError("ModelAveraging: float32 tensors only (as the reference)")
        self.count = sum(t.numel() for t in self.tensors)
        self.prefetch = prefetch
        pin = any(t.is_cuda for t in self.tensors) and torch.cuda.is_available()
        self.buf = torch.empty(self.count, dtype=torch.float32, pin_memory=pin)
        self.peer_buf = torch.empty(self.count, dtype=torch.float32)
        self.engine = runtime.ModelAverager(self.count, name, peer_selection)
        self.last_peer: Optional[int] = None

    # host staging ---------------------------------------------------------
    def _pack(self):
        o = 0
        for t in self.tensors:
            n = t.numel()
            self.buf[o:o + n].copy_(t.detach().reshape(-1), non_blocking=False)
            o += n

    def _unpack(self, src: torch.Tensor):
        o = 0
        with torch.no_grad():
            for t in self.tensors:
                n = t.numel()
                t.copy_(src[o:o + n].view_as(t))
                o += n

    # ops ------------------------------------------------------------------
    def save(self):
        """SaveModel: publish the current model in this peer's store."""
        self._pack()
        self.engine.save(self.buf.data_ptr())

    def request(self) -> Optional[List[torch.Tensor]]:
        """RequestModel: a selected peer's saved model (None if it has not saved one yet)."""
        p = self.engine.request(self.peer_buf.data_ptr())
        if p < 0:
            return None
        self.last_peer = p
        out, o = [], 0
        for t in self.tensors:
            n = t.numel()
            out.append(self.peer_buf[o:o + n].view(t.shape).to(t.device))
            o += n
        return out

    def __call__(self) -> int:
        """Average in place; returns the peer rank averaged with (-1: none available)."""
        self._pack()
        p = (self.engine.async_average if self.prefetch else self.engine.average)(self.buf.data_ptr())
        if p >= 0:
            self._unpack(self.buf)
            self.last_peer = p
        return p

    def wait(self):
        self.engine.wait()


def save_model(tensors: Sequence[torch.Tensor], name: str = "kungfu-model"):
    m = ModelAveraging(tensors, name=name)
    m.save()
    return m


def request_model(tensors: Sequence[torch.Tensor], peer_selection: str = "random",
                  name: str = "kungfu-model") -> Optional[List[torch.Tensor]]:
    return ModelAveraging(tensors, peer_selection, name).request()


def model_averaging(tensors: Sequence[torch.Tensor], peer_selection: str = "random",
                    name: str = "kungfu-model") -> ModelAveraging:
    """Returns a callable that averages ``tensors`` with a peer each call."""
    return ModelAveraging(tensors, peer_selection, name, prefetch=False)


def async_model_averaging(tensors: Sequence[torch.Tensor], peer_selection: str = "random",
                          name: str = "kungfu-model") -> ModelAveraging:
    return ModelAveraging(tensors, peer_selection, name, prefetch=True)
