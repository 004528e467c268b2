"""Topology queries and tree construction.

Parity: ``srcs/python/kungfu/tensorflow/ops/topology.py:4-25`` and
``srcs/cpp/src/tensorflow/ops/cpu/topology.cpp:6-230`` (KungfuRank,
KungfuClusterSize, KungfuGetPeerInfo, KungfuGetPeerLatencies,
KungfuMinimumSpanningTree via AllGatherTransform, KungfuGetNeighbour,
KungfuRoundRobin).  The MST itself is native (Prim, C++).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch

from .._lib import runtime
from ..python import _ensure


def peer_info() -> Tuple[int, int]:
    _ensure()
    return runtime.rank(), runtime.size()


def get_peer_latencies() -> torch.Tensor:
    """Round-trip latency (seconds) to every peer; 0 for self."""
    _ensure()
    return torch.tensor(runtime.peer_latencies(), dtype=torch.float32)


def minimum_spanning_tree(weights: torch.Tensor, root: int = 0) -> torch.Tensor:
    """MST of an n x n weight matrix (symmetrised). Returns edges [n-1, 2]."""
    w = weights.detach().double().cpu().contiguous()
    n = w.shape[0]
    father = runtime.minimum_spanning_tree(w.reshape(-1).tolist(), n, root)
    edges = [(father[v], v) for v in range(n) if v != root]
    return torch.tensor(edges, dtype=torch.int32).reshape(-1, 2)


def mst_father(weights: torch.Tensor, root: int = 0) -> List[int]:
    w = weights.detach().double().cpu().contiguous()
    return list(runtime.minimum_spanning_tree(w.reshape(-1).tolist(), w.shape[0], root))


def all_gather_transform(x: torch.Tensor, out_like: torch.Tensor, fn, name: Optional[str] = None) -> torch.Tensor:
    """Native AllGatherTransform (srcs/cpp/src/session.cpp:162-181): every peer's ``x`` is
    gathered to rank 0, ``fn(gathered [np, *x.shape]) -> tensor shaped like out_like`` runs
    there only, and its result is broadcast to every peer."""
    _ensure()
    from .._lib import dtype_code
    from .collective import _auto_name

    h = x.detach().cpu().contiguous()
    out = torch.zeros_like(out_like, device="cpu").contiguous()
    np_ = runtime.size()

    def run(gptr, gbytes, optr, obytes):
        g = torch.frombuffer(bytearray((ctypes.c_char * gbytes).from_address(gptr)), dtype=h.dtype)
        res = fn(g.view((np_,) + tuple(h.shape))).to(out.dtype).contiguous().view(-1)
        ctypes.memmove(optr, res.data_ptr(), min(obytes, res.numel() * res.element_size()))

    runtime.all_gather_transform(h.data_ptr(), h.numel(), dtype_code(h), out.data_ptr(),
                                 out.numel() * out.element_size(), run, name or _auto_name("agt"))
    return out


def global_minimum_spanning_tree(self_weights: torch.Tensor) -> torch.Tensor:
    """Every peer contributes its row of weights (e.g. latencies to every peer); rank 0
    computes the MST of the gathered matrix and broadcasts the edges (one native
    AllGatherTransform instead of every peer computing it, as in the reference)."""
    n = runtime.size() if runtime.initialized() else 1
    w = self_weights.detach().float()
    return all_gather_transform(w, torch.zeros(max(n - 1, 0), 2, dtype=torch.int32),
                                lambda g: minimum_spanning_tree(g).reshape(-1, 2))


def get_neighbour_mask(edges: torch.Tensor, cluster_size: int = None, self_rank: int = None) -> torch.Tensor:
    _ensure()
    n = runtime.size() if cluster_size is None else cluster_size
    me = runtime.rank() if self_rank is None else self_rank
    if not 0 <= me < n:
        raise ValueError("self_rank in [0, cluster_size) is required")
    mask = torch.zeros(n, dtype=torch.bool)
    for u, v in edges.tolist():
        if u == me:
            mask[v] = True
        if v == me:
            mask[u] = True
    return mask


class RoundRobin:
    """Cycles over the True entries of a mask (stateful, like KungfuRoundRobin)."""

    def __init__(self):
        self.pos = 0

    def __call__(self, mask: Sequence[bool]) -> int:
        m = [bool(x) for x in (mask.tolist() if isinstance(mask, torch.Tensor) else mask)]
        n = len(m)
        for i in range(n):
            idx = (self.pos + i) % n
            if m[idx]:
                self.pos = (idx + 1) % n
                return idx
        return -1


_rr = RoundRobin()


def round_robin(mask) -> int:
    return _rr(mask)
