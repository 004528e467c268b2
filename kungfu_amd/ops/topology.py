"""Topology queries and tree construction.

Parity: ``srcs/python/kungfu/tensorflow/ops/topology.py:4-25`` and
``srcs/cpp/src/tensorflow/ops/cpu/topology.cpp:6-230`` (KungfuRank,
KungfuClusterSize, KungfuGetPeerInfo, KungfuGetPeerLatencies,
KungfuMinimumSpanningTree via AllGatherTransform, KungfuGetNeighbour,
KungfuRoundRobin).  The MST itself is native (Prim, C++).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from .._lib import runtime
from ..python import _ensure
from .collective import all_gather


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


def global_minimum_spanning_tree(self_weights: torch.Tensor) -> torch.Tensor:
    """Every peer contributes its row of weights (e.g. latencies to every
    peer); rows are all-gathered and every peer computes the same MST."""
    w = all_gather(self_weights.detach().float().cpu())
    return minimum_spanning_tree(w)


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
