"""Elastic data sharding.

Parity: ``srcs/python/kungfu/tensorflow/v1/datasets/adaptor.py:4-45`` -- the
global sample offset (``trained_samples``) survives a resize, and each worker
takes its contiguous share of every global batch from that offset, so a
cluster of any size consumes the dataset in the same global order.
"""
from __future__ import annotations

from typing import Iterator, Tuple


def shard_range(global_batch: int, rank: int, size: int) -> Tuple[int, int]:
    """[begin, end) of ``rank``'s contiguous share of a global batch."""
    q, r = divmod(global_batch, size)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


class ElasticShardAdaptor:
    def __init__(self, n_samples: int, global_batch: int, offset: int = 0):
        self.n = n_samples
        self.global_batch = global_batch
        self.offset = offset  # == trained_samples

    def next_indices(self, rank: int, size: int):
        b, e = shard_range(self.global_batch, rank, size)
        idx = [(self.offset + i) % self.n for i in range(b, e)]
        self.offset += self.global_batch
        return idx

    def epoch_iter(self, rank: int, size: int) -> Iterator:
        steps = self.n // self.global_batch
        for _ in range(steps):
            yield self.next_indices(rank, size)
