"""Adaptation / elasticity operators.

Parity: ``srcs/python/kungfu/tensorflow/ops/adapt.py:5-62`` (resize,
resize_cluster_from_url, step_based_schedule, set_tree, calc_stats) and the
TF kernels ``ops/cpu/control.cpp:5-70`` (resize -> (changed, detached)),
``ops/cpu/elastic.cpp:16-81`` (StepBasedSchedule "size:steps,..."),
``ops/cpu/adaptation.cpp:5-46`` (SetTree, CalcStats).

After a membership change the device communicators are dropped
(``ResetNcclHelper`` equivalent) and rebuilt lazily for the new version.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

from .._lib import runtime
from ..python import _ensure


def _after_resize(changed: bool, detached: bool):
    if changed:
        from ..parallel.comm import reset_device_comm

        reset_device_comm()
    return changed, detached


def resize(n: int) -> bool:
    """Resize the cluster to ``n`` peers.  Returns ``changed``; use
    :func:`kungfu_amd.python.detached` to know whether this peer must quit."""
    _ensure()
    changed, detached = runtime.resize_cluster(int(n))
    _after_resize(changed, detached)
    return changed


def resize_cluster(n: int) -> Tuple[bool, bool]:
    _ensure()
    return _after_resize(*runtime.resize_cluster(int(n)))


def resize_cluster_from_url() -> Tuple[bool, bool]:
    """Adopt the cluster published by the config server. Returns (changed, detached)."""
    _ensure()
    return _after_resize(*runtime.resize_cluster_from_url())


class StepBasedSchedule:
    """``config = "size:steps,size:steps,..."`` -> cluster size for a step."""

    def __init__(self, config: str, default: int = 1, strict: bool = False):
        if not config:
            raise ValueError("config can't be empty")
        self.schedule: List[Tuple[int, int, int]] = []
        off = 0
        for part in config.split(","):
            if not part:
                continue
            kv = part.split(":")
            if len(kv) != 2:
                raise ValueError("invalid config %r" % config)
            k, v = int(kv[0]), int(kv[1])
            self.schedule.append((off, off + v, k))
            off += v
        self.default = default
        self.strict = strict

    def __call__(self, step: int) -> int:
        for b, e, k in self.schedule:
            if b <= step < e:
                return k
        if self.strict:
            raise ValueError("schedule not found for step %d" % step)
        return self.default


def step_based_schedule(config: str, step: int, default: int = 1, strict: bool = False) -> int:
    return StepBasedSchedule(config, default, strict)(step)


def set_tree(tree: Sequence[int]) -> bool:
    """Set the default all-reduce tree (father array; tree[i] == i marks the root)."""
    _ensure()
    return runtime.set_tree([int(x) for x in tree])


def set_strategy(name: str) -> bool:
    _ensure()
    return runtime.set_strategy(name)


def calc_stats() -> None:
    _ensure()
    from ..parallel.comm import flush_strategy_stats

    flush_strategy_stats()  # monitored device collectives (HIP-event timed) first
    runtime.calc_stats()


def log_stats() -> None:
    _ensure()
    runtime.log_stats()


def print_strategy_stats() -> None:
    from ..python import print_strategy_stats as p

    p()


def check_interference() -> bool:
    _ensure()
    return runtime.check_interference()


def get_init_checkpoint() -> Optional[str]:
    """Checkpoint path a (re)joining worker should restore from, if any
    (``KUNGFU_INIT_CKPT``)."""
    return os.environ.get("KUNGFU_INIT_CKPT")
