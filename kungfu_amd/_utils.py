"""Small helpers (parity: srcs/python/kungfu/_utils.py:9-50, utils/ema.py)."""
from __future__ import annotations

import os
import time
from typing import Callable, Iterable, List, Optional

_T0 = time.time()


def map_maybe(f: Callable, xs: Iterable) -> List:
    return [None if x is None else f(x) for x in xs]


def measure(f: Callable):
    t0 = time.time()
    r = f()
    return time.time() - t0, r


def show_duration(d: float) -> str:
    if d < 1e-3:
        return "%.1fus" % (d * 1e6)
    if d < 1:
        return "%.1fms" % (d * 1e3)
    return "%.2fs" % d


def _since_proc_start() -> float:
    ts = os.environ.get("KUNGFU_PROC_START_TIMESTAMP")
    return time.time() - (float(ts) if ts else _T0)


def _log_event(name: str):
    """Timestamped event line (parity: kungfu._utils._log_event)."""
    print("TS=%.6f %s :: %s" % (time.time(), name, show_duration(_since_proc_start())), flush=True)


class EMA:
    """Exponential moving average with optional scale cap (parity: kungfu.utils.ema,
    srcs/python/kungfu/utils/ema.py): the first update sets the value; later samples are
    clamped to [value / cap, value * cap] before blending."""

    def __init__(self, alpha: float = 0.9, scale_cap: Optional[float] = None, max_scale: Optional[float] = None):
        self.alpha = alpha
        self.scale_cap = scale_cap if scale_cap is not None else max_scale
        self.value = None

    def _cap(self, x: float) -> float:
        if self.scale_cap is None:
            return x
        up = self.value * self.scale_cap
        if x > up:
            return up
        down = self.value / self.scale_cap
        if x < down:
            return down
        return x

    def update(self, x: float) -> float:
        if self.value is None:
            self.value = x
        else:
            self.value = self.alpha * self.value + (1 - self.alpha) * self._cap(x)
        return self.value

    def get(self) -> Optional[float]:
        return self.value

    def reset(self) -> None:
        self.value = None


Ki, Mi, Gi = 1024, 1024 ** 2, 1024 ** 3


def show_size(s: float) -> str:
    """Human-readable byte count (parity: v1/helpers/utils.py show_size)."""
    if s > Gi:
        return "%.2fGi" % (s / Gi)
    if s > Mi:
        return "%.2fMi" % (s / Mi)
    if s > Ki:
        return "%.2fKi" % (s / Ki)
    return "%d" % s


def show_rate(size: float, duration: float) -> str:
    r = size / duration
    for unit, k in (("GiB/s", Gi), ("MiB/s", Mi), ("KiB/s", Ki)):
        if r >= k:
            return "%.2f%s" % (r / k, unit)
    return "%.2fB/s" % r
