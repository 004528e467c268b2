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
    """Exponential moving average with optional scale cap (parity: kungfu.utils.ema)."""

    def __init__(self, alpha: float = 0.9, max_scale: Optional[float] = None):
        self.alpha, self.max_scale, self.value = alpha, max_scale, None

    def update(self, x: float) -> float:
        if self.value is None:
            self.value = x
        else:
            nv = self.alpha * self.value + (1 - self.alpha) * x
            if self.max_scale is not None and self.value != 0:
                hi, lo = abs(self.value) * self.max_scale, abs(self.value) / self.max_scale
                nv = max(min(nv, hi), -hi) if abs(nv) > hi else nv
                if abs(nv) < lo:
                    nv = lo if nv >= 0 else -lo
            self.value = nv
        return self.value


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
