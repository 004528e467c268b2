"""Stateful scalar helpers: counter and exponential moving average.

Parity: ``srcs/python/kungfu/tensorflow/ops/state.py:4-13`` and the TF kernels
``srcs/cpp/src/tensorflow/ops/cpu/state.cpp:6-77`` (``KungfuCounter``,
``KungfuExponentialMovingAverage``; EMA semantics of
``srcs/cpp/include/kungfu/utils/ema.hpp``: first update sets the value).
"""
from __future__ import annotations

from typing import Optional


class Counter:
    """Returns init, init+incr, ... on successive calls."""

    def __init__(self, init: int = 0, incr: int = 1, debug: bool = False):
        self.value = init
        self.incr = incr
        self.debug = debug

    def __call__(self) -> int:
        v = self.value
        self.value += self.incr
        if self.debug:
            print("counter: %d" % v)
        return v


class ExponentialMovingAverage:
    def __init__(self, alpha: float = 0.9):
        self.alpha = alpha
        self.value: Optional[float] = None

    def update(self, x: float) -> float:
        x = float(x)
        self.value = x if self.value is None else self.alpha * self.value + (1 - self.alpha) * x
        return self.value

    __call__ = update


def counter(init: int = 0, incr: int = 1, debug: bool = False) -> Counter:
    return Counter(init, incr, debug)


def exponential_moving_average(alpha: float = 0.9) -> ExponentialMovingAverage:
    return ExponentialMovingAverage(alpha)
