"""KungFu global training variables (batch size, gradient noise scale, sample counters).

Parity: ``srcs/python/kungfu/tensorflow/variables.py:6-122`` (GraphKeys
BATCH_SIZE / GRADIENT_NOISE_SCALE / TOTAL_SAMPLES / TRAINED_SAMPLES,
get_or_create_*, eval_*, create_setter).  TF graph collections become a
process-wide registry of named values; policies and elastic hooks read and
write them.
"""
from __future__ import annotations

import threading
from typing import Any, Callable, Dict, Optional


class GraphKeys:
    BATCH_SIZE = "kungfu_batch_size"
    GRADIENT_NOISE_SCALE = "kungfu_gradient_noise_scale"
    TOTAL_SAMPLES = "kungfu_total_samples"
    TRAINED_SAMPLES = "kungfu_trained_samples"


_lock = threading.Lock()
_vars: Dict[str, Any] = {}


def get_global_variable(name: str) -> Optional[Any]:
    with _lock:
        v = _vars.get(name)
    return v() if callable(v) else v


def create_global_variable(name: str, init: Any = 0):
    with _lock:
        if name in _vars:
            raise ValueError('"%s" already exists.' % name)
        _vars[name] = init
    return init


def get_or_create_global_variable(name: str, init: Any = 0):
    with _lock:
        if name not in _vars:
            _vars[name] = init
        v = _vars[name]
    return v() if callable(v) else v


def set_global_variable(name: str, value: Any):
    with _lock:
        _vars[name] = value


def eval_global_variable(name: str):
    v = get_global_variable(name)
    if v is None:
        raise RuntimeError('"%s" not exist' % name)
    return v


def create_setter(name: str) -> Callable[[Any], None]:
    return lambda value: set_global_variable(name, value)


def reset():
    with _lock:
        _vars.clear()


def get_or_create_batch_size(init: int = 0) -> int:
    return get_or_create_global_variable(GraphKeys.BATCH_SIZE, init)


def get_batch_size() -> Optional[int]:
    return get_global_variable(GraphKeys.BATCH_SIZE)


def eval_batch_size() -> int:
    return eval_global_variable(GraphKeys.BATCH_SIZE)


def get_or_create_total_samples(init: int = 0) -> int:
    return get_or_create_global_variable(GraphKeys.TOTAL_SAMPLES, init)


def get_or_create_trained_samples(init: int = 0) -> int:
    return get_or_create_global_variable(GraphKeys.TRAINED_SAMPLES, init)


def set_gradient_noise_scale(source) -> None:
    """Registers the GNS optimizer (value read lazily, no host sync here)."""
    set_global_variable(GraphKeys.GRADIENT_NOISE_SCALE, lambda: source.noise_scale)


def eval_gradient_noise_scale() -> Optional[float]:
    return get_global_variable(GraphKeys.GRADIENT_NOISE_SCALE)
