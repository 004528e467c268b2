"""Scoped tracing: roctx ranges + per-scope timing statistics.

Parity: the reference's ``TRACE_SCOPE`` macros (``srcs/cpp/include/kungfu/utils/trace.hpp:1-16``,
compiled in with ``KUNGFU_ENABLE_TRACE``) around NCCL ops and the event spin-wait.  Here
tracing is a run-time switch, ``KUNGFU_CONFIG_ENABLE_TRACE=true``:

* every scope pushes a roctx range (``rocprofv3 --marker-trace`` shows bucket all-reduces,
  optimizer steps, pair-averaging pulls next to the kernels they enqueue);
* host wall time per scope name is accumulated in the native runtime and printed as
  ``[trace] name count= total= mean=`` lines at exit (``trace_report()``).

Native collectives (``session::all_reduce``, ``session::barrier``, ...) are traced by the C++
runtime itself.  Disabled tracing costs one cached boolean check per scope.
"""
from __future__ import annotations

import contextlib
import functools
import os
import time

_ENABLED = os.environ.get("KUNGFU_CONFIG_ENABLE_TRACE", "false").lower() in ("1", "true", "yes", "on")


def enabled() -> bool:
    return _ENABLED


def _rt():
    from .._lib import runtime

    return runtime


@contextlib.contextmanager
def scope(name: str):
    """``with trace.scope("ssgd::bucket"):`` -- a roctx range + a timing sample."""
    if not _ENABLED:
        yield
        return
    rt = _rt()
    rt.trace_push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        rt.trace_record(name, time.perf_counter() - t0)
        rt.trace_pop()


def traced(name: str):
    """Decorator form of :func:`scope`."""

    def deco(f):
        @functools.wraps(f)
        def g(*a, **k):
            if not _ENABLED:
                return f(*a, **k)
            with scope(name):
                return f(*a, **k)

        return g

    return deco


def report() -> str:
    """Accumulated ``[trace]`` statistics of this process (native + Python scopes)."""
    return _rt().trace_report()
