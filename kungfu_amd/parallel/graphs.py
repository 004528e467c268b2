"""Whole-step hipGraph capture: one training step (zero_grad + forward + backward with the
bucketed RCCL all-reduces + the fused optimizer) recorded once and replayed as ONE graph launch.

Why: the eager step is a few hundred kernel launches issued from Python (autograd, the fused
blocks' bookkeeping, the bucket hooks); the host needs ~16 ms to enqueue a ResNet-50 step whose
GPU time is ~21 ms (``tools/diag/cpu_overhead.py``), so any extra host work per step -- more
ranks' RCCL enqueues, slower host CPUs -- would make the step host-bound.  A replay costs the
host one ``hipGraphLaunch``.

What makes a step capturable here:
* every kernel of the engine is launched on the current / comm stream with device-resident
  arguments; host-side decisions (bucket order, BN links, tile choices) are made at capture time
  and stay valid because the replayed step has the same shapes and pointers (static inputs);
* per-step scalars that change between replays live in device tensors refreshed before each
  replay (:meth:`GraphedStep.pre_replay`: the fused optimizers' learning rate);
* the RCCL bucket collectives are captured on the comm stream, which joins the capture through
  the engine's event fence / join; the native watchdog skips registrations made while a stream
  is capturing (graph replays are not watched -- ``rccl_comm.hip`` ``watch``);
* capture happens after ``warmup`` eager steps, once the bucket engine has learned its
  collective order (rank 0's order is adopted on the second step) and every lazily allocated
  workspace (BN statistics slots, flip caches, comm buffers) exists.

N-rank steps: the step is captured as a chain of graph
SEGMENTS cut at every bucket launch and at the end-of-backward join; a replay runs segment 0, issues
the bucket's RCCL collective eagerly on the comm stream (event-fenced after the segment), replays
segment 1, ... -- the compute stream never carries a collective, and the collectives overlap the
following segments exactly as in an eager step (one whole-step graph with the collectives inside
hid them worse than eager streams: r4t33, r5t3).  Host cost per step: one graph launch per segment
plus one RCCL call per bucket.  The segments share one memory pool and are replayed in capture order.

Limits: inputs must be static tensors the caller refills in place; the step's Python code runs
only at capture (counters it keeps stop advancing).  Dropout: the attention / add+LayerNorm
kernels hash a host seed recorded at capture with a device word that :meth:`pre_replay`
advances (``ops.dropout_seed``), so every replay draws fresh masks.  Parity: none in the reference (TF
graphs are its equivalent); MI355X-first replacement for a tracing compiler.
"""
from __future__ import annotations

import weakref
from typing import Callable, List, Optional

import torch

from .. import knobs

# Every captured graph that may hold RCCL collectives: RCCL keeps per-graph resources alive until the
# graph is destroyed, and finalizing the communicator first waits for them (a hang at exit, measured
# with 2 colocated ranks) -- kungfu_amd.finalize() releases these graphs before the communicators.
_live = weakref.WeakSet()


def track(graph: torch.cuda.CUDAGraph) -> torch.cuda.CUDAGraph:
    """Register a captured graph for :func:`release_all` (called by ``kungfu_amd.finalize``)."""
    _live.add(graph)
    return graph


def release_all() -> None:
    """Destroy every tracked graph (device-synchronised first)."""
    if not _live:
        return
    try:
        torch.cuda.synchronize()
    except Exception:  # noqa: BLE001 -- shutting down
        pass
    for g in list(_live):
        try:
            g.reset()
        except Exception:  # noqa: BLE001
            pass
    _live.clear()


def _lr_holders(opt) -> List[object]:
    """Objects with a device ``_lr_t`` scalar mirroring ``param_groups[0]['lr']``."""
    out, seen = [], set()
    stack = [opt]
    while stack:
        o = stack.pop()
        if o is None or id(o) in seen:
            continue
        seen.add(id(o))
        if hasattr(o, "_lr_t") and hasattr(o, "param_groups"):
            out.append(o)
        for attr in ("inner", "optimizer", "_opt"):
            stack.append(getattr(o, attr, None))
    return out


def _drain_watchdog(timeout_s: float = 2.0) -> None:
    """Wait (after a device synchronize) until the native RCCL watchdog has retired every event:
    its thread polls every 50 ms, and an event recorded before the capture on a stream that then
    joins the capture cannot be queried during it."""
    import time

    from .._lib import hip, hip_available

    if not hip_available():
        return
    t_end = time.time() + timeout_s
    while hip().rccl_watchdog_info()["pending"] and time.time() < t_end:
        time.sleep(0.01)


def _graph_nodes(g: torch.cuda.CUDAGraph) -> int:
    """Node count of a captured (kept, not yet instantiated) graph: hipGraphGetNodes."""
    import ctypes

    global _HIP_RT
    if _HIP_RT is None:
        _HIP_RT = ctypes.CDLL("libamdhip64.so")
        _HIP_RT.hipGraphGetNodes.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
        _HIP_RT.hipGraphGetNodes.restype = ctypes.c_int
    n = ctypes.c_size_t(0)
    rc = _HIP_RT.hipGraphGetNodes(ctypes.c_void_p(g.raw_cuda_graph()), None, ctypes.byref(n))
    if rc != 0:
        raise RuntimeError("hipGraphGetNodes failed (%d)" % rc)
    return int(n.value)


_HIP_RT = None


class GraphedStep:
    """``step = GraphedStep(fn, optimizer)``; ``loss = step()`` runs ``fn`` eagerly for ``warmup``
    calls, then captures it and replays the graph on every later call (returning the captured
    output tensor, refreshed by each replay)."""

    def __init__(self, fn: Callable[[], torch.Tensor], optimizer=None, warmup: int = 3,
                 capture_error_mode: str = "thread_local"):
        self.fn = fn
        self.opt = optimizer
        self.warmup = warmup
        self.mode = capture_error_mode
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        # segmented capture: graph segments and the replay program [("g", k) | ("bucket", j) | ("join",)]
        self.segs: List[torch.cuda.CUDAGraph] = []
        self.program: List[tuple] = []
        self._cur: Optional[torch.cuda.CUDAGraph] = None
        self._pool = None
        self.out = None
        self.calls = 0
        self.replays = 0
        self.disabled = False
        self._lr = _lr_holders(optimizer) if optimizer is not None else []
        # warm-up AND capture run on this one side stream: autograd's AccumulateGrad nodes remember
        # the stream they were created on, and a node created on the default stream by a warm-up step
        # whose graph is still alive (a kept loss tensor) makes the capture wait across streams
        self.stream = torch.cuda.Stream()

    def pre_replay(self):
        from ..ops import dropout_seed

        for o in self._lr:
            o._lr_t.fill_(o.param_groups[0]["lr"])
        dropout_seed.advance()  # fresh hashed dropout masks for this replay

    def capture(self) -> bool:
        """Record one step.  Every rank must agree: a capture that failed anywhere (an op that
        cannot be captured) is dropped on ALL ranks, which then stay eager -- nothing ran during
        any rank's capture, so the ranks' collective sequences stay aligned."""
        from .._lib import runtime

        torch.cuda.synchronize()
        _drain_watchdog()  # no RCCL completion event left to query while streams are capturing
        g = torch.cuda.CUDAGraph()
        err = None
        reducer = getattr(self.opt, "reducer", None)
        plane = getattr(getattr(reducer, "comm", None), "plane", "rccl") if reducer is not None else "rccl"
        if plane not in ("rccl", "emulate", "skip"):
            # the host-staged plane synchronises and copies through host memory inside every
            # collective: not capturable (decided identically on every rank, nothing attempted)
            err = RuntimeError("the %s data plane cannot be captured" % plane)
        comm = getattr(reducer, "comm", None)
        # the N-rank layout (comm stream as the capture's origin): real multi-rank RCCL, and the 1-GPU
        # emulation of an N-rank job (bench.py --emulate-comm), which must model the same graph shape
        multi = reducer is not None and ((plane == "rccl" and getattr(comm, "size", 1) > 1)
                                         or (plane == "emulate" and getattr(comm, "ranks", 1) > 1))
        if err is None and getattr(reducer, "_hier", None) is not None:
            # hierarchical across hosts: a host thread all-reduces between the local reduce and the
            # local broadcast -- host work inside the step, not capturable
            err = RuntimeError("the cross-host hierarchical all-reduce cannot be captured")
        elif multi and knobs.get("KUNGFU_GRAPH_MULTIRANK") != "1":
            err = RuntimeError("multi-rank RCCL capture is disabled (KUNGFU_GRAPH_MULTIRANK=0)")
        try:
            if err is not None:
                raise err
            if multi:
                # N ranks: graph segments cut at every bucket launch, the collectives issued eagerly
                # between replays.  (Round 6: the whole-graph layout with the collectives inside -- the
                # comm stream as the capture's origin, compute forked from it -- is gone: measured
                # slower (r5t6) and its capture failed intermittently inside RCCL on colocated ranks.)
                self._capture_segments(reducer)
            else:
                with torch.cuda.graph(g, stream=self.stream, capture_error_mode=self.mode):
                    self.out = self.fn()
        except Exception as e:  # noqa: BLE001 -- reported, then the step runs eagerly
            err = e
            if self._cur is not None:  # a segment still capturing: end it (discarded)
                try:
                    with torch.cuda.stream(self.stream):
                        self._cur.capture_end()
                except Exception:  # noqa: BLE001
                    pass
                self._cur = None
            reducer = getattr(self.opt, "reducer", None)
            if reducer is not None:
                reducer.segmenter = None
            self.segs, self.program = [], []
        torch.cuda.synchronize()
        ok = err is None
        if runtime.size() > 1:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
            from .. import ops

            ok = bool(ops.all_reduce(flag, op="min", name="kf:graph:capture_ok:%d" % self.calls).item())
        if not ok:
            import sys

            print("kungfu_amd: whole-step hipGraph capture %s; training continues eagerly" % (
                "failed: %s" % err if err is not None else "failed on another rank"), file=sys.stderr, flush=True)
            self.out, self.disabled = None, True
            reducer = getattr(self.opt, "reducer", None)
            if reducer is not None:  # the aborted step left its bucket bookkeeping half done
                reducer._reset_buckets()
            return False
        if self.segs:
            for sg in self.segs:
                track(sg)
            self.graph = self.segs[-1]
        else:
            self.graph = track(g)
        return True

    # ------------------------------------------------------------ segmented capture
    def _begin(self):
        # keep_graph: the captured graph is instantiated only after the capture, so segments that
        # captured nothing (two cut points with no kernel between) can be dropped first
        g = torch.cuda.CUDAGraph(keep_graph=True)
        # "relaxed": a segment begun on the caller's thread is ended by the autograd worker thread at
        # a bucket launch (thread-local captures must end on the thread that began them)
        g.capture_begin(pool=self._pool, capture_error_mode="relaxed")
        self._cur = g

    def _end(self):
        self._cur.capture_end()
        self.segs.append(self._cur)
        self.program.append(("g", len(self.segs) - 1))
        self._cur = None

    def cut(self, op: tuple):
        """Called by the reducer (on the capturing stream) at a bucket launch / the final join: end the
        current segment, record ``op`` for the replay program, begin the next segment."""
        self._end()
        self.program.append(op)
        self._begin()

    def _capture_segments(self, reducer):
        import gc

        gc.collect()
        self.segs, self.program = [], []
        self._pool = torch.cuda.graph_pool_handle()
        reducer.segmenter = self
        try:
            with torch.cuda.stream(self.stream):
                self._begin()
                self.out = self.fn()
                self._end()
        finally:
            reducer.segmenter = None
        if not any(op[0] == "join" for op in self.program):
            raise RuntimeError("segmented capture saw no end-of-backward join (no bucket engine in the step?)")
        # drop the empty segments (each graph launch costs the GPU a few microseconds), instantiate the rest
        keep, prog = [], []
        for op in self.program:
            if op[0] == "g":
                sg = self.segs[op[1]]
                if _graph_nodes(sg) == 0:
                    sg.reset()
                    continue
                sg.instantiate()
                keep.append(sg)
                op = ("g", len(keep) - 1)
            prog.append(op)
        self.segs, self.program = keep, prog

    def _replay_segments(self):
        reducer = self.opt.reducer
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            for op in self.program:
                if op[0] == "g":
                    self.segs[op[1]].replay()
                elif op[0] == "bucket":
                    reducer._issue(reducer.buckets[op[1]])
                else:
                    reducer.comm.join()
        cur.wait_stream(self.stream)
        reducer.steps += 1  # names the next replay's collectives for the watchdog

    def _eager(self):
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            out = self.fn()
        cur.wait_stream(self.stream)
        return out

    def __call__(self):
        self.calls += 1
        if self.graph is None:
            if self.calls <= self.warmup or self.disabled:
                return self._eager()
            if not self.capture():  # records without executing: replay now so this call did a step
                return self._eager()
        self.pre_replay()
        if self.segs:
            self._replay_segments()
        else:
            self.graph.replay()
        self.replays += 1
        return self.out
