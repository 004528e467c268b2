"""Bucketed gradient all-reduce overlapped with backward (the S-SGD engine).

Parity: the reference's gradient synchronisation for S-SGD --
``srcs/python/kungfu/tensorflow/optimizers/sync_sgd.py:78-109`` (per-tensor or
fused NCCL all-reduce, then divide by np) and the NCCL order scheduler
(``srcs/cpp/src/nccl/scheduler.cpp:9-131``: identical collective order on
every rank, learned from rank 0's arrival order).

MI355X design:
* gradients are views of one flat buffer (:class:`FlatParamSpace`); buckets
  are contiguous slices of it, in backward order, so each bucket is one
  in-place RCCL all-reduce -- no pack/unpack.
* a post-accumulate-grad hook counts ready grads per bucket; when a bucket is
  complete it is launched on the high-priority comm stream after an event on
  the compute stream, overlapping with the rest of backward.
* buckets are launched in one fixed order on every rank (a ready bucket waits
  for its predecessors): index order first, then -- from the first step whose
  bucket completions are known -- rank 0's observed completion order,
  broadcast once (the reference scheduler's auto-order), decided by the native
  ``kungfu::OrderedScheduler`` (csrc/runtime/scheduler.cpp).
* an autograd end-of-backward callback launches any bucket whose params got
  no gradient (unused params keep zeros) and makes the compute stream wait
  for the comm stream, so ``loss.backward()`` returns with the reduced
  gradients correctly ordered before the optimizer kernels -- no host sync.
* bucket sizing: the first bucket is small (starts communication early), the
  rest default to 32 MiB: few, large collectives suit RCCL rings over the
  point-to-point xGMI links; tunable via ``KUNGFU_BUCKET_MB``.
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional

import torch

from ..utils.trace import traced
from .comm import get_device_comm
from .flat import FlatParamSpace


class Bucket:
    __slots__ = ("index", "start", "end", "params", "pending", "launched", "staged", "staged_off")

    def __init__(self, index: int, start: int, end: int, params: List[int]):
        self.index, self.start, self.end, self.params = index, start, end, params
        self.pending = len(params)
        self.launched = False
        self.staged: List[torch.Tensor] = []  # direct gradients waiting for the bucket
        self.staged_off: List[int] = []


class GradReducer:
    def __init__(self, space: FlatParamSpace, op: str = "avg", bucket_mb: Optional[float] = None,
                 first_bucket_mb: float = 1.0, comm_dtype: Optional[torch.dtype] = None,
                 skip_single: bool = True):
        # skip_single: with one peer the average of the gradients IS the local
        # gradient, so no collective is issued (the engine's hooks still run).
        self.space = space
        self.op = op
        cap_mb = float(os.environ.get("KUNGFU_BUCKET_MB", bucket_mb if bucket_mb is not None else 32.0))
        esz = space.flat_grad.element_size()
        self.comm = get_device_comm()
        self.comm_dtype = comm_dtype
        # KUNGFU_GPU_ALLREDUCE=graph: buckets follow the session's KungFu strategy graphs
        # (set_tree / set_strategy / adaptation) as device send/recv rounds instead of RCCL's
        # own all-reduce algorithm
        self.graph = os.environ.get("KUNGFU_GPU_ALLREDUCE", "rccl") == "graph"
        self.skip = skip_single and self.comm.size == 1
        self.buckets: List[Bucket] = []
        cap = max(1, int(first_bucket_mb * (1 << 20) / esz))
        start = None
        cur: List[int] = []
        last_end = 0
        for i, (o, n) in enumerate(space.offsets):
            if start is None:
                start = o
            cur.append(i)
            end = o + n
            if (end - start) >= cap:
                self.buckets.append(Bucket(len(self.buckets), start, end, cur))
                cap = max(1, int(cap_mb * (1 << 20) / esz))
                start, cur = None, []
            last_end = end
        if cur:
            self.buckets.append(Bucket(len(self.buckets), start, last_end, cur))
        # pad each bucket to the next param offset so slices tile the buffer
        for b, nb in zip(self.buckets, self.buckets[1:]):
            b.end = nb.start
        self.buckets[-1].end = space.numel
        self.param_bucket = {}
        for b in self.buckets:
            for i in b.params:
                self.param_bucket[i] = b
        # Expected gradient accumulations per param per backward.  Unknown on
        # the first backward (learned, like a static graph): that step reduces
        # every bucket at the end of backward; later steps overlap.
        self._expected: Optional[List[int]] = None
        self._fires = [0] * len(space.params)
        # Collective order (identical on every rank): bucket index order until
        # the auto-order step, then rank 0's observed completion order --
        # kungfu::OrderedScheduler in the C++ runtime.
        from .._lib import runtime

        self.sched = runtime.OrderedScheduler(len(self.buckets))
        self._ordered = False
        self._armed = False
        self._enabled = True
        self._hooks = []
        self._warned = False
        # Optional callbacks (used by the monitoring optimizers):
        #   pre_reduce(bucket, local_grad_view)  on the comm stream, before the all-reduce
        #   post_finish()                        on the compute stream, after all buckets
        self.pre_reduce = None
        self.post_finish = None
        for i, p in enumerate(space.params):
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        # direct gradients (parallel/mixed.py) are delivered to put()
        self._prev_sink = getattr(space, "sink", None)
        space.sink = self
        self._reset()

    # ------------------------------------------------------------------ hooks
    def _make_hook(self, i: int):
        def hook(p):
            if not self._enabled:
                return
            g = p.grad
            v = self.space.grad_view(i)
            if g is not None and g.data_ptr() != v.data_ptr():
                # user replaced .grad (e.g. zero_grad(set_to_none=True)): re-home it
                with torch.no_grad():
                    v.copy_(g)
                p.grad = v
            self._mark(i)

        return hook

    def put(self, i: int, g: torch.Tensor):
        """Sink for direct gradients: stage ``g`` (bf16/f32, the parameter's
        memory layout) for parameter ``i``; it is added into the flat gradient
        buffer by one multi-tensor kernel when its bucket launches."""
        b = self.param_bucket[i]
        o, n = self.space.offsets[i]
        if (not self._enabled or b.launched or g.dtype not in (torch.bfloat16, torch.float32)
                or g.stride() != self.space.strides[i] or not g.is_cuda):
            with torch.no_grad():
                self.space.grad_view(i).add_(g)
        else:
            b.staged.append(g)
            b.staged_off.append(o)
        if self._enabled:
            self._mark(i)

    def _mark(self, i: int):
        if not self._armed:
            self._armed = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finish)
        self._fires[i] += 1
        if self._expected is None:
            return
        b = self.param_bucket[i]
        if b.launched:
            if not self._warned:
                self._warned = True
                print("[kungfu_amd] warning: parameter %s received a gradient after its bucket was "
                      "reduced (dynamic graph); overlap disabled" % self.space.names[i])
            self._expected = None
            return
        b.pending -= 1
        if b.pending == 0:
            for j in self.sched.ready(b.index):
                self._launch(self.buckets[j])

    def _land(self, b: Bucket):
        """Add the bucket's staged direct gradients into the flat buffer (one kernel)."""
        if b.staged:
            from .._lib import hip

            hip().grad_accumulate(self.space.flat_grad, b.staged, b.staged_off, 1.0)
            b.staged, b.staged_off = [], []

    @traced("ssgd::bucket_launch")
    def _launch(self, b: Bucket):
        b.launched = True
        self._land(b)
        if self.skip:
            return
        comm = self.comm
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(comm.device))
        comm.stream.wait_event(ev)
        g = self.space.flat_grad[b.start:b.end]
        if self.pre_reduce is not None:
            with torch.cuda.stream(comm.stream):
                self.pre_reduce(b, g)
        if self.comm_dtype is not None and self.comm_dtype != g.dtype:
            with torch.cuda.stream(comm.stream):
                c = g.to(self.comm_dtype)
                self._reduce(comm, c)
                g.copy_(c)
                c.record_stream(comm.stream)
        else:
            self._reduce(comm, g)

    def _reduce(self, comm, g):
        if not self.graph:
            comm.all_reduce(g, op=self.op)
            return
        comm.graph_all_reduce(g, op="sum")
        if self.op == "avg":
            with torch.cuda.stream(comm.stream):
                g.mul_(1.0 / comm.size)

    def _finish(self):
        for j in self.sched.flush():
            if not self.buckets[j].launched:
                self._launch(self.buckets[j])
        if not self.skip:
            torch.cuda.current_stream(self.comm.device).wait_stream(self.comm.stream)
        if self._expected is not None and not self._ordered and not self.skip:
            # first step with known bucket completion: every rank adopts rank 0's
            # arrival order for its collectives from now on (native auto-order)
            self.sched.auto_order()
            self._ordered = True
        if self._expected is None and not self._warned:
            self._expected = list(self._fires)
        self._reset()
        if self.post_finish is not None:
            self.post_finish()

    def _reset(self):
        for b in self.buckets:
            b.pending = sum(self._expected[i] for i in b.params) if self._expected is not None else 1
            b.launched = False
        self._fires = [0] * len(self.space.params)
        self.sched.reset()
        self._armed = False

    # ------------------------------------------------------------------ API
    def synchronize(self):
        """Called by the optimizer before stepping (no-op when the backward
        callback already ran)."""
        if self._armed:
            self._finish()

    def reduce_all_now(self):
        """Reduce every bucket immediately (for grads computed without hooks)."""
        self._reset()
        for j in self.sched.flush():
            self._launch(self.buckets[j])
        if not self.skip:
            torch.cuda.current_stream(self.comm.device).wait_stream(self.comm.stream)

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (gradient accumulation micro-steps)."""
        old = self._enabled
        self._enabled = False
        try:
            yield
        finally:
            self._enabled = old

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if getattr(self.space, "sink", None) is self:
            self.space.sink = self._prev_sink
