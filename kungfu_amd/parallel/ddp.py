"""Bucketed gradient all-reduce overlapped with backward (the S-SGD engine).

Parity: the reference's gradient synchronisation for S-SGD --
``srcs/python/kungfu/tensorflow/optimizers/sync_sgd.py:78-109`` (per-tensor or
fused NCCL all-reduce, then divide by np), the NCCL order scheduler
(``srcs/cpp/src/nccl/scheduler.cpp:9-131``: identical collective order on
every rank, learned from rank 0's arrival order) and the NCCL re-initialisation
after a resize (``srcs/cpp/src/tensorflow/ops/gpu/scheduler.cpp:54-68``).

MI355X design:
* gradients are views of one flat buffer (:class:`FlatParamSpace`); buckets
  are contiguous slices of it, in backward order, so each bucket is one
  in-place RCCL all-reduce -- no pack/unpack.
* a post-accumulate-grad hook counts ready grads per bucket; when a bucket is
  complete it is launched on the comm stream (normal priority, see
  ``comm.py``) after an event on the compute stream, overlapping with the rest
  of backward.
* buckets are launched in one fixed order on every rank (a ready bucket waits
  for its predecessors): index order first, then -- from the second step after
  (re)binding to a communicator -- rank 0's observed completion order,
  broadcast once (the reference scheduler's auto-order), decided by the native
  ``kungfu::OrderedScheduler`` (csrc/runtime/scheduler.cpp).  The per-gradient
  bookkeeping (arrival counts, per-bucket countdown, launched flags, late
  detection, the scheduler query) is ONE native call per hook,
  ``kungfu::BucketTracker::mark``.
* an autograd end-of-backward callback launches any bucket whose params got
  no gradient (unused params keep zeros) and makes the compute stream wait
  for the comm stream, so ``loss.backward()`` returns with the reduced
  gradients correctly ordered before the optimizer kernels -- no host sync.
* the communicator is bound lazily, at the first gradient of a backward, and
  re-bound whenever the cluster changed (elastic resize): the peer count
  (``skip``), the scheduler and its learned order are rebuilt for the new
  membership.  Nothing collective happens in the constructor, so a worker
  that joins a running job constructs its optimizer without blocking on
  peers that are still inside their own step.
* a gradient that arrives after its bucket was launched (a parameter used
  more times than during the step the engine learned from) is an error, as in
  ``torch.nn.parallel.DistributedDataParallel``: the autograd engine has
  already accumulated it into the slice RCCL is reducing, so the step cannot
  be repaired consistently on every rank.  Parameters used several times per
  step are fine (their accumulation count is learned on the first step);
  models whose use count changes between steps need ``overlap=False``.
* bucket sizing: the first bucket is small (starts communication early), the
  rest default to 32 MiB: few, large collectives suit RCCL rings over the
  point-to-point xGMI links; tunable via ``KUNGFU_BUCKET_MB``.  The last
  ``tail_bucket_mb`` (4 MiB, ``KUNGFU_TAIL_BUCKET_MB``) of the buffer -- the first
  layers, whose gradients arrive last -- is bucketed separately so the
  collective that cannot overlap with backward is small.
* ``comm_dtype=torch.bfloat16`` halves the bytes on the wire: the bucket is
  cast into a persistent bf16 comm buffer on the comm stream (HIP kernel),
  reduced there, and cast back (f32 accumulation stays in the flat buffer).
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional

import torch

from ..utils.trace import traced
from .comm import comm_epoch, get_device_comm
from .flat import FlatParamSpace


class Bucket:
    __slots__ = ("index", "start", "end", "params", "launched", "staged", "staged_off")

    def __init__(self, index: int, start: int, end: int, params: List[int]):
        self.index, self.start, self.end, self.params = index, start, end, params
        self.launched = False
        self.staged: List[torch.Tensor] = []  # direct gradients waiting for the bucket
        self.staged_off: List[int] = []


class LateGradientError(RuntimeError):
    pass


class _CrossHostStage:
    """The middle and last steps of a hierarchical bucket all-reduce with several hosts
    (parity: ``CrossAllReduceGpu``, srcs/cpp/src/nccl/controller.cpp:8-40): one worker
    thread takes the buckets in launch order -- the same order on every rank -- and, on
    the host's root, waits for the local reduce, stages the bucket through host memory,
    all-reduces it among the local roots over the host transport and copies it back; then
    every local rank issues the local broadcast on a SECOND local communicator from this
    thread (each communicator is driven by exactly one thread, in one order).  Backward
    keeps running meanwhile; ``drain`` (end of backward) waits for the queue and orders
    the compute stream after the broadcasts."""

    def __init__(self, reducer: "GradReducer", bcast_comm):
        import queue
        import threading

        from .._lib import runtime

        self.r, self.bcast = reducer, bcast_comm
        self.cuda = reducer.space.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=reducer.space.device) if self.cuda else None
        self.root = runtime.local_rank() == 0
        self.size = runtime.size()
        self.version = runtime.cluster_version()
        self.q = queue.Queue()
        self.err = None
        self.seq = 0
        self.th = threading.Thread(target=self._loop, name="kungfu-cross-host", daemon=True)
        self.th.start()

    def submit(self, g: torch.Tensor, tag: str, post=None):
        """``post()``: issued on the stage stream after the local broadcast (e.g. the cast of
        a bf16 wire buffer back into the f32 gradient) -- it must not run on the comm stream,
        which is not ordered after this stage's work."""
        ev = None
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(self.r.comm.stream)
        self.seq += 1
        self.q.put((g, ev, tag, self.seq, post))

    def _loop(self):
        from .._lib import dtype_code, op_code, runtime

        if self.cuda:
            torch.cuda.set_device(self.r.space.device)
        while True:
            item = self.q.get()
            if item is None:
                self.q.task_done()
                return
            g, ev, tag, seq, post = item
            try:
                ctx = torch.cuda.stream(self.stream) if self.cuda else contextlib.nullcontext()
                with ctx:
                    if self.cuda:
                        self.stream.wait_event(ev)
                    if self.root:
                        if self.cuda:
                            ev.synchronize()
                            h = g.to("cpu")
                        else:
                            h = g
                        runtime.cross_all_reduce(h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h), op_code("sum"),
                                                 "kf:hier:v%d:%d" % (self.version, seq))
                        if self.r.op == "avg":
                            h.mul_(1.0 / self.size)
                        if self.cuda:
                            g.copy_(h)
                    self.bcast.broadcast(g, root=0, stream=self.stream, tag=tag + " (local broadcast)")
                    if post is not None:
                        post()
            except BaseException as e:  # noqa: BLE001 -- re-raised by drain()
                self.err = e
            self.q.task_done()

    def drain(self):
        self.q.join()
        if self.err is not None:
            e, self.err = self.err, None
            raise e
        if self.cuda:
            torch.cuda.current_stream(self.r.space.device).wait_stream(self.stream)

    def stop(self):
        self.q.put(None)
        self.th.join(timeout=30)


class GradReducer:
    def __init__(self, space: FlatParamSpace, op: str = "avg", bucket_mb: Optional[float] = None,
                 first_bucket_mb: float = 1.0, comm_dtype: Optional[torch.dtype] = None,
                 tail_bucket_mb: float = 4.0,
                 skip_single: bool = True, monitored: bool = False, hierarchical: bool = False):
        # skip_single: with one peer the average of the gradients IS the local
        # gradient, so no collective is issued (the engine's hooks still run).
        # skip_single=False sends every bucket through the communicator even
        # with one peer (exercises the RCCL path / stream ordering at N=1).
        self.space = space
        self.op = op
        self.skip_single = skip_single
        # monitored: every bucket's all-reduce feeds the session's strategy statistics
        # (SynchronousSGDOptimizer(monitor=True); parity sync_sgd.py:96-97)
        self.monitored = monitored
        # hierarchical: local reduce -> cross-host all-reduce among the hosts' local roots ->
        # local broadcast, per bucket, during backward (the reference's
        # ScheduledHierarchicalNcclAllReduce per tensor through its ordered scheduler,
        # srcs/cpp/src/tensorflow/ops/gpu/collective.cpp:105-156)
        self.hierarchical = hierarchical
        self._hier = None
        cap_mb = float(os.environ.get("KUNGFU_BUCKET_MB", bucket_mb if bucket_mb is not None else 32.0))
        esz = space.flat_grad.element_size()
        if comm_dtype is not None and comm_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("comm_dtype must be float32 or bfloat16")
        self.comm_dtype = comm_dtype if comm_dtype != space.flat_grad.dtype else None
        if self.comm_dtype is not None and space.device.type != "cuda":
            self.comm_dtype = None  # host transport: f32 on the wire
        self._cbuf: Optional[torch.Tensor] = None
        # KUNGFU_GPU_ALLREDUCE=graph: buckets follow the session's KungFu strategy graphs
        # (set_tree / set_strategy / adaptation) as device send/recv rounds instead of RCCL's
        # own all-reduce algorithm
        self.graph = os.environ.get("KUNGFU_GPU_ALLREDUCE", "rccl") == "graph"
        self.buckets: List[Bucket] = []
        cap = max(1, int(first_bucket_mb * (1 << 20) / esz))
        # The last bucket is launched only when backward has produced its final
        # gradient, so its whole all-reduce is exposed: the tail of the buffer (the
        # model's first layers) gets buckets of at most tail_mb.
        tail_mb = float(os.environ.get("KUNGFU_TAIL_BUCKET_MB", tail_bucket_mb))
        tail_cap = max(1, int(tail_mb * (1 << 20) / esz))
        tail_start = space.numel - tail_cap
        start = None
        cur: List[int] = []
        last_end = 0
        for i, (o, n) in enumerate(space.offsets):
            if start is None:
                start = o
            cur.append(i)
            end = o + n
            nxt = space.offsets[i + 1][0] if i + 1 < len(space.offsets) else None
            # close before the next param crosses into the tail region (keeps the tail separate)
            enter_tail = nxt is not None and start < tail_start <= nxt + space.offsets[i + 1][1] and end <= tail_start
            if (end - start) >= cap or (enter_tail and end - start > 0) or (start >= tail_start and end - start >= tail_cap):
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
        from .._lib import runtime

        # Native per-gradient accounting (csrc/runtime/scheduler.cpp BucketTracker): expected
        # gradient accumulations per param per backward are unknown on the first backward (learned,
        # like a static graph: that step reduces every bucket at the end of backward); later steps
        # count each bucket down and launch it, in the scheduler's order, when it completes.
        self.tracker = runtime.BucketTracker(len(self.buckets),
                                             [self.param_bucket[i].index for i in range(len(space.params))])
        self._late_code = runtime.BucketTracker.LATE
        # Communicator binding (lazy; see _bind).
        self.comm = None
        self.skip = True
        self._bound = None  # (cluster version, comm epoch) bound at
        self._steps_bound = 0  # completed backward passes since the last (re)bind
        self._ordered = False
        self.rebinds = 0
        self.steps = 0  # completed backward passes (names collectives for the watchdog)
        self._tag = ""
        self._armed = False
        self._enabled = True
        self._hooks = []
        # Optional callbacks (used by the monitoring optimizers):
        #   pre_reduce(bucket, local_grad_view)  on the comm stream, before the all-reduce
        #   post_finish()                        on the compute stream, after all buckets
        self.pre_reduce = None
        self.post_finish = None
        # comm probe (bench.py verify.comm_per_bucket_ms / exposed_comm_ms): when a list, every
        # backward appends its per-bucket HIP timing events (see :meth:`probe_summary`)
        self.probe: Optional[list] = None
        self._probe_cur = None
        # set by a segmented GraphedStep capture (parallel/graphs.py): bucket launches and the
        # end-of-backward join become cut points between captured graph segments
        self.segmenter = None
        for i, p in enumerate(space.params):
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        # direct gradients (parallel/mixed.py) are delivered to put()
        self._prev_sink = getattr(space, "sink", None)
        space.sink = self
        self._reset_buckets()

    # ------------------------------------------------------------ binding
    def _bind(self):
        """(Re)bind to the current cluster: called at the start of every backward.
        Cheap when nothing changed (two integer reads)."""
        from .._lib import runtime

        key = (runtime.cluster_version(), comm_epoch())
        if key == self._bound:
            return
        size = runtime.size()
        self.skip = self.skip_single and size == 1
        if self._hier is not None:
            self._hier.stop()
            self._hier = None
        if self.hierarchical and not self.skip:
            self.comm = get_device_comm("local", device=self.space.device)
            if runtime.host_count() > 1:
                self._hier = _CrossHostStage(self, get_device_comm("local:bcast", device=self.space.device))
        else:
            self.comm = None if self.skip else get_device_comm(device=self.space.device)
        # The learned collective order belongs to the old membership: start again
        # from index order; the new rank 0's arrival order is adopted after one step.
        self.tracker.set_order(list(range(len(self.buckets))))
        self._ordered = False
        self._steps_bound = 0
        if self._bound is not None:
            self.rebinds += 1
        self._bound = key

    @property
    def bytes_per_step(self) -> int:
        """Bytes each rank hands to the collective per step (0 when skipped)."""
        if self.skip:
            return 0
        esz = torch.empty((), dtype=self.comm_dtype or self.space.flat_grad.dtype).element_size()
        return self.space.numel * esz

    def describe(self) -> dict:
        from .._lib import runtime

        return {
            "hierarchical": self.hierarchical,
            "buckets": len(self.buckets),
            "bucket_mb": round(max(b.end - b.start for b in self.buckets) * self.space.flat_grad.element_size()
                               / (1 << 20), 2),
            "comm_ranks": (self.comm.size if self.comm is not None and not self.hierarchical else runtime.size()),
            "comm_plane": ("skip" if self.skip else getattr(self.comm, "plane", "?")),
            "comm_dtype": str(self.comm_dtype or self.space.flat_grad.dtype).replace("torch.", ""),
            "comm_bytes_per_step": self.bytes_per_step,
            "overlap": True,
        }

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
        if self._enabled and b.launched:
            self._late(i)  # raises unless no collective is in flight (one peer)
        # a late gradient (its bucket already landed) is added now: staging it would
        # carry it into the next step's gradient
        if (not self._enabled or b.launched or g.dtype not in (torch.bfloat16, torch.float32)
                or g.stride() != self.space.strides[i] or not g.is_cuda):
            from .mixed import SideStream

            SideStream.join()
            with torch.no_grad():
                self.space.grad_view(i).add_(g)
        else:
            b.staged.append(g)
            b.staged_off.append(o)
        if self._enabled:
            self._mark(i)

    def put_direct(self, i: int):
        """Sink for a direct gradient its producer already added into parameter ``i``'s flat f32
        slot on the compute stream (ops/linear.py's split-K reduce): only the bucket accounting."""
        b = self.param_bucket[i]
        if self._enabled and b.launched:
            self._late(i)  # (already added: with one peer nothing else to do)
        if self._enabled:
            self._mark(i)

    def _late(self, i: int):
        if self.skip:  # no collective in flight: the late gradient simply accumulates
            return
        raise LateGradientError(
            "kungfu_amd: parameter %r received a gradient after its bucket's all-reduce was launched "
            "(it was used more often in this backward than in the step the engine learned from). Use "
            "SynchronousSGDOptimizer(..., overlap=False) for models whose parameter use changes between "
            "steps." % self.space.names[i])

    def _mark(self, i: int):
        if not self._armed:
            self._armed = True
            self._bind()
            torch.autograd.Variable._execution_engine.queue_callback(self._finish)
        go = self.tracker.mark(i)
        if go:
            if go[0] == self._late_code:
                self._late(i)
                return
            for j in go:
                self._launch(self.buckets[j])

    def _land(self, b: Bucket):
        """Add the bucket's staged direct gradients into the flat buffer (one kernel)."""
        if b.staged:
            from .._lib import hip
            from .mixed import SideStream

            SideStream.join()  # weight gradients still running on the side stream
            hip().grad_accumulate(self.space.flat_grad, b.staged, b.staged_off, 1.0)
            b.staged, b.staged_off = [], []

    @traced("ssgd::bucket_launch")
    def _launch(self, b: Bucket):
        b.launched = True
        from .mixed import SideStream

        SideStream.join()  # direct weight gradients reduced into this bucket on the side stream
        self._land(b)
        if self.skip:
            return
        if self.segmenter is not None:
            # segmented capture (parallel/graphs.py): the compute captured so far becomes one graph
            # segment; this bucket's collective is issued eagerly between segment replays
            self.segmenter.cut(("bucket", b.index))
            return
        self._issue(b)

    def _issue(self, b: Bucket):
        """The comm-stream side of a bucket launch: fence, pre-reduce callback, wire cast, collective."""
        comm = self.comm
        # names the collective for the watchdog: "bucket 3/5 of step 12"
        self._tag = "bucket %d/%d of step %d" % (b.index, len(self.buckets), self.steps)
        probe = self._probe_begin(comm, b)
        comm.fence()
        g = self.space.flat_grad[b.start:b.end]
        if self.pre_reduce is not None:
            with comm.on_stream():
                self.pre_reduce(b, g)
        if self.comm_dtype is not None:
            from .._lib import hip

            if self._cbuf is None:
                self._cbuf = torch.empty(self.space.numel, dtype=self.comm_dtype, device=self.space.device)
            c = self._cbuf[b.start:b.end]
            with comm.on_stream():
                hip().cast_copy(c, g, 1.0)

            def cast_back():  # on whichever stream the reduction of ``c`` ends
                hip().cast_copy(g, c, 1.0)

            self._reduce(comm, c, post=cast_back)
        else:
            self._reduce(comm, g)
        if probe is not None:
            with comm.on_stream():
                probe[-1].record()

    # ------------------------------------------------------------ comm probe
    def _probe_begin(self, comm, b: Bucket):
        """Timing events of one bucket: ready (compute stream: its last gradient produced), start /
        end of its collective (comm stream).  None unless probing a device plane."""
        if self.probe is None or getattr(comm, "stream", None) is None or self._hier is not None:
            return None
        if self._probe_cur is None:
            self._probe_cur = {"buckets": [], "bwd_end": None}
        ready, st, en = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        ready.record()
        comm.fence()
        with comm.on_stream():
            st.record()
        rec = [b.index, (b.end - b.start) * self.space.flat_grad.element_size(), ready, st, en]
        self._probe_cur["buckets"].append(rec)
        return rec

    def probe_summary(self) -> Optional[dict]:
        """Per-bucket collective time and the exposed communication tail over the probed steps
        (medians; synchronises the device).  ``comm_per_bucket_ms``: device time of each bucket's
        collective, in launch order; ``wait_per_bucket_ms``: from the bucket's gradients being
        ready to its collective starting (queueing behind earlier buckets); ``exposed_comm_ms``:
        from the end of backward's compute to the end of the last collective -- the part of the
        communication the step could not hide."""
        steps = [r for r in (self.probe or []) if r["buckets"] and r["bwd_end"] is not None]
        if not steps:
            return None
        torch.cuda.synchronize()

        def med(v):
            v = sorted(v)
            return v[len(v) // 2]

        nb = len(steps[0]["buckets"])
        steps = [r for r in steps if len(r["buckets"]) == nb]
        comm_ms = [med([r["buckets"][k][3].elapsed_time(r["buckets"][k][4]) for r in steps]) for k in range(nb)]
        wait_ms = [med([r["buckets"][k][2].elapsed_time(r["buckets"][k][3]) for r in steps]) for k in range(nb)]
        exposed = [max(0.0, max(r["bwd_end"].elapsed_time(b[4]) for b in r["buckets"])) for r in steps]
        return {"steps": len(steps), "bucket_order": [b[0] for b in steps[0]["buckets"]],
                "bucket_mb": [round(b[1] / (1 << 20), 2) for b in steps[0]["buckets"]],
                "comm_per_bucket_ms": [round(v, 3) for v in comm_ms],
                "wait_per_bucket_ms": [round(v, 3) for v in wait_ms],
                "comm_total_ms": round(sum(comm_ms), 3),
                "exposed_comm_ms": round(med(exposed), 3)}

    def _reduce(self, comm, g, post=None):
        """Reduce ``g`` in place; ``post()`` is then issued on the stream the reduction ends
        on (the comm stream, or the cross-host stage's stream)."""
        if self.hierarchical:
            if self._reduce_hierarchical(comm, g, post):
                return
        else:
            self._reduce_flat(comm, g)
        if post is not None:
            with comm.on_stream():
                post()

    def _reduce_flat(self, comm, g):
        if not self.graph:
            # one rank: the average IS the sum, and RCCL's in-place one-rank sum is free while
            # its one-rank average is a scaled copy of the bucket (oneRankReduce<PreMulSum>:
            # 1.4 ms/step of HBM traffic for VGG-16's 528 MB of gradients)
            op = self.op if comm.size > 1 or self.op != "avg" else "sum"
            if self.monitored:
                comm.monitored_all_reduce(g, op=op, tag=self._tag)
            else:
                comm.all_reduce(g, op=op, tag=self._tag)
            return
        comm.graph_all_reduce(g, op="sum", monitored=True)
        if self.op == "avg":
            with comm.on_stream():
                g.mul_(1.0 / comm.size)

    def _reduce_hierarchical(self, comm, g, post=None) -> bool:
        """Local reduce to the host's root on the comm stream; then either (one host) the
        local broadcast right behind it -- all stream-ordered, no host sync -- or (several
        hosts) hand the bucket to the cross-host stage, which runs the host all-reduce among
        the local roots, the local broadcast and ``post`` on its own thread and stream.
        Returns True when ``post`` was handed over (the caller must not issue it)."""
        from .._lib import runtime

        comm.reduce(g, op="sum", root=0, tag=self._tag + " (local reduce)")
        if self._hier is not None:
            self._hier.submit(g, self._tag, post)
            return True
        if self.op == "avg" and comm.rank == 0:
            with comm.on_stream():
                g.mul_(1.0 / runtime.size())
        comm.broadcast(g, root=0, tag=self._tag + " (local broadcast)")
        return False

    def _finish(self):
        from .mixed import SideStream, reset_pending

        reset_pending()  # a tied table's use whose producer never ran in this backward is stale
        for j in self.tracker.flush():
            self._launch(self.buckets[j])
        if self._hier is not None:
            self._hier.drain()
        SideStream.join()  # nothing computed on the side stream outlives backward
        if self._probe_cur is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()  # backward's compute is done (before the wait for the comm stream)
            self._probe_cur["bwd_end"] = ev
            self.probe.append(self._probe_cur)
            self._probe_cur = None
        if not self.skip:
            if self.segmenter is not None:
                self.segmenter.cut(("join",))  # the compute waits for the comm stream between replays
            else:
                self.comm.join()
            if self._steps_bound == 1 and not self._ordered:
                # second step on this communicator: every rank adopts rank 0's
                # arrival order for its collectives from now on (native auto-order).
                # The step count since binding is the same on every rank (old
                # members and workers that just joined), so all of them take
                # part in this broadcast.
                self.tracker.auto_order()
                self._ordered = True
        if not self.tracker.learned():
            self.tracker.learn()
        self._steps_bound += 1
        self.steps += 1
        self._reset_buckets()
        if self.post_finish is not None:
            self.post_finish()

    def _reset_buckets(self):
        for b in self.buckets:
            b.launched = False
            if b.staged:  # never carry staged gradients into another step
                self._land(b)
        self.tracker.reset()
        self._armed = False

    # ------------------------------------------------------------------ API
    def synchronize(self):
        """Called by the optimizer before stepping (no-op when the backward
        callback already ran)."""
        if self._armed:
            self._finish()

    def reduce_all_now(self):
        """Reduce every bucket immediately (for grads computed without hooks)."""
        self._bind()
        self._reset_buckets()
        for j in self.tracker.flush():
            self._launch(self.buckets[j])
        if not self.skip:
            self.comm.join()
        self._reset_buckets()

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
