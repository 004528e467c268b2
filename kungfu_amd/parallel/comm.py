"""Device data plane: one RCCL communicator per cluster version.

Parity: the reference's NCCL subsystem (``srcs/cpp/src/nccl/gpu_collective.cpp``,
``controller.cpp``, ``helper.cpp``): a global communicator bootstrapped by
broadcasting ``ncclUniqueId`` over the KungFu host transport, re-created after
an elastic resize (``ResetNcclHelper``, ``ops/gpu/scheduler.cpp:54-68``), and a
local (per-host) communicator for the hierarchical path.

MI355X design: collectives run on a dedicated HIP stream and are ordered
against compute with events -- no ``hipStreamSynchronize`` on the hot path
(the reference synchronises after every NCCL op).

Every communicator class exposes the same stream-ordering surface, which the
training engines (``ddp.GradReducer``, SMA, AdaSGD, the monitors) use instead
of touching HIP streams directly, so the same engine code also runs over the
host transport (CPU tensors, or GPU ranks that share one device):

* ``fence()``      -- the comm stream waits for work issued so far on compute;
* ``on_stream()``  -- context manager: issue kernels on the comm stream;
* ``join()``       -- the compute stream waits for everything on the comm stream.

Communicators are cached per (scope, plane) and keyed by the cluster version:
:func:`get_device_comm` rebuilds one lazily after an elastic resize, and
:func:`comm_epoch` lets long-lived users (bucket reducers, optimizers) notice
that they must re-bind (see ``GradReducer._bind``).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
from typing import Dict, Optional, Tuple

import torch

from .._lib import dtype_code, hip, op_code, runtime

_U8 = 0
_lock = threading.Lock()
_comms: Dict[Tuple[str, str], object] = {}
_epoch = [0]  # bumped by every reset/destroy: users re-bind when it changes


def _bcast_bytes(data: bytes, name: str) -> bytes:
    buf = ctypes.create_string_buffer(data, len(data))
    addr = ctypes.addressof(buf)
    runtime.broadcast(addr, addr, len(data), _U8, name)
    return buf.raw


def _local_bcast_bytes(data: bytes, name: str) -> bytes:
    buf = ctypes.create_string_buffer(data, len(data))
    addr = ctypes.addressof(buf)
    runtime.local_broadcast(addr, addr, len(data), _U8, name)
    return buf.raw


def _scope_rank_size(scope: str):
    """"global", or a per-host scope ("local", "local:<purpose>" -- separate communicators
    over the same host group, e.g. one per issuing thread)."""
    if scope == "global":
        return runtime.rank(), runtime.size()
    return runtime.local_rank(), runtime.local_size()


def _graph_plan(owner, pairs, rank: int, count: int):
    """(rounds, scratch elems) of a graph all-reduce, cached per (pairs, count) on ``owner``."""
    if pairs is None:
        pairs = runtime.global_strategy_pairs()
    key = (tuple((tuple(a), tuple(b)) for a, b in pairs), count)
    cache = owner.__dict__.setdefault("_graph_plans", {})
    plan = cache.get(key)
    if plan is None:
        if len(cache) > 64:
            cache.clear()
        plan = runtime.plan_graph_all_reduce([(list(a), list(b)) for a, b in key[0]], rank, count)
        cache[key] = plan
    return plan


class _DeviceStats:
    """Strategy statistics for device-plane graph all-reduces (parity: the monitored
    all-reduce of ``srcs/go/kungfu/session/monitoring.go:15-35`` feeding
    ``adaptiveStrategies.go:61-121``): each monitored collective is bracketed by two HIP
    events on its stream; completed pairs are converted to (begin, end) seconds on the
    device timeline (relative to one base event) and accounted to the session's current
    global strategy, so ``calc_stats`` / ``check_interference`` / ``set_tree`` adaptation
    works for GPU training.  No host sync on the hot path: events are only queried, and
    drained by :func:`flush_strategy_stats` (called by ``calc_stats``)."""

    def _stat_begin(self, stream):
        if getattr(self, "_stat_base", None) is None:
            # anchor the device timeline to the runtime's steady clock once (one host
            # sync per communicator), so device and host-plane timings share one clock
            # in StrategyStat's (first_begin, last_end) window
            self._stat_base = torch.cuda.Event(enable_timing=True)
            self._stat_base.record(stream)
            self._stat_base.synchronize()
            self._stat_base_host = runtime.now()
            self._stat_pending = []
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        return ev

    def _stat_end(self, start, stream, nbytes: int):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        self._stat_pending.append((start, ev, nbytes))
        self.flush_stats(block=False)

    def flush_stats(self, block: bool = True):
        pend = getattr(self, "_stat_pending", None)
        if not pend:
            return
        keep = []
        for st, en, nb in pend:
            if not block and not en.query():
                keep.append((st, en, nb))
                continue
            en.synchronize()
            b = self._stat_base_host + self._stat_base.elapsed_time(st) / 1e3
            e = self._stat_base_host + self._stat_base.elapsed_time(en) / 1e3
            runtime.record_strategy_stat(b, e, int(nb))
        self._stat_pending = keep


class _StreamOrdered:
    """fence / on_stream / join over ``self.stream`` (a torch.cuda.Stream, or None on CPU)."""

    stream = None
    device = None

    def fence(self):
        if self.stream is not None:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))

    def on_stream(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def join(self):
        if self.stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)


class DeviceComm(_StreamOrdered, _DeviceStats):
    """RCCL communicator + comm stream for the current cluster version."""

    plane = "rccl"

    def __init__(self, scope: str = "global"):
        H = hip()
        self.scope = scope
        self.version = runtime.cluster_version()
        self.rank, self.size = _scope_rank_size(scope)
        leader = self.rank == 0
        self.device = torch.cuda.current_device()
        _colocate_env()
        # collectives captured into a hipGraph (parallel/graphs.py) take the same data path as eager
        # ones: no user-buffer registration at capture (RCCL's NCCL_GRAPH_REGISTER, default on,
        # registers the captured buffers for zero-copy P2P -- an IPC path this pool only supports
        # through dmabuf).  Read once, at the process's first communicator.
        os.environ.setdefault("NCCL_GRAPH_REGISTER", "0")
        H.rccl_watchdog_set_label("rank %d/%d (cluster v%d, %s)" % (runtime.rank(), runtime.size(), self.version,
                                                                    runtime.self_spec()))
        uid = H.rccl_unique_id() if leader else bytes(128)
        name = "kungfu::rccl_uid::%s::v%d" % (scope, self.version)
        uid = _bcast_bytes(uid, name) if scope == "global" else _local_bcast_bytes(uid, name)
        # non-blocking init against a deadline (KUNGFU_RCCL_INIT_TIMEOUT_S): a peer that
        # never arrives raises here instead of hanging; collectives are then watched by
        # the native watchdog (KUNGFU_RCCL_TIMEOUT_S), see rccl_comm.hip
        self.comm = H.RcclComm(uid, self.rank, self.size, self.device, 0.0, *_cta_budget(scope))
        self.ctas = tuple(self.comm.ctas())  # (min, max); 0 = RCCL's default
        # Normal priority: a high-priority HIP stream measured 2x SLOWER for the
        # whole ResNet-50 step on MI355X (63 vs 32 ms, 1 GPU, profiles/README.md).
        self.stream = torch.cuda.Stream(device=self.device)

    # -- collectives on an explicit stream (default: the comm stream) ---------
    def _s(self, stream) -> int:
        s = stream if stream is not None else self.stream
        return s.cuda_stream if hasattr(s, "cuda_stream") else int(s)

    def all_reduce(self, inp: torch.Tensor, out: Optional[torch.Tensor] = None, op="sum", stream=None, tag=""):
        out = inp if out is None else out
        self.comm.all_reduce(inp, out, op_code(op), self._s(stream), tag)
        return out

    def monitored_all_reduce(self, t: torch.Tensor, op="sum", stream=None, tag=""):
        """In-place all-reduce whose bytes and device time feed the strategy statistics
        (parity: ``MonitoredAllReduce``, srcs/go/kungfu/session/monitoring.go:15-35)."""
        s = stream if stream is not None else self.stream
        if not hasattr(s, "cuda_stream"):
            s = torch.cuda.ExternalStream(int(s), device=self.device)
        st = self._stat_begin(s)
        self.comm.all_reduce(t, t, op_code(op), s.cuda_stream, tag)
        self._stat_end(st, s, t.numel() * t.element_size())
        return t

    def broadcast(self, t: torch.Tensor, root: int = 0, stream=None, tag=""):
        self.comm.broadcast(t, root, self._s(stream), tag)
        return t

    def reduce(self, inp, out=None, op="sum", root=0, stream=None, tag=""):
        out = inp if out is None else out
        self.comm.reduce(inp, out, op_code(op), root, self._s(stream), tag)
        return out

    def all_gather(self, inp, out, stream=None, tag=""):
        self.comm.all_gather(inp, out, self._s(stream), tag)
        return out

    def reduce_scatter(self, inp, out, op="sum", stream=None, tag=""):
        self.comm.reduce_scatter(inp, out, op_code(op), self._s(stream), tag)
        return out

    def send(self, t, peer, stream=None):
        self.comm.send(t, peer, self._s(stream))

    def recv(self, t, peer, stream=None):
        self.comm.recv(t, peer, self._s(stream))

    def group_start(self):
        self.comm.group_start()

    def group_end(self):
        self.comm.group_end()

    def watch(self, what: str, stream=None):
        """Register everything issued on ``stream`` so far with the native watchdog."""
        self.comm.watch(self._s(stream), what)

    def graph_all_reduce(self, t: torch.Tensor, op="sum", pairs=None, stream=None, monitored: bool = False):
        """In-place all-reduce along KungFu strategy graphs (default: the session's current
        global strategy, which ``set_tree`` / ``set_strategy`` / adaptation swap) as grouped
        RCCL send/recv rounds + the K1 reduce kernel (see ``plan_graph_all_reduce``).
        ``monitored``: account its bytes and device time to the strategy statistics."""
        if self.size == 1:
            return t
        rounds, nscratch = _graph_plan(self, pairs, self.rank, t.numel())
        scratch = torch.empty(max(int(nscratch), 1), dtype=t.dtype, device=t.device)
        s = stream if stream is not None else self.stream
        if not hasattr(s, "cuda_stream"):
            s = torch.cuda.ExternalStream(int(s), device=self.device)
        if s != torch.cuda.current_stream(t.device):
            scratch.record_stream(s)
        st = self._stat_begin(s) if monitored else None
        self.comm.graph_run(t, scratch, rounds, op_code(op), s.cuda_stream)
        if monitored:
            self._stat_end(st, s, t.numel() * t.element_size())
        return t

    def destroy(self):
        if self.comm is not None:
            try:
                torch.cuda.synchronize(self.device)
            except Exception:
                pass
            self.comm.destroy()
            self.comm = None


class HostComm(_StreamOrdered):
    """The DeviceComm interface over the host runtime (TCP/UDS graph collectives).

    * ``device="cpu"``: CPU tensors, no staging, no streams -- the engines
      (bucketed S-SGD, SMA, AdaSGD, monitors) run unchanged on CPU peers, which
      is how their multi-process / elastic behaviour is tested without GPUs.
    * ``device`` a GPU (``KUNGFU_GPU_DATAPLANE=host``): staged through host
      memory, for ranks that share one GPU (RCCL refuses duplicate devices) and
      hosts without a usable RCCL.  Every call synchronises its stream -- a
      functional fallback, not a fast path.

    Op names are sequence numbers, which match across ranks because every rank
    issues the same collective sequence (the ordered scheduler guarantees it
    for the bucket engine)."""

    plane = "host"

    def __init__(self, scope: str = "global", device=None):
        self.scope = scope
        self.version = runtime.cluster_version()
        self.rank, self.size = _scope_rank_size(scope)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        self.staged = device.type == "cuda"
        self.device = torch.cuda.current_device() if self.staged else device
        self.stream = torch.cuda.Stream(device=self.device) if self.staged else None
        self.comm = self  # "valid" marker for get_device_comm
        self._seq = 0

    def _name(self, kind):
        self._seq += 1
        return "kf:hostcomm:%s:%s:v%d:%d" % (self.scope, kind, self.version, self._seq)

    def _run(self, inp, out, stream, fn, write=True):
        """fn(h) on a contiguous host copy of ``inp``; the result lands in ``out``
        (default ``inp``) when ``write``."""
        dst = inp if out is None else out
        if not self.staged:
            h = inp if inp.is_contiguous() and dst is inp else inp.detach().contiguous().clone()
            fn(h)
            if write and h is not dst:
                dst.copy_(h.view_as(dst))
            return dst
        s = stream if stream is not None else self.stream
        if not isinstance(s, torch.cuda.Stream):
            s = torch.cuda.ExternalStream(int(s), device=self.device)
        with torch.cuda.stream(s):
            h = inp.detach().to("cpu").contiguous()  # synchronises s
            fn(h)
            if write:
                dst.copy_(h.view_as(dst))
            s.synchronize()
        return dst

    def _ar(self, h, op, nm):
        red = op if op != "avg" else "sum"
        args = (h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h))
        if self.scope == "global":
            runtime.all_reduce(*args, op_code(red), nm)
        else:  # per-host: reduce to the local root, then broadcast back
            runtime.local_reduce(*args, op_code(red), nm + ":r")
            runtime.local_broadcast(*args, nm + ":b")
        if op == "avg":
            if h.is_floating_point():
                h.div_(self.size)
            else:
                h.floor_divide_(self.size)

    def all_reduce(self, inp, out=None, op="sum", stream=None, tag=""):
        nm = self._name("ar")
        return self._run(inp, out, stream, lambda h: self._ar(h, op, nm))

    def monitored_all_reduce(self, t, op="sum", stream=None, tag=""):
        """All-reduce along the session's current strategy with strategy statistics: CPU
        tensors use the runtime's native monitored all-reduce; staged GPU tensors are
        timed on the runtime's clock around the (synchronous) staged collective."""
        if not self.staged:
            return self.graph_all_reduce(t, op=op, monitored=True)
        t0 = runtime.now()
        self.all_reduce(t, op=op, stream=stream)
        runtime.record_strategy_stat(t0, runtime.now(), t.numel() * t.element_size())
        return t

    def graph_all_reduce(self, t, op="sum", pairs=None, stream=None, monitored: bool = False):
        """CPU tensors: the host runtime executes the strategy graphs itself (monitored:
        native strategy statistics).  Staged GPU tensors: the device graph plane's round
        plan (``plan_graph_all_reduce``, the same one RCCL executes) with host transfers
        (``send_to`` / ``recv_from``) and the device K1 reduce kernel -- so the plan and
        the kernel are testable with ranks that share one GPU."""
        if not self.staged:
            nm = self._name("gar")
            red = op if op != "avg" else "sum"
            c = t if t.is_contiguous() else t.contiguous()
            if monitored or pairs is not None:
                tree = list(pairs[0][0]) if pairs is not None and len(pairs) == 1 and pairs[0][0] == pairs[0][1] else []
                runtime.monitored_all_reduce(c.data_ptr(), c.data_ptr(), c.numel(), dtype_code(c), op_code(red), nm,
                                             tree)
            else:
                runtime.all_reduce(c.data_ptr(), c.data_ptr(), c.numel(), dtype_code(c), op_code(red), nm)
            if op == "avg":
                c.div_(self.size)
            if c is not t:
                t.copy_(c)
            return t
        if self.size == 1:
            return t
        from .._lib import hip

        rounds, nscratch = _graph_plan(self, pairs, self.rank, t.numel())
        nm = self._name("graph")
        s = stream if stream is not None else self.stream
        if not isinstance(s, torch.cuda.Stream):
            s = torch.cuda.ExternalStream(int(s), device=self.device)
        esz = t.element_size()
        t0 = runtime.now()
        with torch.cuda.stream(s):
            flat = t.view(-1)
            scratch = torch.empty(max(int(nscratch), 1), dtype=t.dtype, device=t.device)
            for ri, rnd in enumerate(rounds):
                s.synchronize()  # the previous round's reduces are complete before sending
                for recv, peer, off, ln, sc in rnd:
                    if not recv and ln:
                        h = flat[off:off + ln].to("cpu")
                        runtime.send_to(peer, "%s:r%d:%d" % (nm, ri, off), h.data_ptr(), ln * esz)
                for recv, peer, off, ln, sc in rnd:
                    if recv and ln:
                        h = torch.empty(ln, dtype=t.dtype)
                        runtime.recv_from(peer, "%s:r%d:%d" % (nm, ri, off), h.data_ptr(), ln * esz)
                        dst = scratch[sc:sc + ln] if sc >= 0 else flat[off:off + ln]
                        dst.copy_(h)
                        if sc >= 0:  # K1: reduce the received chunk into place on the device
                            hip().reduce(flat[off:off + ln], flat[off:off + ln], dst, op_code(op))
            s.synchronize()
        if monitored:
            runtime.record_strategy_stat(t0, runtime.now(), t.numel() * esz)
        return t

    def broadcast(self, t, root: int = 0, stream=None, tag=""):
        nm = self._name("bc")
        if root == 0:
            fn = runtime.broadcast if self.scope == "global" else runtime.local_broadcast
            return self._run(t, None, stream,
                             lambda h: fn(h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h), nm))

        # any other root: a sum in which every non-root contributes zeros (exact: x + 0 == x)
        def f(h):
            if self.rank != root:
                h.zero_()
            self._ar(h, "sum", nm)

        return self._run(t, None, stream, f)

    def reduce(self, inp, out=None, op="sum", root=0, stream=None, tag=""):
        """Result on ``root`` only; the other ranks' ``out`` is left untouched (RCCL semantics)."""
        nm = self._name("rd")
        red = op if op != "avg" else "sum"
        if root == 0:
            fn = runtime.reduce if self.scope == "global" else runtime.local_reduce

            def f(h):
                fn(h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h), op_code(red), nm)
                if op == "avg" and self.rank == 0:
                    h.div_(self.size)
        else:
            def f(h):
                self._ar(h, op, nm)

        if self.rank == root:
            return self._run(inp, out, stream, f)
        # non-roots take part in the collective but keep their buffers
        self._run(inp, inp.detach().clone() if out is None else out.detach().clone(), stream, f, write=False)
        return inp if out is None else out

    def all_gather(self, inp, out, stream=None, tag=""):
        nm = self._name("ag")

        def run():
            h = inp.detach().to("cpu").contiguous()
            ho = torch.empty((self.size,) + tuple(h.shape), dtype=h.dtype)
            runtime.all_gather(h.data_ptr(), ho.data_ptr(), h.numel(), dtype_code(h), nm)
            out.copy_(ho.view_as(out))

        if not self.staged:
            run()
            return out
        s = stream if stream is not None else self.stream
        with torch.cuda.stream(s if isinstance(s, torch.cuda.Stream) else torch.cuda.ExternalStream(int(s))):
            run()
        return out

    def reduce_scatter(self, inp, out, op="sum", stream=None, tag=""):
        full = inp.detach().clone()
        self.all_reduce(full, op=op, stream=stream)
        n = out.numel()
        out.copy_(full.view(-1)[self.rank * n:(self.rank + 1) * n].view_as(out))
        return out

    def group_start(self):
        pass

    def group_end(self):
        pass

    def watch(self, what: str, stream=None):
        pass  # host ops are watched by the runtime's op watchdog (KUNGFU_OP_TIMEOUT_S)

    def destroy(self):
        self.comm = None


# Kept for callers of the round-1 name.
HostStagedComm = HostComm


class EmulatedComm(_StreamOrdered):
    """One-GPU stand-in for the all-reduces of an ``ranks``-rank job (``bench.py --emulate-comm``,
    ``KUNGFU_COMM_EMULATE="ranks=8,ctas=16,busbw=350,lat_us=25"``): every all-reduce of B bytes
    launches ``comm_emu.hip`` on the comm stream -- ``ctas`` workgroups, resident for the
    modelled ring time 2(r-1)/r * B / busbw + lat, copying 2(r-1)/r * B bytes (a read plus a write:
    the ~4(r-1)/r * B bytes of local HBM traffic such an all-reduce makes) -- so its cost to the overlapped backward (CUs, HBM,
    stream ordering) shows up in a 1-GPU step time.  The data is NOT reduced (one rank: the
    gradient already is the average).  A model: no inter-rank skew, no link congestion."""

    plane = "emulate"

    def __init__(self, spec: str):
        kv = dict(p.split("=", 1) for p in spec.split(",") if "=" in p)
        self.ranks = int(kv.get("ranks", 8))
        self.ctas_n = int(kv.get("ctas", 16))
        self.busbw = float(kv.get("busbw", 350.0)) * 1e9  # bytes/s
        self.lat = float(kv.get("lat_us", 25.0)) * 1e-6
        self.scope = "global"
        self.version = runtime.cluster_version()
        self.rank, self.size = 0, 1
        self.device = torch.cuda.current_device()
        self.stream = torch.cuda.Stream(device=self.device)
        self.comm = self
        self.ctas = (self.ctas_n, self.ctas_n)
        self._scratch = None
        self.calls = 0
        self.modelled_s = 0.0

    def model_seconds(self, nbytes: int) -> float:
        r = self.ranks
        return 2.0 * (r - 1) / r * nbytes / self.busbw + self.lat

    def all_reduce(self, inp, out=None, op="sum", stream=None, tag=""):
        out = inp if out is None else out
        if out is not inp:
            out.copy_(inp)
        nb = inp.numel() * inp.element_size()
        nb16 = max(16, (nb + 15) // 16 * 16)
        s = stream if stream is not None else self.stream
        if not isinstance(s, torch.cuda.Stream):
            s = torch.cuda.ExternalStream(int(s), device=inp.device)
        if self._scratch is None or self._scratch.numel() < 2 * nb16:
            # allocated on the stream that uses it: when a larger bucket replaces it, the caching
            # allocator only hands the old block out again in that stream's order, i.e. after the
            # paced kernels still writing it have finished
            with torch.cuda.stream(s):
                self._scratch = torch.empty(2 * nb16, dtype=torch.uint8, device=inp.device)
        src, dst = self._scratch[:nb16], self._scratch[nb16:2 * nb16]
        r = self.ranks
        t = self.model_seconds(nb)
        # bytes COPIED: 2(r-1)/r x B, i.e. a read plus a write of that much = the 4(r-1)/r x B of
        # local HBM traffic a ring all-reduce makes (comm_emu.hip header; r4 passed the traffic
        # itself here and so doubled the modelled contention -- ADVICE r4)
        hip().comm_emulate(src, dst, int(2 * (r - 1) / r * nb), self.ctas_n, t, s.cuda_stream)
        self.calls += 1
        self.modelled_s += t
        return out

    monitored_all_reduce = all_reduce

    def broadcast(self, t, root: int = 0, stream=None, tag=""):
        return t

    def watch(self, what: str, stream=None):
        pass

    def destroy(self):
        self.comm = None

    def describe(self) -> dict:
        return {"ranks": self.ranks, "ctas": self.ctas_n, "busbw_gbs": self.busbw / 1e9, "lat_us": self.lat * 1e6,
                "calls": self.calls, "modelled_comm_ms_total": round(self.modelled_s * 1e3, 3)}


def _cta_budget(scope: str):
    """(min, max) RCCL CTAs for a communicator of ``scope``: KUNGFU_RCCL_{MIN,MAX}_CTAS, with
    per-scope overrides KUNGFU_RCCL_{MIN,MAX}_CTAS_<SCOPE> (``local``, ``local_bcast``); 0 = RCCL
    default.  The hierarchical mode's two local communicators run concurrently from two
    threads: giving each at most half the chip keeps their kernels co-resident."""
    key = scope.upper().replace(":", "_")

    def get(kind):
        v = os.environ.get("KUNGFU_RCCL_%s_CTAS_%s" % (kind, key), os.environ.get("KUNGFU_RCCL_%s_CTAS" % kind, "0"))
        return int(v or 0)

    return get("MIN"), get("MAX")


def _colocate_env() -> None:
    """``KUNGFU_RCCL_COLOCATE=1``: several RCCL ranks on ONE GPU (tests on a one-GPU box).
    RCCL rejects two ranks of one communicator on the same device of the same host
    ("Duplicate GPU detected"); giving every rank its own host identity
    (``NCCL_HOSTID``) makes them distinct "hosts" joined by RCCL's socket transport over
    loopback -- a real multi-rank RCCL communicator (bootstrap, ordering, ncclAvg,
    rebuild after resize, abort) whose bandwidth means nothing.  Must run before the
    process's first RCCL call."""
    if os.environ.get("KUNGFU_RCCL_COLOCATE", "0") != "1":
        return
    os.environ["NCCL_HOSTID"] = "kungfu-colocated-%s" % runtime.self_spec()
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")


def _use_host_staging() -> bool:
    return os.environ.get("KUNGFU_GPU_DATAPLANE", "rccl") == "host"


def _emulate_spec() -> str:
    return os.environ.get("KUNGFU_COMM_EMULATE", "")


def flush_strategy_stats() -> None:
    """Account every completed monitored device collective to the strategy statistics
    (waits for the pending ones).  Called by ``calc_stats``."""
    with _lock:
        comms = list(_comms.values())
    for c in comms:
        f = getattr(c, "flush_stats", None)
        if f is not None:
            f(block=True)


def comm_epoch() -> int:
    """Changes whenever the communicators are reset (elastic resize) -- users
    that cached a communicator compare it with the value they bound at."""
    return _epoch[0]


def get_device_comm(scope: str = "global", device=None):
    """Current communicator for ``scope`` ("global" or "local"); rebuilt when the
    cluster version changed (resize).  ``device`` selects the plane: a CPU
    device gives the host-transport :class:`HostComm`, otherwise RCCL (or the
    host-staged fallback under ``KUNGFU_GPU_DATAPLANE=host``)."""
    from ..python import _ensure

    _ensure()
    cpu = device is not None and torch.device(device).type == "cpu"
    emu = _emulate_spec()
    if emu and runtime.size() != 1:
        raise RuntimeError("KUNGFU_COMM_EMULATE models an N-rank job on ONE rank; this job has %d" % runtime.size())
    kind = "cpu" if cpu else ("emulate" if emu and scope == "global" else "staged" if _use_host_staging() else "rccl")
    with _lock:
        ver = runtime.cluster_version()
        cur = _comms.get((scope, kind))
        if cur is None or cur.version != ver or cur.comm is None:
            if cur is not None:
                cur.destroy()
            if kind == "cpu":
                cur = HostComm(scope, device="cpu")
            elif kind == "staged":
                cur = HostComm(scope)
            elif kind == "emulate":
                cur = EmulatedComm(emu)
            else:
                cur = DeviceComm(scope)
            _comms[(scope, kind)] = cur
        return cur


def destroy_device_comm():
    with _lock:
        for c in _comms.values():
            try:
                c.destroy()
            except Exception:
                pass
        _comms.clear()
        _epoch[0] += 1


def reset_device_comm():
    """Parity: ``KungfuResetNcclHelper`` -- drop communicators after a resize."""
    destroy_device_comm()
