"""Device data plane: one RCCL communicator per cluster version.

Parity: the reference's NCCL subsystem (``srcs/cpp/src/nccl/gpu_collective.cpp``,
``controller.cpp``, ``helper.cpp``): a global communicator bootstrapped by
broadcasting ``ncclUniqueId`` over the KungFu host transport, re-created after
an elastic resize (``ResetNcclHelper``, ``ops/gpu/scheduler.cpp:54-68``), and a
local (per-host) communicator for the hierarchical path.

MI355X design: collectives run on a dedicated high-priority HIP stream and are
ordered against compute with events -- no ``hipStreamSynchronize`` on the hot
path (the reference synchronises after every NCCL op).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

from .._lib import dtype_code, hip, op_code, runtime

_U8 = 0
_lock = threading.Lock()
_global: Optional["DeviceComm"] = None
_local: Optional["DeviceComm"] = None


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


class DeviceComm:
    """RCCL communicator + comm stream for the current cluster version."""

    def __init__(self, scope: str = "global"):
        H = hip()
        self.scope = scope
        self.version = runtime.cluster_version()
        if scope == "global":
            self.rank, self.size = runtime.rank(), runtime.size()
            leader = self.rank == 0
        else:
            self.rank, self.size = runtime.local_rank(), runtime.local_size()
            leader = self.rank == 0
        self.device = torch.cuda.current_device()
        uid = H.rccl_unique_id() if leader else bytes(128)
        name = "kungfu::rccl_uid::%s::v%d" % (scope, self.version)
        uid = _bcast_bytes(uid, name) if scope == "global" else _local_bcast_bytes(uid, name)
        self.comm = H.RcclComm(uid, self.rank, self.size, self.device)
        # Normal priority: a high-priority HIP stream measured 2x SLOWER for the
        # whole ResNet-50 step on MI355X (63 vs 32 ms, 1 GPU, profiles/README.md).
        prio = int(os.environ.get("KUNGFU_COMM_STREAM_PRIORITY", "0"))
        self.stream = torch.cuda.Stream(device=self.device, priority=prio)

    # -- collectives on an explicit stream (default: the comm stream) ---------
    def _s(self, stream) -> int:
        s = stream if stream is not None else self.stream
        return s.cuda_stream if hasattr(s, "cuda_stream") else int(s)

    def all_reduce(self, inp: torch.Tensor, out: Optional[torch.Tensor] = None, op="sum", stream=None):
        out = inp if out is None else out
        self.comm.all_reduce(inp, out, op_code(op), self._s(stream))
        return out

    def broadcast(self, t: torch.Tensor, root: int = 0, stream=None):
        self.comm.broadcast(t, root, self._s(stream))
        return t

    def reduce(self, inp, out=None, op="sum", root=0, stream=None):
        out = inp if out is None else out
        self.comm.reduce(inp, out, op_code(op), root, self._s(stream))
        return out

    def all_gather(self, inp, out, stream=None):
        self.comm.all_gather(inp, out, self._s(stream))
        return out

    def reduce_scatter(self, inp, out, op="sum", stream=None):
        self.comm.reduce_scatter(inp, out, op_code(op), self._s(stream))
        return out

    def send(self, t, peer, stream=None):
        self.comm.send(t, peer, self._s(stream))

    def recv(self, t, peer, stream=None):
        self.comm.recv(t, peer, self._s(stream))

    def group_start(self):
        hip().rccl_group_start()

    def group_end(self):
        hip().rccl_group_end()

    def graph_all_reduce(self, t: torch.Tensor, op="sum", pairs=None, stream=None):
        """In-place all-reduce along KungFu strategy graphs (default: the session's current
        global strategy, which ``set_tree`` / ``set_strategy`` / adaptation swap) as grouped
        RCCL send/recv rounds + the K1 reduce kernel (see ``plan_graph_all_reduce``)."""
        if self.size == 1:
            return t
        if pairs is None:
            pairs = runtime.global_strategy_pairs()
        key = (tuple((tuple(a), tuple(b)) for a, b in pairs), t.numel())
        cache = self.__dict__.setdefault("_graph_plans", {})
        plan = cache.get(key)
        if plan is None:
            if len(cache) > 64:
                cache.clear()
            plan = runtime.plan_graph_all_reduce([(list(a), list(b)) for a, b in key[0]], self.rank, t.numel())
            cache[key] = plan
        rounds, nscratch = plan
        scratch = torch.empty(max(int(nscratch), 1), dtype=t.dtype, device=t.device)
        s = stream if stream is not None else self.stream
        if hasattr(s, "cuda_stream") and s != torch.cuda.current_stream(t.device):
            scratch.record_stream(s)
        self.comm.graph_run(t, scratch, rounds, op_code(op), self._s(stream))
        return t

    def destroy(self):
        if self.comm is not None:
            try:
                torch.cuda.synchronize(self.device)
            except Exception:
                pass
            self.comm.destroy()
            self.comm = None


class HostStagedComm:
    """The DeviceComm interface over the host runtime (TCP/UDS graph collectives),
    staging through pinned host memory.  Selected with ``KUNGFU_GPU_DATAPLANE=host``:
    for ranks that share one GPU (RCCL refuses duplicate devices) and hosts
    without a usable RCCL.  Every call synchronises its stream -- a functional
    fallback, not a fast path.  Op names are sequence numbers, which match
    across ranks because every rank issues the same collective sequence (the
    ordered scheduler guarantees it for the bucket engine)."""

    def __init__(self, scope: str = "global"):
        self.scope = scope
        self.version = runtime.cluster_version()
        if scope == "global":
            self.rank, self.size = runtime.rank(), runtime.size()
        else:
            self.rank, self.size = runtime.local_rank(), runtime.local_size()
        self.device = torch.cuda.current_device()
        self.stream = torch.cuda.Stream(device=self.device)
        self.comm = self  # "valid" marker for get_device_comm
        self._seq = 0

    def _name(self, kind):
        self._seq += 1
        return "kf:staged:%s:%s:v%d:%d" % (self.scope, kind, self.version, self._seq)

    def _run(self, inp, out, stream, fn):
        s = stream if stream is not None else self.stream
        if not isinstance(s, torch.cuda.Stream):
            s = torch.cuda.ExternalStream(int(s), device=self.device)
        with torch.cuda.stream(s):
            h = inp.detach().to("cpu").contiguous()  # synchronises s
            fn(h)
            (inp if out is None else out).copy_(h.view_as(inp))
            s.synchronize()
        return inp if out is None else out

    def all_reduce(self, inp, out=None, op="sum", stream=None):
        nm = self._name("ar")
        red = op if op != "avg" else "sum"

        def f(h):
            args = (h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h))
            if self.scope == "global":
                runtime.all_reduce(*args, op_code(red), nm)
            else:  # per-host: reduce to the local root, then broadcast back
                runtime.local_reduce(*args, op_code(red), nm + ":r")
                runtime.local_broadcast(*args, nm + ":b")
            if op == "avg":
                h.div_(self.size)

        return self._run(inp, out, stream, f)

    def graph_all_reduce(self, t, op="sum", pairs=None, stream=None):
        # the host runtime executes the session's strategy graphs itself
        return self.all_reduce(t, t, op=op, stream=stream)

    def broadcast(self, t, root: int = 0, stream=None):
        if root != 0:
            raise NotImplementedError("host-staged broadcast supports root 0")
        nm = self._name("bc")
        fn = runtime.broadcast if self.scope == "global" else runtime.local_broadcast
        return self._run(t, None, stream, lambda h: fn(h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h), nm))

    def reduce(self, inp, out=None, op="sum", root=0, stream=None):
        return self.all_reduce(inp, out, op, stream)

    def all_gather(self, inp, out, stream=None):
        nm = self._name("ag")
        s = stream if stream is not None else self.stream
        with torch.cuda.stream(s if isinstance(s, torch.cuda.Stream) else torch.cuda.ExternalStream(int(s))):
            h = inp.detach().to("cpu").contiguous()
            ho = torch.empty((self.size,) + tuple(h.shape), dtype=h.dtype)
            runtime.all_gather(h.data_ptr(), ho.data_ptr(), h.numel(), dtype_code(h), nm)
            out.copy_(ho.view_as(out))
        return out

    def reduce_scatter(self, inp, out, op="sum", stream=None):
        full = inp.detach().clone()
        self.all_reduce(full, op=op, stream=stream)
        n = out.numel()
        out.copy_(full.view(-1)[self.rank * n:(self.rank + 1) * n].view_as(out))
        return out

    def group_start(self):
        pass

    def group_end(self):
        pass

    def destroy(self):
        self.comm = None


def _use_host_staging() -> bool:
    return os.environ.get("KUNGFU_GPU_DATAPLANE", "rccl") == "host"


def get_device_comm(scope: str = "global"):
    """Current communicator; rebuilt when the cluster version changed (resize)."""
    global _global, _local
    from ..python import _ensure

    _ensure()
    with _lock:
        ver = runtime.cluster_version()
        cur = _global if scope == "global" else _local
        if cur is None or cur.version != ver or cur.comm is None:
            if cur is not None:
                cur.destroy()
            cur = HostStagedComm(scope) if _use_host_staging() else DeviceComm(scope)
            if scope == "global":
                _global = cur
            else:
                _local = cur
        return cur


def destroy_device_comm():
    global _global, _local
    with _lock:
        for c in (_global, _local):
            if c is not None:
                try:
                    c.destroy()
                except Exception:
                    pass
        _global = _local = None


def reset_device_comm():
    """Parity: ``KungfuResetNcclHelper`` -- drop communicators after a resize."""
    destroy_device_comm()
