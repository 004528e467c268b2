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

    def destroy(self):
        if self.comm is not None:
            try:
                torch.cuda.synchronize(self.device)
            except Exception:
                pass
            self.comm.destroy()
            self.comm = None


def get_device_comm(scope: str = "global") -> DeviceComm:
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
            cur = DeviceComm(scope)
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
