"""Collective operators on torch tensors.

Parity: TF ops in ``srcs/python/kungfu/tensorflow/ops/collective.py:8-133``
(barrier, consensus, broadcast, all_reduce(op), monitored_all_reduce(tree),
all_gather, group_all_reduce, group_nccl_all_reduce,
group_hierarchical_nccl_all_reduce) and the torch ops in
``srcs/python/kungfu/torch/ops/collective.py:8-52`` (all_reduce_fn,
inplace_all_reduce_op, inplace_all_reduce_async_op, wait_handle,
wait_all_handles, broadcast_parameters, all_gather).

Dispatch by device:
* CPU tensors -> the C++ host runtime (graph collectives over TCP/UDS), any dtype.
* GPU tensors -> RCCL on the current HIP stream (stream-ordered, no host sync);
  ``KUNGFU_GPU_DATAPLANE=host`` stages through host memory instead (the
  reference torch behaviour: D2H -> TCP all-reduce -> H2D).

Names: host collectives are matched across peers by name; when the caller
gives none, a per-process counter ("kf:<op>:<n>") is used, which matches as
long as every peer issues the same sequence of ops (the reference uses TF
node names the same way).
"""
from __future__ import annotations

import itertools
import os
import threading
from typing import Dict, List, Optional, Sequence

import torch

from .._lib import dtype_code, op_code, runtime
from ..python import _ensure

_counters: Dict[str, itertools.count] = {}
_clock = threading.Lock()


_counter_version = [None]


def _auto_name(kind: str) -> str:
    """Per-cluster-version op counter: after an elastic resize every member of
    the new cluster (old and newly spawned workers) counts from 0 again, so
    auto-named collectives keep matching across peers."""
    ver = runtime.cluster_version()
    with _clock:
        if _counter_version[0] != ver:
            _counters.clear()
            _counter_version[0] = ver
        c = _counters.setdefault(kind, itertools.count())
        return "kf:%s:v%d:%d" % (kind, ver, next(c))


def _gpu_host_staging() -> bool:
    return os.environ.get("KUNGFU_GPU_DATAPLANE", "rccl") == "host"


def _dev_comm():
    from ..parallel.comm import get_device_comm

    return get_device_comm()


def _cs():
    return torch.cuda.current_stream()


def rank() -> int:
    _ensure()
    return runtime.rank()


def cluster_size() -> int:
    _ensure()
    return runtime.size()


def barrier() -> None:
    _ensure()
    runtime.barrier()


def consensus(x, name: Optional[str] = None) -> bool:
    """True iff every peer passed byte-identical data (tensor, bytes or str)."""
    _ensure()
    if isinstance(x, torch.Tensor):
        data = x.detach().cpu().contiguous().numpy().tobytes()
    elif isinstance(x, str):
        data = x.encode()
    else:
        data = bytes(x)
    return runtime.consensus(data, name or _auto_name("consensus"))


# --------------------------------------------------------------------- host path

def _host_call(fn, t: torch.Tensor, out: torch.Tensor, *args):
    fn(t.data_ptr(), out.data_ptr(), t.numel(), dtype_code(t), *args)


def _host_all_reduce_(t: torch.Tensor, op: str, name: str) -> torch.Tensor:
    c = t if t.is_contiguous() else t.contiguous()
    runtime.all_reduce(c.data_ptr(), c.data_ptr(), c.numel(), dtype_code(c), op_code(op if op != "avg" else "sum"),
                       name)
    if op == "avg":
        if c.is_floating_point():
            c.div_(runtime.size())
        else:
            c.floor_divide_(runtime.size())
    if c is not t:
        t.copy_(c)
    return t


def _staged(t: torch.Tensor, fn):
    """Run a host collective on a GPU tensor through pinned host memory."""
    h = t.detach().to("cpu", non_blocking=False).contiguous()
    fn(h)
    t.copy_(h, non_blocking=False)
    return t


# --------------------------------------------------------------------- all-reduce

def inplace_all_reduce_op(x: torch.Tensor, op: str = "sum", name: Optional[str] = None) -> torch.Tensor:
    _ensure()
    op = op or "sum"
    if x.is_cuda:
        if _gpu_host_staging():
            nm = name or _auto_name("allreduce")
            return _staged(x, lambda h: _host_all_reduce_(h, op, nm))
        c = x if x.is_contiguous() else x.contiguous()
        _dev_comm().all_reduce(c, op=op, stream=_cs())
        if c is not x:
            x.copy_(c)
        return x
    return _host_all_reduce_(x, op, name or _auto_name("allreduce"))


def all_reduce(x: torch.Tensor, op: str = "sum", name: Optional[str] = None) -> torch.Tensor:
    y = x.detach().clone(memory_format=torch.contiguous_format)
    return inplace_all_reduce_op(y, op=op, name=name)


all_reduce_fn = all_reduce


class Handle:
    """Completion handle of an async op (host: runtime handle; GPU: event)."""

    def __init__(self, host_handle=None, event=None, post=None, keep=None):
        self.host_handle, self.event, self.post = host_handle, event, post
        self.keep = keep  # the tensor the op writes into stays alive until wait()

    def wait(self):
        if self.host_handle is not None:
            runtime.wait(self.host_handle)
            self.host_handle = None
        if self.event is not None:
            _cs().wait_event(self.event)
            self.event = None
        if self.post is not None:
            self.post()
            self.post = None
        self.keep = None

    def __del__(self):
        # never free a buffer a runtime thread may still be writing into
        if self.host_handle is not None:
            try:
                runtime.wait(self.host_handle)
            except Exception:
                pass


def inplace_all_reduce_async_op(x: torch.Tensor, name: Optional[str] = None, op: str = "sum") -> Handle:
    _ensure()
    op = op or "sum"
    if x.is_cuda and not _gpu_host_staging():
        comm = _dev_comm()
        ev = torch.cuda.Event()
        ev.record(_cs())
        comm.stream.wait_event(ev)
        comm.all_reduce(x, op=op)
        x.record_stream(comm.stream)
        done = torch.cuda.Event()
        done.record(comm.stream)
        return Handle(event=done, keep=x)
    if x.is_cuda:
        inplace_all_reduce_op(x, op=op, name=name)
        return Handle()
    if not x.is_contiguous():
        raise ValueError("async all-reduce needs a contiguous CPU tensor")
    nm = name or _auto_name("allreduce")
    h = runtime.all_reduce_async(x.data_ptr(), x.data_ptr(), x.numel(), dtype_code(x),
                                 op_code("sum" if op == "avg" else op), nm)
    post = None
    if op == "avg":
        post = (lambda: x.div_(runtime.size())) if x.is_floating_point() else (lambda: x.floor_divide_(runtime.size()))
    return Handle(host_handle=h, post=post, keep=x)


def wait_handle(h: Handle) -> None:
    h.wait()


def wait_all_handles(hs: Sequence[Handle]) -> None:
    hosts = [h.host_handle for h in hs if h.host_handle is not None]
    if hosts:
        runtime.wait_all(hosts)
        for h in hs:
            h.host_handle = None
    for h in hs:
        h.wait()


def group_all_reduce_(tensors: List[Optional[torch.Tensor]], op: str = "sum",
                      names: Optional[List[str]] = None) -> List[Optional[torch.Tensor]]:
    """All-reduce a list in place; ``None`` entries are skipped (``map_maybe``).

    GPU lists are issued as one RCCL group (one launch batch); CPU lists run
    concurrently on the host runtime.
    """
    _ensure()
    live = [(i, t) for i, t in enumerate(tensors) if t is not None]
    if not live:
        return tensors
    if live[0][1].is_cuda and not _gpu_host_staging():
        comm = _dev_comm()
        comm.group_start()
        try:
            for _, t in live:
                comm.all_reduce(t, op=op, stream=_cs())
        finally:
            comm.group_end()
        return tensors
    hs = []
    for i, t in live:
        nm = names[i] if names else None
        hs.append(inplace_all_reduce_async_op(t, name=nm, op=op))
    wait_all_handles(hs)
    return tensors


def group_all_reduce(tensors, op="sum"):
    return group_all_reduce_([None if t is None else t.detach().clone() for t in tensors], op=op)


# Parity names for the fused / NCCL variants of the reference.
def group_nccl_all_reduce(tensors, op="sum"):
    return group_all_reduce(tensors, op=op)


def monitored_all_reduce_(x: torch.Tensor, tree: Optional[Sequence[int]] = None, name: Optional[str] = None,
                          op: str = "sum") -> torch.Tensor:
    """All-reduce along the strategy graphs (or along ``tree``, a father array), recording
    strategy throughput on the host plane (see ``calc_stats``).  GPU tensors on the RCCL
    plane run the same graphs on the device: grouped send/recv rounds over xGMI + the K1
    reduce kernel (``DeviceComm.graph_all_reduce``)."""
    _ensure()
    if x.is_cuda:
        # device graph plane (RCCL rounds, or the host-staged rounds under
        # KUNGFU_GPU_DATAPLANE=host), timed into the strategy statistics
        c = x if x.is_contiguous() else x.contiguous()
        pairs = [(list(tree), list(tree))] if tree else None
        _dev_comm().graph_all_reduce(c, op=op, pairs=pairs, stream=_cs(), monitored=True)
        if c is not x:
            x.copy_(c)
        return x
    runtime.monitored_all_reduce(x.data_ptr(), x.data_ptr(), x.numel(), dtype_code(x), op_code(op),
                                 name or _auto_name("mallreduce"), list(tree or []))
    return x


def monitored_all_reduce(x, tree=None, op="sum"):
    return monitored_all_reduce_(x.detach().clone(), tree=tree, op=op)


def all_reduce_with(x: torch.Tensor, tree: Sequence[int], op: str = "sum") -> torch.Tensor:
    return monitored_all_reduce(x, tree=tree, op=op)


# --------------------------------------------------------------------- broadcast etc.

def inplace_broadcast_(x: torch.Tensor, name: Optional[str] = None) -> torch.Tensor:
    """Broadcast from rank 0 in place."""
    _ensure()
    from ..parallel.flat import note_param_write

    note_param_write()
    if x.is_cuda and not _gpu_host_staging():
        c = x if x.is_contiguous() else x.contiguous()
        _dev_comm().broadcast(c, root=0, stream=_cs())
        if c is not x:
            x.copy_(c)
        return x
    nm = name or _auto_name("bcast")

    def run(h):
        runtime.broadcast(h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h), nm)

    if x.is_cuda:
        return _staged(x, run)
    c = x if x.is_contiguous() else x.contiguous()
    run(c)
    if c is not x:
        x.copy_(c)
    return x


def broadcast(x: torch.Tensor, name: Optional[str] = None) -> torch.Tensor:
    return inplace_broadcast_(x.detach().clone(memory_format=torch.contiguous_format), name=name)


def inplace_broadcast_async_op(x: torch.Tensor, name: str) -> Handle:
    _ensure()
    if x.is_cuda or not x.is_contiguous():
        inplace_broadcast_(x, name)
        return Handle()
    return Handle(host_handle=runtime.broadcast_async(x.data_ptr(), x.data_ptr(), x.numel(), dtype_code(x), name),
                  keep=x)


def broadcast_parameters(state, name_prefix: str = "kf:bcast_param:") -> None:
    """Broadcast a state_dict / named tensors / module from rank 0, in place.

    GPU tensors are packed into one flat buffer per dtype and broadcast in a
    single RCCL call (K7 pack/unpack); CPU tensors use async host broadcasts.
    """
    _ensure()
    if isinstance(state, torch.nn.Module):
        items = list(state.state_dict().items())
    elif isinstance(state, dict):
        items = list(state.items())
    else:
        items = list(state)
    tensors = [(k, v) for k, v in items if isinstance(v, torch.Tensor)]
    gpu = [(k, v) for k, v in tensors if v.is_cuda]
    cpu = [(k, v) for k, v in tensors if not v.is_cuda]
    if gpu:
        from .fuse import fuse, defuse

        by_dtype: Dict[torch.dtype, list] = {}
        for k, v in gpu:
            by_dtype.setdefault(v.dtype, []).append(v)
        for dt, vs in by_dtype.items():
            flat = fuse(vs)
            inplace_broadcast_(flat)
            defuse(flat, vs)
    hs = [inplace_broadcast_async_op(v, name_prefix + k) for k, v in cpu if v.is_contiguous()]
    for k, v in cpu:
        if not v.is_contiguous():
            inplace_broadcast_(v, name_prefix + k)
    wait_all_handles(hs)


def all_gather(x: torch.Tensor, name: Optional[str] = None) -> torch.Tensor:
    _ensure()
    np_ = runtime.size()
    x = x.contiguous()
    y = x.new_empty((np_,) + tuple(x.shape))
    if x.is_cuda and not _gpu_host_staging():
        _dev_comm().all_gather(x, y, stream=_cs())
        return y
    nm = name or _auto_name("allgather")
    if x.is_cuda:
        h = x.cpu()
        hy = y.cpu()
        runtime.all_gather(h.data_ptr(), hy.data_ptr(), h.numel(), dtype_code(h), nm)
        y.copy_(hy)
        return y
    runtime.all_gather(x.data_ptr(), y.data_ptr(), x.numel(), dtype_code(x), nm)
    return y


def gather(x: torch.Tensor, name: Optional[str] = None) -> Optional[torch.Tensor]:
    """Gather to rank 0: returns [np, ...] on rank 0, the input elsewhere."""
    _ensure()
    np_ = runtime.size()
    h = x.detach().cpu().contiguous()
    y = h.new_empty((np_,) + tuple(h.shape))
    runtime.gather(h.data_ptr(), y.data_ptr(), h.numel(), dtype_code(h), name or _auto_name("gather"))
    if runtime.rank() != 0:
        return x
    return y.to(x.device)


def reduce(x: torch.Tensor, op: str = "sum", name: Optional[str] = None) -> torch.Tensor:
    """Reduce to rank 0 (result meaningful on rank 0 only)."""
    _ensure()
    if x.is_cuda and not _gpu_host_staging():
        y = x.detach().clone()
        _dev_comm().reduce(y, op=op, root=0, stream=_cs())
        return y
    h = x.detach().cpu().contiguous().clone()
    runtime.reduce(h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h), op_code(op), name or _auto_name("reduce"))
    return h.to(x.device)


def cross_all_reduce_(x: torch.Tensor, op: str = "sum", name: Optional[str] = None) -> torch.Tensor:
    """All-reduce among the local masters only (one peer per host)."""
    _ensure()
    nm = name or _auto_name("cross")

    def run(h):
        runtime.cross_all_reduce(h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h), op_code(op), nm)

    if x.is_cuda:
        return _staged(x, run)
    run(x)
    return x


def local_reduce_(x: torch.Tensor, op: str = "sum", name: Optional[str] = None) -> torch.Tensor:
    _ensure()
    nm = name or _auto_name("lreduce")

    def run(h):
        runtime.local_reduce(h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h), op_code(op), nm)

    return _staged(x, run) if x.is_cuda else (run(x) or x)


def local_broadcast_(x: torch.Tensor, name: Optional[str] = None) -> torch.Tensor:
    _ensure()
    nm = name or _auto_name("lbcast")

    def run(h):
        runtime.local_broadcast(h.data_ptr(), h.data_ptr(), h.numel(), dtype_code(h), nm)

    return _staged(x, run) if x.is_cuda else (run(x) or x)


def hierarchical_all_reduce_(x: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """Local reduce -> cross-host all-reduce among local masters -> local
    broadcast (reference: ``KungfuScheduledHierarchicalNcclAllReduce``,
    ``srcs/cpp/src/tensorflow/ops/gpu/collective.cpp:105-156``).

    GPU: local RCCL reduce/broadcast over xGMI (intra-node communicator) and
    the host transport between hosts (staged through host memory on the
    local master only).  CPU: host graph collectives for all three steps.
    """
    _ensure()
    if not x.is_cuda:
        local_reduce_(x, op=op)
        if runtime.local_rank() == 0:
            cross_all_reduce_(x, op=op)
        local_broadcast_(x)
        return x
    from ..parallel.comm import get_device_comm

    lc = get_device_comm("local")
    lc.reduce(x, op=op, root=0, stream=_cs())
    if runtime.host_count() > 1 and runtime.local_rank() == 0:
        cross_all_reduce_(x, op=op)
    lc.broadcast(x, root=0, stream=_cs())
    return x


def group_hierarchical_nccl_all_reduce(tensors, op="sum"):
    return [None if t is None else hierarchical_all_reduce_(t.detach().clone(), op=op) for t in tensors]
