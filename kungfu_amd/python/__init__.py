"""Process-level API: init / rank / size / barrier / elastic control.

Parity: ``srcs/python/kungfu/python/__init__.py:15-107`` (uid, detached,
current_rank, current_local_rank, current_cluster_size, current_local_size,
run_barrier, propose_new_size, check_interference, calc_stats, log_stats,
print_strategy_stats, _get_cuda_index, show_cuda_version, show_nccl_version).

Peer discovery, in priority order:
1. ``KUNGFU_SELF_SPEC`` set (launched by ``kungfu-run``): the env contract.
2. ``torch.distributed.run`` env (``WORLD_SIZE`` > 1, ``MASTER_ADDR``): every
   rank binds a free port and publishes ``ip:port`` in torchrun's TCPStore;
   the peer list is ordered by rank.
3. Otherwise single mode (np = 1, no server).

Unlike the reference, importing the package does not start a peer; the first
API call (or an explicit :func:`init`) does.
"""
from __future__ import annotations

import atexit
import os
import socket
import threading

from .._lib import runtime

_lock = threading.Lock()
_mode = None


def _free_port(ip: str) -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind(("0.0.0.0", 0))
        return s.getsockname()[1]
    finally:
        s.close()


def _torchrun_env() -> bool:
    return int(os.environ.get("WORLD_SIZE", "1")) > 1 and "MASTER_ADDR" in os.environ and "RANK" in os.environ


def _self_ip() -> str:
    ip = os.environ.get("KUNGFU_SELF_IP")
    if ip:
        return ip
    local = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if local == world:
        return "127.0.0.1"
    return socket.gethostbyname(socket.gethostname())


def _init_from_torchrun(strategy: str = ""):
    import datetime

    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    host = os.environ["MASTER_ADDR"]
    port = int(os.environ["MASTER_PORT"])
    store = dist.TCPStore(host, port, world_size=None, is_master=False, timeout=datetime.timedelta(seconds=300),
                          wait_for_workers=False)
    prefix = "kungfu_amd/%s/" % os.environ.get("TORCHELASTIC_RUN_ID", "run")
    ip = _self_ip()
    me = "%s:%d" % (ip, _free_port(ip))
    store.set(prefix + "peer/%d" % rank, me)
    peers = [store.get(prefix + "peer/%d" % r).decode() for r in range(world)]
    strategy = strategy or os.environ.get("KUNGFU_ALLREDUCE_STRATEGY", "")
    runtime.init_explicit(self=me, peers=",".join(peers), strategy=strategy, version=0)


def init(strategy: str = "") -> None:
    """Start this process's peer (idempotent)."""
    global _mode
    with _lock:
        if runtime.initialized():
            return
        if "KUNGFU_SELF_SPEC" in os.environ:
            runtime.init()
            _mode = "kungfu-run"
        elif _torchrun_env():
            _init_from_torchrun(strategy)
            _mode = "torchrun"
        else:
            runtime.init()
            _mode = "single"
        atexit.register(finalize)


def finalize() -> None:
    from ..parallel import comm as _comm
    from ..parallel import graphs as _graphs

    _graphs.release_all()  # graphs holding RCCL work go before their communicators
    _comm.destroy_device_comm()
    if runtime.initialized():
        runtime.finalize()


def _ensure():
    if not runtime.initialized():
        init()


def launch_mode() -> str:
    _ensure()
    return _mode


def uid() -> int:
    _ensure()
    return runtime.uid()


def detached() -> bool:
    _ensure()
    return runtime.detached()


def current_rank() -> int:
    _ensure()
    return runtime.rank()


def current_cluster_size() -> int:
    _ensure()
    return runtime.size()


def current_local_rank() -> int:
    _ensure()
    return runtime.local_rank()


def current_local_size() -> int:
    _ensure()
    return runtime.local_size()


def current_host_count() -> int:
    _ensure()
    return runtime.host_count()


def cluster_version() -> int:
    _ensure()
    return runtime.cluster_version()


def run_barrier() -> None:
    _ensure()
    runtime.barrier()


def propose_new_size(new_size: int) -> bool:
    _ensure()
    return runtime.propose_new_size(int(new_size))


def resize_cluster(new_size: int):
    """Returns (changed, detached).  See ``kungfu_amd.ops.resize``."""
    _ensure()
    return runtime.resize_cluster(int(new_size))


def resize_cluster_from_url():
    _ensure()
    return runtime.resize_cluster_from_url()


def check_interference() -> bool:
    _ensure()
    return runtime.check_interference()


def calc_stats() -> None:
    _ensure()
    from ..parallel.comm import flush_strategy_stats

    flush_strategy_stats()
    runtime.calc_stats()


def log_stats() -> None:
    _ensure()
    runtime.log_stats()


def print_strategy_stats() -> None:
    _ensure()
    for i, t in enumerate(runtime.strategy_throughputs()):
        print("strategy #%d throughput %.3f MiB/s" % (i, t / (1 << 20)))


def get_hip_index() -> int:
    """GPU index for this worker (parity: ``_get_cuda_index``).

    Under ``kungfu-run`` every GPU stays visible by default and the worker's
    slot from the launcher's GPU pool is ``KUNGFU_HIP_DEVICE_ORDINAL`` (so RCCL
    can use P2P/IPC over xGMI); with ``-isolate-gpus`` the worker sees exactly
    its GPU (``HIP_VISIBLE_DEVICES``) and the index is 0.  Under torchrun it is
    ``LOCAL_RANK``.  ``KUNGFU_FORCE_DEVICE`` overrides (tests that co-locate
    several peers on one GPU).
    """
    if "KUNGFU_FORCE_DEVICE" in os.environ:
        return int(os.environ["KUNGFU_FORCE_DEVICE"])
    if "KUNGFU_SELF_SPEC" in os.environ:
        if os.environ.get("KUNGFU_ALLOW_XGMI", "true") == "true":
            slot = os.environ.get("KUNGFU_HIP_DEVICE_ORDINAL")
            return int(slot) if slot not in (None, "") else current_local_rank()
        return 0
    return int(os.environ.get("LOCAL_RANK", "0"))


_get_cuda_index = get_hip_index


def show_hip_version() -> str:
    import torch

    return "HIP %s (torch %s)" % (torch.version.hip, torch.__version__)


def show_rccl_version() -> str:
    from .._lib import hip

    v = hip().rccl_version()
    return "RCCL %d.%d.%d" % (v // 10000, (v // 100) % 100, v % 100)


show_cuda_version = show_hip_version
show_nccl_version = show_rccl_version
