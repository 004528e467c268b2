"""kungfu-amd: an adaptive data-parallel training engine for AMD MI355X.

Capabilities of KungFu (S-SGD, SMA, pair averaging, AdaSGD, gradient noise
scale / variance monitors, elastic resize, topology strategies, kungfu-run)
re-designed for PyTorch-ROCm: a C++ host runtime (``_kungfu``), RCCL over
xGMI and hand-written CDNA4 HIP kernels (``_hip``).

Quick start::

    import kungfu_amd as kf
    kf.init()
    opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(model.parameters(), lr=0.1))
    kf.broadcast_parameters(model.state_dict())
"""
__version__ = "0.1.0"

from .python import (cluster_version, current_cluster_size, current_host_count, current_local_rank,
                     current_local_size, current_rank, detached, finalize, get_hip_index, init, launch_mode,
                     propose_new_size, resize_cluster, resize_cluster_from_url, run_barrier, show_hip_version,
                     show_rccl_version, uid)
from . import checkpoint, knobs, ops, optimizers  # noqa: E402
from .ops import broadcast_parameters  # noqa: E402

get_cuda_index = get_hip_index

knobs.check_environ_once()  # warn about misspelt / ignored KUNGFU_* settings
