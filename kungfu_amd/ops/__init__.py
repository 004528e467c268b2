"""kungfu_amd.ops -- the operator surface of the reference's ``kungfu.tensorflow.ops``
(``srcs/python/kungfu/tensorflow/ops/__init__.py:1-83``) and ``kungfu.torch.ops``,
re-implemented for PyTorch-ROCm tensors.
"""
from .adapt import (StepBasedSchedule, calc_stats, check_interference, get_init_checkpoint, log_stats,
                    print_strategy_stats, resize, resize_cluster, resize_cluster_from_url, set_strategy, set_tree,
                    step_based_schedule)
from .collective import (Handle, all_gather, all_reduce, all_reduce_fn, all_reduce_with, barrier, broadcast,
                         broadcast_parameters, cluster_size, consensus, cross_all_reduce_, gather, group_all_reduce,
                         group_all_reduce_, group_hierarchical_nccl_all_reduce, group_nccl_all_reduce,
                         hierarchical_all_reduce_, inplace_all_reduce_async_op, inplace_all_reduce_op,
                         inplace_broadcast_, inplace_broadcast_async_op, local_broadcast_, local_reduce_,
                         monitored_all_reduce, monitored_all_reduce_, rank, reduce, wait_all_handles, wait_handle)
from .fuse import defuse, fuse, split_like
from .local import save_variable, save_variables
from .model_avg import (ModelAveraging, async_model_averaging, model_averaging, request_model,
                        save_model)
from .monitor import (GlobalNoiseScale, egress_rates, global_gradient_noise_scale, global_noise_scale,
                      gradient_variance, noise_scale_estimates, sum_squares)
from .p2p import request_variable, request_variable_with_template
from .state import Counter, ExponentialMovingAverage, counter, exponential_moving_average
from .topology import (RoundRobin, get_neighbour_mask, get_peer_latencies, global_minimum_spanning_tree, minimum_spanning_tree, mst_father,
                       peer_info, round_robin)

__all__ = [n for n in dir() if not n.startswith("_")]
