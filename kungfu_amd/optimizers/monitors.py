"""Monitoring optimizers: gradient noise scale and gradient variance.

Parity:
* ``MonitorGradientNoiseScaleOptimizer(opt, device_batch_size, monitor_interval,
  alpha)`` -- ``srcs/python/kungfu/tensorflow/optimizers/grad_noise_scale.py:11-88``:
  S-SGD plus, every ``monitor_interval`` steps, the gradient noise scale
  EMA(S_biased)/EMA(G_biased) from |g_local|^2 (batch b) and |g_avg|^2
  (batch B = b*np) (McCandlish et al., "An Empirical Model of Large-Batch
  Training").  Stored like the reference's ``kungfu_gradient_noise_scale``
  global variable (``kungfu_amd.variables``).
* ``MonitorGradientVarianceOptimizer(opt, monitor_interval)`` --
  ``grad_variance.py:9-75``: all-reduce g^2 as well and report
  sum_tensors || E[g^2] - E[g]^2 ||_2.

GPU design: the gradient all-reduce is the bucketed in-place engine; the
local |g|^2 is accumulated per bucket on the comm stream *before* that
bucket's all-reduce (K5, one pass over the bucket), the global |g_avg|^2 after
the last bucket, and the noise-scale EMA update runs on device (K5 epilogue):
no extra gradient copy and no host sync on the training path.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import ops, variables
from .._lib import hip
from .core import KungFuOptimizer
from .sync_sgd import _SynchronousSGD


class _GradientNoiseScale(_SynchronousSGD):
    def __init__(self, optimizer, device_batch_size: int, named_parameters=None, monitor_interval: int = 1,
                 alpha: float = 0.6, verbose: bool = False, fused: bool = True):
        super().__init__(optimizer, named_parameters, op="avg", fused=fused)
        self.device_batch_size = float(device_batch_size)
        self.np = ops.cluster_size()
        self.global_batch_size = self.device_batch_size * self.np
        self.interval = max(1, int(monitor_interval))
        self.alpha = alpha
        self.verbose = verbose
        self.step_count = 0
        self._ema_g = ops.ExponentialMovingAverage(alpha)
        self._ema_s = ops.ExponentialMovingAverage(alpha)
        self._last = None
        if self.reducer is not None:
            dev = self.space.device
            self._local_sq = torch.zeros(1, dtype=torch.float32, device=dev)
            self._state = torch.zeros(4, dtype=torch.float32, device=dev)  # ema_G, ema_S, gns, count
            self.reducer.pre_reduce = self._pre_reduce
            self.reducer.post_finish = self._post_finish

    def _monitoring(self) -> bool:
        return self.step_count % self.interval == 0 and self.np > 1

    # GPU path -----------------------------------------------------------------
    def _pre_reduce(self, bucket, g):
        if self._monitoring():
            self._local_sq.add_(hip().sumsq2(g)[:1])

    def _post_finish(self):
        if not self._monitoring():
            return
        big = hip().sumsq2(self.space.flat_grad)
        hip().gns_update(self._local_sq, big[:1], self.device_batch_size, self.global_batch_size, self.alpha,
                         self._state)
        self._local_sq.zero_()

    # CPU path ------------------------------------------------------------------
    def sync_gradients(self):
        if self.space is not None or not self._monitoring():
            return super().sync_gradients()
        grads = [p.grad for p in self.params if p.grad is not None]
        local = ops.fuse([g.detach() for g in grads]).clone()
        super().sync_gradients()
        avg = ops.fuse([g.detach() for g in grads])
        sq = ops.sum_squares(local, avg).tolist()
        g_b, s_b = ops.noise_scale_estimates(self.device_batch_size, self.global_batch_size, sq[0], sq[1])
        self._last = self._ema_s(s_b) / self._ema_g(g_b)

    def _after_step(self):
        if self._monitoring():
            variables.set_gradient_noise_scale(self)
            if self.verbose:
                print("Gradient Noise Scale: %s" % self.noise_scale, flush=True)
        self.step_count += 1

    @property
    def noise_scale(self) -> Optional[float]:
        """Latest EMA(S)/EMA(G) (reads the device state: host sync)."""
        if self.reducer is not None:
            return float(self._state[2].item()) if float(self._state[3].item()) > 0 else None
        return self._last


def MonitorGradientNoiseScaleOptimizer(optimizer, device_batch_size: int, named_parameters=None,
                                       monitor_interval: int = 1, alpha: float = 0.6, verbose: bool = False,
                                       fused: bool = True, name=None, use_locking=False):
    return _GradientNoiseScale(optimizer, device_batch_size, named_parameters, monitor_interval=monitor_interval,
                               alpha=alpha, verbose=verbose, fused=fused)


class _GradVariance(_SynchronousSGD):
    def __init__(self, optimizer, named_parameters=None, monitor_interval: int = 1, verbose: bool = True,
                 fused: bool = True):
        super().__init__(optimizer, named_parameters, op="avg", fused=fused)
        self.interval = max(1, int(monitor_interval))
        self.verbose = verbose
        self.step_count = 0
        self.variance: Optional[float] = None
        self.np = ops.cluster_size()
        if self.reducer is not None:
            dev = self.space.device
            self._sq = torch.zeros_like(self.space.flat_grad)
            offs = [o for o, _ in self.space.offsets] + [self.space.numel]
            self._seg = torch.tensor(offs, dtype=torch.int64, device=dev)
            self._var_t = torch.zeros((), dtype=torch.float32, device=dev)
            self.reducer.pre_reduce = self._pre_reduce
            self.reducer.post_finish = self._post_finish

    def _monitoring(self) -> bool:
        return self.step_count % self.interval == 0

    def _pre_reduce(self, bucket, g):
        if self._monitoring():
            sq = self._sq[bucket.start:bucket.end]
            hip().square(sq, g)
            self.reducer.comm.all_reduce(sq, op="avg")

    def _post_finish(self):
        if self._monitoring():
            self._var_t = hip().seg_variance(self.space.flat_grad, self._sq, self._seg, 1.0)

    def sync_gradients(self):
        if self.space is not None or not self._monitoring():
            return super().sync_gradients()
        grads = [p.grad for p in self.params if p.grad is not None]
        sq = [g.detach() * g.detach() for g in grads]
        super().sync_gradients()
        ops.group_all_reduce_(sq, op="avg")
        self.variance = float(sum((s - g * g).norm() for s, g in zip(sq, grads)))

    def _after_step(self):
        if self._monitoring():
            if self.reducer is not None:
                self.variance = float(self._var_t.item())
            if self.verbose:
                print("Variance: %s" % self.variance, flush=True)
        self.step_count += 1


def MonitorGradientVarianceOptimizer(optimizer, named_parameters=None, monitor_interval: int = 1,
                                     verbose: bool = True, fused: bool = True, name=None, use_locking=False):
    return _GradVariance(optimizer, named_parameters, monitor_interval=monitor_interval, verbose=verbose, fused=fused)
