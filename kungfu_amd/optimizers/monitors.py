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

Engine design: the gradient all-reduce is the bucketed in-place engine; the
local |g|^2 is accumulated per bucket on the comm stream *before* that
bucket's all-reduce (K5, one pass over the bucket), the global |g_avg|^2 after
the last bucket, and the noise-scale EMA update runs on device (K5 epilogue):
no extra gradient copy and no host sync on the training path.

The peer count (B = b * np) is read from the current cluster at every
monitored step, so the estimate stays right across elastic resizes.  With one
peer the estimator is undefined (B == b); ``monitor_single=True`` still runs the
K5 reductions every step (the bucket collectives are forced through the
communicator) so they can be profiled, and the device EMA keeps its state.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import ops, variables
from ..parallel.flat import sumsq
from .sync_sgd import _SynchronousSGD


def _gns_update_host(sq_small: float, sq_big: float, b: float, B: float, alpha: float, state: torch.Tensor):
    """CPU twin of the device ``gns_update`` kernel (csrc/kernels/norms.hip)."""
    if not B > b:
        return
    G = (B * sq_big - b * sq_small) / (B - b)
    S = (sq_small - sq_big) / (1.0 / b - 1.0 / B)
    cnt = float(state[3])
    eg = G if cnt == 0 else alpha * float(state[0]) + (1 - alpha) * G
    es = S if cnt == 0 else alpha * float(state[1]) + (1 - alpha) * S
    state[0], state[1] = eg, es
    state[2] = es / eg if eg != 0 else 0.0
    state[3] = cnt + 1


class _GradientNoiseScale(_SynchronousSGD):
    def __init__(self, optimizer, device_batch_size: int, named_parameters=None, monitor_interval: int = 1,
                 alpha: float = 0.6, verbose: bool = False, fused: bool = True, monitor_single: bool = False,
                 flat=None, comm_dtype: Optional[torch.dtype] = None):
        # comm_dtype: the gradient dtype on the wire (sync_sgd.SynchronousSGDOptimizer); |g_big|^2 is
        # then taken of the bf16-averaged gradient (a ~2^-9 relative perturbation of the estimate)
        super().__init__(optimizer, named_parameters, op="avg", fused=fused, force_comm=monitor_single, flat=flat,
                         comm_dtype=comm_dtype)
        self.device_batch_size = float(device_batch_size)
        self.interval = max(1, int(monitor_interval))
        self.alpha = alpha
        self.verbose = verbose
        self.monitor_single = monitor_single
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

    @property
    def np(self) -> int:
        return ops.cluster_size()

    @property
    def global_batch_size(self) -> float:
        return self.device_batch_size * self.np

    def _monitoring(self) -> bool:
        return self.step_count % self.interval == 0 and (self.np > 1 or self.monitor_single)

    # flat-space path ------------------------------------------------------------
    def _pre_reduce(self, bucket, g):
        if self._monitoring():
            self._local_sq.add_(sumsq(g)[:1])

    def _post_finish(self):
        if not self._monitoring():
            return
        big = sumsq(self.space.flat_grad)
        if self._state.is_cuda:
            from .._lib import hip

            hip().gns_update(self._local_sq, big[:1], self.device_batch_size, self.global_batch_size, self.alpha,
                             self._state)
        else:
            _gns_update_host(float(self._local_sq), float(big[0]), self.device_batch_size, self.global_batch_size,
                             self.alpha, self._state)
        self._local_sq.zero_()

    # per-tensor CPU path ---------------------------------------------------------
    def sync_gradients(self):
        if self.space is not None or not self._monitoring() or self.np == 1:
            return super().sync_gradients()  # B == b with one peer: the estimate is undefined
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

    def _kf_scalars(self):
        return [self.step_count]

    def _kf_load_scalars(self, vals):
        self.step_count = int(vals[0])


def MonitorGradientNoiseScaleOptimizer(optimizer, device_batch_size: int, named_parameters=None,
                                       monitor_interval: int = 1, alpha: float = 0.6, verbose: bool = False,
                                       fused: bool = True, name=None, use_locking=False, monitor_single: bool = False,
                                       flat=None, comm_dtype: Optional[torch.dtype] = None):
    return _GradientNoiseScale(optimizer, device_batch_size, named_parameters, monitor_interval=monitor_interval,
                               alpha=alpha, verbose=verbose, fused=fused, monitor_single=monitor_single, flat=flat,
                               comm_dtype=comm_dtype)


class _GradVariance(_SynchronousSGD):
    def __init__(self, optimizer, named_parameters=None, monitor_interval: int = 1, verbose: bool = True,
                 fused: bool = True, flat=None):
        super().__init__(optimizer, named_parameters, op="avg", fused=fused, flat=flat)
        self.interval = max(1, int(monitor_interval))
        self.verbose = verbose
        self.step_count = 0
        self.variance: Optional[float] = None
        if self.reducer is not None:
            dev = self.space.device
            self._sq = torch.zeros_like(self.space.flat_grad)
            offs = [o for o, _ in self.space.offsets] + [self.space.numel]
            self._seg_host = offs
            self._seg = torch.tensor(offs, dtype=torch.int64, device=dev)
            self._var_t = torch.zeros((), dtype=torch.float32, device=dev)
            self.reducer.pre_reduce = self._pre_reduce
            self.reducer.post_finish = self._post_finish

    @property
    def np(self) -> int:
        return ops.cluster_size()

    def _monitoring(self) -> bool:
        return self.step_count % self.interval == 0

    def _pre_reduce(self, bucket, g):
        if self._monitoring():
            sq = self._sq[bucket.start:bucket.end]
            if sq.is_cuda:
                from .._lib import hip

                hip().square(sq, g)
            else:
                torch.mul(g, g, out=sq)
            self.reducer.comm.all_reduce(sq, op="avg")

    def _post_finish(self):
        if not self._monitoring():
            return
        if self.reducer.skip:  # one peer: E[g^2] = g^2 (the pre-reduce hook did not run)
            if self._sq.is_cuda:
                from .._lib import hip

                hip().square(self._sq, self.space.flat_grad)
            else:
                torch.mul(self.space.flat_grad, self.space.flat_grad, out=self._sq)
        if self._sq.is_cuda:
            from .._lib import hip

            self._var_t = hip().seg_variance(self.space.flat_grad, self._sq, self._seg, 1.0)
        else:
            g, s, o = self.space.flat_grad, self._sq, self._seg_host
            self._var_t = torch.tensor(sum(float((s[a:b] - g[a:b] * g[a:b]).norm()) for a, b in zip(o, o[1:])))

    def sync_gradients(self):
        if self.space is not None or not self._monitoring() or self.np == 1:
            return super().sync_gradients()  # B == b with one peer: the estimate is undefined
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

    def _kf_scalars(self):
        return [self.step_count]

    def _kf_load_scalars(self, vals):
        self.step_count = int(vals[0])


def MonitorGradientVarianceOptimizer(optimizer, named_parameters=None, monitor_interval: int = 1,
                                     verbose: bool = True, fused: bool = True, name=None, use_locking=False,
                                     flat=None):
    return _GradVariance(optimizer, named_parameters, monitor_interval=monitor_interval, verbose=verbose, fused=fused,
                         flat=flat)
