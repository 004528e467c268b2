"""Monitoring operators: gradient noise scale, gradient variance, egress rates.

Parity: ``srcs/python/kungfu/tensorflow/ops/monitor.py:6-27`` (global_noise_scale,
egress_rates) and ``ops/cpu/collective.cpp:212-260`` (NoiseScale: EMA(S)/EMA(G)).

GPU tensors use the K5/K6 HIP reductions (one pass over both gradients, f32
accumulation, deterministic two-stage reduce); CPU tensors use torch.
"""
from __future__ import annotations

from typing import Optional

import torch

from .._lib import hip, runtime
from ..python import _ensure
from .state import ExponentialMovingAverage


def sum_squares(a: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[sum(a^2), sum(b^2)] (f32).  One fused pass on GPU."""
    a = a.contiguous()
    if a.is_cuda and a.dtype in (torch.float32, torch.bfloat16):
        return hip().sumsq2(a.reshape(-1), None if b is None else b.contiguous().reshape(-1))
    sa = a.double().pow(2).sum().float()
    sb = b.double().pow(2).sum().float() if b is not None else torch.zeros((), dtype=torch.float32)
    return torch.stack([sa, sb])


def noise_scale_estimates(batch_small: float, batch_big: float, sq_small: float, sq_big: float):
    """(G_biased, S_biased) from |g_small|^2 and |g_big|^2 (McCandlish et al.)."""
    g = (batch_big * sq_big - batch_small * sq_small) / (batch_big - batch_small)
    s = (sq_small - sq_big) / (1.0 / batch_small - 1.0 / batch_big)
    return g, s


class GlobalNoiseScale:
    """Stateful noise-scale estimator: EMA(S_biased) / EMA(G_biased)."""

    def __init__(self, alpha: float = 0.6):
        self.g_ema = ExponentialMovingAverage(alpha)
        self.s_ema = ExponentialMovingAverage(alpha)

    def __call__(self, batch_small, batch_big, tensor, avg_tensor) -> float:
        sq = sum_squares(tensor, avg_tensor).tolist()
        g, s = noise_scale_estimates(batch_small, batch_big, sq[0], sq[1])
        return self.s_ema(s) / self.g_ema(g)


_gns = {}


def global_noise_scale(batch_small, batch_big, tensor, avg_tensor, alpha: float = 0.6, key: str = "default") -> float:
    est = _gns.setdefault((key, alpha), GlobalNoiseScale(alpha))
    return est(batch_small, batch_big, tensor, avg_tensor)


global_gradient_noise_scale = global_noise_scale


def gradient_variance(sum_g: torch.Tensor, sum_g2: torch.Tensor, n: int) -> float:
    """sum_i | E[g^2]_i - E[g]_i^2 | from the all-reduced sums over n peers (K6)."""
    if sum_g.is_cuda:
        return float(hip().variance(sum_g.contiguous().reshape(-1).float(), sum_g2.contiguous().reshape(-1).float(),
                                    1.0 / n).item())
    m = sum_g.double() / n
    return float((sum_g2.double() / n - m * m).abs().sum())


def egress_rates() -> torch.Tensor:
    """Bytes/s sent to every peer over the last monitoring window
    (requires KUNGFU_CONFIG_ENABLE_MONITORING=true)."""
    _ensure()
    return torch.tensor(runtime.egress_rates(), dtype=torch.float32)
