"""Distributed optimizer wrappers.

Parity: ``srcs/python/kungfu/tensorflow/optimizers/__init__.py:1-12``
(SynchronousSGDOptimizer, SynchronousAveragingOptimizer, PairAveragingOptimizer,
AdaptiveSGDOptimizer, MonitorGradientNoiseScaleOptimizer,
MonitorGradientVarianceOptimizer) and ``srcs/python/kungfu/torch/optimizers``.
"""
from .ada_sgd import AdaptiveSGDOptimizer
from .core import KungFuOptimizer
from .fused import FusedAdam, FusedSGD
from .monitors import MonitorGradientNoiseScaleOptimizer, MonitorGradientVarianceOptimizer
from .pair_avg import PairAveragingOptimizer
from .sma import SynchronousAveragingOptimizer
from .sync_sgd import SynchronousSGDOptimizer

# Aliases matching the reference's wrapper class names.
KungFuTorchOptimizer = KungFuOptimizer
