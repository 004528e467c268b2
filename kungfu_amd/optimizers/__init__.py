"""Distributed optimizer wrappers.

Parity: ``srcs/python/kungfu/tensorflow/optimizers/__init__.py:1-12`` and
``srcs/python/kungfu/torch/optimizers``.
"""
from .core import KungFuOptimizer
from .fused import FusedAdam, FusedSGD
from .sync_sgd import SynchronousSGDOptimizer
