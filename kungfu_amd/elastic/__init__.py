"""Elastic training: resize the cluster while training, then re-synchronise.

Parity:
* ``srcs/python/kungfu/tensorflow/experimental/hook/elastic.py:11-116``
  (``ElasticHook(local_batch_size, epochs, epoch_size)`` + ``ResizeProfiler``):
  after every step ask the config server for the cluster (resize_cluster_from_url);
  on change, sync the trained-samples offset (all-reduce max) and broadcast the
  model; a detached peer stops.
* ``srcs/python/kungfu/tensorflow/hooks/elastic.py:14-87``
  (``KungFuElasticTrainHook(schedule, max_step)``): resize following a
  "size:steps,..." schedule.
* ``tests/python/integration/test_tensorflow_resize.py``: sync step with
  all-reduce max after a change.

Device communicators are rebuilt lazily for the new cluster version (see
``kungfu_amd.parallel.comm``); collective names are versioned, so newly
spawned workers match the survivors.
"""
from __future__ import annotations

import time
from typing import Optional

import torch

from .. import ops
from .._lib import runtime
from .._utils import show_duration
from ..initializer import broadcast_model
from ..python import _ensure, current_cluster_size, detached


class ResizeProfiler:
    def __init__(self):
        self._begin = None
        self._old = None
        self.records = []

    def begin(self):
        self._begin = time.time()
        self._old = current_cluster_size()

    def end(self):
        if self._begin is None:
            return
        dur = time.time() - self._begin
        new = current_cluster_size() if not detached() else 0
        print("resize %d -> %d took %s" % (self._old, new, show_duration(dur)), flush=True)
        self.records.append((dur, self._old, new))
        self._begin = None

    def cancel(self):
        self._begin = None

    def report(self):
        for i, (d, a, b) in enumerate(self.records):
            print("resize #%d %d -> %d took %s" % (i, a, b, show_duration(d)))


def sync_offset(value: int) -> int:
    """All-reduce max of an integer counter (step / trained samples)."""
    t = torch.tensor([int(value)], dtype=torch.int64)
    return int(ops.all_reduce(t, op="max", name="kf:elastic:offset:v%d" % runtime.cluster_version())[0])


class ElasticTrainer:
    """Loop helper: ``before_step`` syncs state after membership changes,
    ``after_step`` resizes (from the config server or a schedule) and says
    whether this peer must stop."""

    def __init__(self, model: torch.nn.Module, optimizer=None, local_batch_size: int = 1,
                 total_samples: Optional[int] = None, schedule: Optional[str] = None):
        _ensure()
        self.model, self.optimizer = model, optimizer
        self.local_batch_size = local_batch_size
        self.total_samples = total_samples
        self.schedule = ops.StepBasedSchedule(schedule) if schedule else None
        self.step = 0
        self.trained_samples = 0
        self.need_sync = True
        self.exit_reason = None
        self.profiler = ResizeProfiler()

    def before_step(self):
        if self.need_sync:
            self.step = sync_offset(self.step)
            self.trained_samples = sync_offset(self.trained_samples)
            broadcast_model(self.model, self.optimizer)
            self.need_sync = False
            self.profiler.end()

    def after_step(self) -> bool:
        """Returns True when training should stop on this peer."""
        self.step += 1
        self.trained_samples += self.local_batch_size * current_cluster_size()
        self.profiler.begin()
        if self.schedule is not None:
            want = self.schedule(self.step)
            if want != current_cluster_size():
                changed, det = ops.resize_cluster(want)
            else:
                changed, det = False, False
        else:
            changed, det = ops.resize_cluster_from_url()
        if det:
            self.exit_reason = "change cluster"
            self.profiler.end()
            return True
        if changed:
            self.need_sync = True
        else:
            self.profiler.cancel()
        if self.total_samples is not None and self.trained_samples >= self.total_samples:
            self.exit_reason = "finished"
            return True
        return False


class ElasticHook(ElasticTrainer):
    """Parity name: ElasticHook(local_batch_size, epochs, epoch_size)."""

    def __init__(self, model, optimizer, local_batch_size: int, epochs: int, epoch_size: int):
        super().__init__(model, optimizer, local_batch_size=local_batch_size, total_samples=epochs * epoch_size)


class KungFuElasticTrainHook(ElasticTrainer):
    """Parity name: resize following a "size:steps,..." schedule up to max_step."""

    def __init__(self, model, optimizer, schedule: str, max_step: int, local_batch_size: int = 1):
        super().__init__(model, optimizer, local_batch_size=local_batch_size, schedule=schedule)
        self.max_step = max_step

    def after_step(self) -> bool:
        if super().after_step():
            return True
        if self.step >= self.max_step:
            self.exit_reason = "finished"
            return True
        return False
