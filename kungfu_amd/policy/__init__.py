"""Training policies (adaptive batch size, elastic scaling decisions, ...).

Parity: ``srcs/python/kungfu/tensorflow/policy/base_policy.py:5-31`` and
``policy_hook.py:8-77``: a policy receives before/after train/epoch/step
callbacks; ``PolicyRunner`` (the PolicyHook equivalent) drives them from a
plain PyTorch loop, maintains the KungFu global variables (TRAINED_SAMPLES,
TOTAL_SAMPLES, BATCH_SIZE) and stops when the sample budget is reached or the
peer was detached by a resize.
"""
from __future__ import annotations

from typing import List, Optional

from .. import variables as kv
from ..python import current_cluster_size, detached


class BasePolicy:
    def before_train(self):
        pass

    def before_epoch(self):
        pass

    def before_step(self):
        pass

    def after_step(self):
        pass

    def after_epoch(self):
        pass

    def after_train(self):
        pass


class PolicyRunner:
    def __init__(self, policies: List[BasePolicy], epoch_size: int, epoch_num: int,
                 init_batch_size: Optional[int] = None):
        self.policies = policies
        self.epoch_size = epoch_size
        self.total_samples = int(epoch_size * epoch_num)
        self.trained_epochs = 0
        self.last_trained_epochs = -1
        self.stopped = False
        kv.set_global_variable(kv.GraphKeys.TRAINED_SAMPLES, 0)
        kv.set_global_variable(kv.GraphKeys.TOTAL_SAMPLES, self.total_samples)
        if init_batch_size is not None:
            kv.set_global_variable(kv.GraphKeys.BATCH_SIZE, init_batch_size)
        for p in self.policies:
            p.before_train()

    def before_step(self):
        if self.trained_epochs > self.last_trained_epochs:
            for p in self.policies:
                p.before_epoch()
            self.last_trained_epochs = self.trained_epochs
        for p in self.policies:
            p.before_step()

    def after_step(self) -> bool:
        """Returns True when training should stop."""
        bs = kv.get_batch_size() or 0
        trained = (kv.get_global_variable(kv.GraphKeys.TRAINED_SAMPLES) or 0) + bs * current_cluster_size()
        kv.set_global_variable(kv.GraphKeys.TRAINED_SAMPLES, trained)
        self.trained_epochs = int(trained / self.epoch_size)
        for p in reversed(self.policies):
            p.after_step()
        if self.trained_epochs > self.last_trained_epochs:
            for p in reversed(self.policies):
                p.after_epoch()
        if trained >= self.total_samples or detached():
            self.stopped = True
        return self.stopped

    def end(self):
        for p in reversed(self.policies):
            p.after_train()


PolicyHook = PolicyRunner
