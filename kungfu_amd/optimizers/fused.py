"""Fused optimizers over a :class:`FlatParamSpace` (K8).

One HIP kernel per step for the whole model: read w, g, m; write w, m (and
optionally a bf16 shadow copy of w) -- 5 x 4 B per parameter of HBM traffic,
versus torch's per-tensor (or foreach multi-pass) SGD.  The gradient
averaging factor (1/np) can be folded in via ``grad_scale``.

Parity: the wrapped ``tf.train.Optimizer.apply_gradients``
(``srcs/python/kungfu/tensorflow/optimizers/core.py:13-15``) -- the reference
applies the framework optimizer per tensor; this is the MI355X-native apply.

The learning rate lives in ``param_groups[0]['lr']`` (torch LR schedulers
work) and is also mirrored into a 1-element device tensor so a captured
hipGraph replays with the current LR.
"""
from __future__ import annotations

import torch

from .._lib import hip
from ..parallel.flat import FlatParamSpace


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, space: FlatParamSpace, lr: float = 0.01, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, grad_scale: float = 1.0,
                 bf16_shadow: bool = False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov)
        super().__init__(space.params, defaults)
        self.space = space
        self.grad_scale = grad_scale
        dev = space.device
        self.momentum_buffer = torch.zeros_like(space.flat_param) if momentum else None
        self.shadow = torch.empty(space.numel, dtype=torch.bfloat16, device=dev) if bf16_shadow else None
        self._lr_t = torch.full((1,), lr, dtype=torch.float32, device=dev)
        self._first = True
        self._gpu = dev.type == "cuda"
        if self._gpu:
            hip()  # fail loudly if the kernels are missing on a GPU machine

    def zero_grad(self, set_to_none: bool = False):  # keep the flat grad views
        self.space.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        lr, mu, damp, wd, nes = g["lr"], g["momentum"], g["dampening"], g["weight_decay"], g["nesterov"]
        sp = self.space
        if self._gpu:
            if not torch.cuda.is_current_stream_capturing():  # replays get it from GraphedStep.pre_replay
                self._lr_t.fill_(lr)
            hip().sgd_step(sp.flat_param, sp.flat_grad, self.momentum_buffer, self.shadow, lr, self._lr_t, mu, damp,
                           wd, self.grad_scale, nes, self._first)
        else:
            d = sp.flat_grad * self.grad_scale
            if wd:
                d.add_(sp.flat_param, alpha=wd)
            if mu:
                m = self.momentum_buffer
                if self._first:
                    m.copy_(d)
                else:
                    m.mul_(mu).add_(d, alpha=1.0 - damp)
                d = d.add(m, alpha=mu) if nes else m
            sp.flat_param.add_(d, alpha=-lr)
            if self.shadow is not None:
                self.shadow.copy_(sp.flat_param)
        self._first = False
        return loss

    # host-side scalars that must match across replicas (broadcast_optimizer_state):
    # a worker that joins a running job must not re-initialise the broadcast momentum
    def _kf_scalars(self):
        return [float(self._first)]

    def _kf_load_scalars(self, vals):
        self._first = bool(vals[0])

    def state_dict(self):
        sd = super().state_dict()
        sd["kungfu_flat"] = {"momentum_buffer": self.momentum_buffer, "first": self._first}
        return sd

    def load_state_dict(self, sd):
        flat = sd.pop("kungfu_flat", None)
        super().load_state_dict(sd)
        if flat is not None:
            if flat["momentum_buffer"] is not None and self.momentum_buffer is not None:
                self.momentum_buffer.copy_(flat["momentum_buffer"])
            self._first = flat["first"]


class FusedAdam(torch.optim.Optimizer):
    """Adam / AdamW over a flat space; one kernel per step, bias correction on device."""

    def __init__(self, space: FlatParamSpace, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, adamw: bool = True, grad_scale: float = 1.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(space.params, defaults)
        self.space = space
        self.adamw = adamw
        self.grad_scale = grad_scale
        self.exp_avg = torch.zeros_like(space.flat_param)
        self.exp_avg_sq = torch.zeros_like(space.flat_param)
        self._step_t = torch.zeros(1, dtype=torch.float32, device=space.device)
        self._lr_t = torch.full((1,), lr, dtype=torch.float32, device=space.device)
        self._gpu = space.device.type == "cuda"
        if self._gpu:
            hip()

    def zero_grad(self, set_to_none: bool = False):
        self.space.zero_grad()

    def state_dict(self):
        sd = super().state_dict()
        sd["kungfu_flat"] = {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "step": self._step_t}
        return sd

    def load_state_dict(self, sd):
        flat = sd.pop("kungfu_flat", None)
        super().load_state_dict(sd)
        if flat is not None:
            self.exp_avg.copy_(flat["exp_avg"])
            self.exp_avg_sq.copy_(flat["exp_avg_sq"])
            self._step_t.copy_(flat["step"])

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
        sp = self.space
        self._step_t.add_(1.0)
        if self._gpu:
            if not torch.cuda.is_current_stream_capturing():
                self._lr_t.fill_(lr)
            # the bf16 compute shadow is written by the same kernel (eager steps): the next forward's cast of
            # the whole model is skipped (FlatParamSpace.mark_shadow_fresh; -0.14 ms per BERT-base step)
            sh = sp.flat_shadow if (sp.flat_shadow is not None and not torch.cuda.is_current_stream_capturing()) else None
            hip().adam_step(sp.flat_param, sp.flat_grad, self.exp_avg, self.exp_avg_sq, lr, self._lr_t, b1, b2, eps,
                            wd, self.adamw, self.grad_scale, self._step_t, sh)
            if sh is not None:
                sp.mark_shadow_fresh()
        else:
            t = float(self._step_t.item())
            gr = sp.flat_grad * self.grad_scale
            if self.adamw:
                sp.flat_param.mul_(1 - lr * wd)
            elif wd:
                gr = gr.add(sp.flat_param, alpha=wd)
            self.exp_avg.mul_(b1).add_(gr, alpha=1 - b1)
            self.exp_avg_sq.mul_(b2).addcmul_(gr, gr, value=1 - b2)
            denom = (self.exp_avg_sq.sqrt() / (1 - b2 ** t) ** 0.5).add_(eps)
            sp.flat_param.addcdiv_(self.exp_avg, denom, value=-lr / (1 - b1 ** t))
        return loss
