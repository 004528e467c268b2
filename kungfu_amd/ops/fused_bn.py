"""Fused NHWC BatchNorm(+residual)+ReLU(+MaxPool) modules backed by HIP kernels (bn.hip).

``BatchNormAct2d``    y = relu(bn(x))               (relu optional)
``BatchNormAddAct2d`` y = relu(bn(x) + residual)    (ResNet bottleneck tail)
``BatchNormAct2d.forward_pool``  y = maxpool3x3s2p1(relu(bn(x)))  (ResNet stem)

Both subclass ``nn.BatchNorm2d`` (same parameters, buffers and state_dict
keys).  The HIP path runs for bf16, 4-D, channels_last inputs on GPU with a
supported channel count (C % 8 == 0 with C/8 in {4, 6, 8, 10, 12, 16, 20, 24, 32,
40, 48, 56, 64, 128, 256}: every ResNet and Inception-v3 BN, 32 to 2048 channels);
anything else uses the PyTorch composition, so results are the same model either way.

What is saved for backward is chosen to minimise HBM traffic: x (already kept
alive as the producing conv's output), the per-channel forward coefficients
(the ReLU mask is recomputed from x), and for the residual variant a 1-bit
ReLU mask.  y itself is never re-read.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._lib import hip, hip_available
from ..parallel.mixed import deliver, direct_target

import os

# CONCAT_ENABLED = False (module attribute): apply deferred branch BNs and concatenate with torch.cat (A/B, tests)
CONCAT_ENABLED = True  # module switch (tests)


def available() -> bool:
    return torch.cuda.is_available() and hip_available()


def _fusable(x: torch.Tensor, res: Optional[torch.Tensor]) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    if not x.is_contiguous(memory_format=torch.channels_last):
        return False
    if res is not None and (res.dtype != torch.bfloat16 or res.shape != x.shape or
                            not res.is_contiguous(memory_format=torch.channels_last)):
        return False
    return hip().bn_supported_channels(x.shape[1])


def _param_grads(ctx, dw, db):
    """Gamma/beta gradients: handed to the flat space's sink when the params
    are registered for direct gradients (parallel/mixed.py), else returned."""
    if ctx.direct is None:
        return dw, db
    tw, tb = ctx.direct
    deliver(tw, dw)
    deliver(tb, db)
    return None, None


def _direct(weight, bias):
    tw, tb = direct_target(weight), direct_target(bias)
    return (tw, tb) if tw is not None and tb is not None else None


class BNLink:
    """Link from a BN+ReLU output to the ONE convolution that consumes it (ops/conv.py): that
    conv's data gradient IS the gradient of this output, so its epilogue can accumulate this BN's
    backward sums (sum dz, sum dz*x under the ReLU gate) into ``ws`` -- the BN backward then skips
    its reduction pass.  ``dx_ptr`` lets the BN check it received exactly that tensor.  Only
    created where the model guarantees a single consumer (an in-place autograd accumulation
    of a second consumer's gradient would otherwise keep the pointer but change the values)."""
    __slots__ = ("ws", "y", "coef", "ready", "dx_ptr")

    def __init__(self, ws, y, coef):
        self.ws, self.y, self.coef = ws, y, coef
        self.ready = False
        self.dx_ptr = 0


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, weight, bias, running_mean, running_var, momentum, eps, training, relu, nbt, sums=None,
                link_ws=None):
        y, mean, invstd, coef, mask = hip().bn_forward(x, res, weight, bias, running_mean, running_var, momentum, eps,
                                                       training, relu, nbt, sums)
        ctx.save_for_backward(x, mean, invstd, weight, coef, mask)
        ctx.relu, ctx.training, ctx.has_res = relu, training, res is not None
        ctx.direct = _direct(weight, bias)
        ctx.link = BNLink(link_ws, x, coef) if link_ws is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, invstd, weight, coef, mask = ctx.saved_tensors
        link, sums = ctx.link, None
        if link is not None:
            if link.ready and dy.data_ptr() == link.dx_ptr:
                sums = link.ws  # the consumer conv's epilogue produced this BN's backward sums
            elif link.ready:
                link.ws.zero_()  # sums of a gradient that is not the one we got: discard
            link.ready, link.y, link.coef = False, None, None
        dx, dres, dw, db = hip().bn_backward(dy, x, mean, invstd, weight, coef, mask, ctx.relu, ctx.training,
                                             ctx.has_res, sums)
        dw, db = _param_grads(ctx, dw, db)
        return dx, (dres if ctx.has_res else None), dw, db, None, None, None, None, None, None, None, None, None


class _BNActPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, training, nbt, sums):
        y, mean, invstd, coef, arg, xarg = hip().bn_pool_forward(x, weight, bias, running_mean, running_var, momentum,
                                                                 eps, training, nbt, sums)
        # xarg (training): pre-BN value of each window's argmax -> the backward's BN sums run
        # over the pooled map
        ctx.save_for_backward(x, mean, invstd, weight, coef, arg, xarg)
        ctx.training = training
        ctx.direct = _direct(weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, invstd, weight, coef, arg, xarg = ctx.saved_tensors
        dx, dw, db, _ = hip().bn_pool_backward(dy, arg, x, mean, invstd, weight, coef, ctx.training, xarg)
        dw, db = _param_grads(ctx, dw, db)
        return dx, dw, db, None, None, None, None, None, None, None


def bn_act(x, weight, bias, running_mean, running_var, training: bool, momentum: float, eps: float,
           relu: bool = True, res: Optional[torch.Tensor] = None,
           num_batches_tracked: Optional[torch.Tensor] = None, sums: Optional[torch.Tensor] = None,
           link_ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Functional fused BN(+res)(+ReLU); falls back to torch ops when not fusable.

    ``num_batches_tracked`` (if given, training mode) is incremented on device.  ``sums``
    (training): batch statistics already accumulated by the producing conv's epilogue
    (``ops.conv.conv2d_stats``), consumed and re-zeroed -- no statistics pass.  ``link_ws``
    (training, BN+ReLU without residual): the output gets a :class:`BNLink` (``._kf_link``) so
    its single consuming conv produces this BN's backward sums into ``link_ws`` (zeroed)."""
    if _fusable(x, res) and weight is not None and momentum is not None:
        lw = link_ws if (training and relu and res is None) else None
        y = _BNActFn.apply(x, res, weight, bias, running_mean, running_var, momentum, eps, training, relu,
                           num_batches_tracked if training else None, sums if training else None, lw)
        if lw is not None and y.grad_fn is not None:
            y._kf_link = y.grad_fn.link
        return y
    if sums is not None:
        sums.zero_()  # not consumed by the fallback below
    if training and num_batches_tracked is not None:
        num_batches_tracked.add_(1)
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if res is not None:
        y = y + res
    return F.relu(y) if relu else y


def bn_act_pool(x, weight, bias, running_mean, running_var, training: bool, momentum: float, eps: float,
                num_batches_tracked: Optional[torch.Tensor] = None, sums: Optional[torch.Tensor] = None) -> torch.Tensor:
    """maxpool3x3s2p1(relu(bn(x))) -- one HIP forward kernel pass, one gather backward.

    ``sums``: batch statistics already accumulated by the producing conv's epilogue
    (``ops.stem``), consumed and re-zeroed -- no statistics pass."""
    if (_fusable(x, None) and weight is not None and momentum is not None and
            hip().bn_pool_supported(x.shape[1], x.shape[2], x.shape[3])):
        return _BNActPoolFn.apply(x, weight, bias, running_mean, running_var, momentum, eps, training,
                                  num_batches_tracked if training else None, sums if training else None)
    if sums is not None:
        sums.zero_()  # not consumed by the fallback below
    y = bn_act(x, weight, bias, running_mean, running_var, training, momentum, eps, relu=True,
               num_batches_tracked=num_batches_tracked)
    return F.max_pool2d(y, 3, 2, 1)


class Deferred:
    """A BN+ReLU whose application is deferred to a concatenation (:func:`bn_relu_concat`):
    ``y`` is the BN input (the conv output), ``bn`` the :class:`BatchNormAct2d`, ``sums`` the
    batch statistics its producing conv's epilogue accumulated (or None)."""
    __slots__ = ("y", "bn", "sums")

    def __init__(self, y, bn, sums=None):
        self.y, self.bn, self.sums = y, bn, sums

    def materialize(self) -> torch.Tensor:
        return self.bn(self.y, sums=self.sums)


class _ConcatSpec:
    __slots__ = ("items", "ctot")

    def __init__(self, items, ctot):
        self.items, self.ctot = items, ctot  # items: (bn module, sums) or None for a plain tensor


# the concatenation's BN finalizes batched, one launch per direction (Inception-v3 12607 -> 12809 img/s,
# r4t25); KUNGFU_BN_BATCH_FIN=0: one per BN
_BATCH_FIN = True  # module switch (tests)


class _BNConcatFn(torch.autograd.Function):
    """``torch.cat([relu(bn_i(y_i)) ..., t_j ...], 1)`` without the copy: each BN+ReLU apply pass
    writes straight into its channel slice of the concatenation (a strided HIP store), the plain
    pieces (e.g. a max-pool branch) are copied into theirs; backward reads each slice of the
    output gradient in place (the BN backward takes a strided gradient)."""

    @staticmethod
    def forward(ctx, spec: _ConcatSpec, *args):
        H = hip()
        first = args[0]
        N, _, Hh, W = first.shape
        out = torch.empty((N, spec.ctot, Hh, W), dtype=torch.bfloat16, device=first.device,
                          memory_format=torch.channels_last)
        saved, direct, k, c0 = [], [], 0, 0
        # the conv-statistics BNs of the block: finalized together in ONE launch (bn_finalize_multi),
        # then each applies straight into its slice with those coefficients
        pre = {}
        if _BATCH_FIN:
            fin, kk = [], 0
            for idx, item in enumerate(spec.items):
                if item is not None:
                    if item[1] is not None:
                        fin.append((idx, args[kk], args[kk + 1], args[kk + 2], item))
                    kk += 3
                else:
                    kk += 1
            if 2 <= len(fin) <= 8:
                cols = [[], [], [], [], [], [], [], [], []]
                for _, y, g, b, (m, sums) in fin:
                    a, nbt = m._args()
                    for lst, v in zip(cols, (y, sums, g, b, a[2], a[3], nbt, float(a[5]), float(a[6]))):
                        lst.append(v)
                for (idx, *_), r in zip(fin, H.bn_finalize_multi(*cols)):
                    pre[idx] = r
        for idx, item in enumerate(spec.items):
            if item is not None:
                y, g, b = args[k:k + 3]
                k += 3
                m, sums = item
                a, nbt = m._args()
                C = int(y.shape[1])
                _, mean, invstd, coef, _ = H.bn_forward(y, None, g, b, a[2], a[3], a[5], a[6], True, True, nbt, sums,
                                                        None, True, out[:, c0:c0 + C], pre.get(idx))
                saved += [y, mean, invstd, g, coef]
                direct.append(_direct(g, b))
            else:
                t = args[k]
                k += 1
                C = int(t.shape[1])
                out[:, c0:c0 + C].copy_(t)
            c0 += C
        ctx.save_for_backward(*saved)
        ctx.spec, ctx.direct = spec, direct
        ctx.plain = [int(t.shape[1]) for t, it in zip(_plain_args(spec, args), spec.items) if it is None]
        return out

    @staticmethod
    def backward(ctx, dout):
        H = hip()
        if not dout.is_contiguous(memory_format=torch.channels_last):
            dout = dout.contiguous(memory_format=torch.channels_last)
        saved = list(ctx.saved_tensors)
        grads, c0, si, pi, bi = [], 0, 0, 0, 0
        multi = None
        nbn = sum(1 for it in ctx.spec.items if it is not None)
        if _BATCH_FIN and 2 <= nbn <= 8:
            # every branch BN's reduce pass, ONE batched finalize, every apply (bn_backward_multi)
            cols, cc, ss, pp = [[], [], [], [], [], []], 0, 0, 0
            for item in ctx.spec.items:
                if item is not None:
                    y, mean, invstd, g, coef = saved[ss:ss + 5]
                    ss += 5
                    C = int(y.shape[1])
                    for lst, v in zip(cols, (dout[:, cc:cc + C], y, mean, invstd, g, coef)):
                        lst.append(v)
                    cc += C
                else:
                    cc += ctx.plain[pp]
                    pp += 1
            multi = iter(H.bn_backward_multi(*cols))
        for item in ctx.spec.items:
            if item is not None:
                y, mean, invstd, g, coef = saved[si:si + 5]
                si += 5
                C = int(y.shape[1])
                if multi is not None:
                    dx, dw, db = next(multi)
                else:
                    dx, _, dw, db = H.bn_backward(dout[:, c0:c0 + C], y, mean, invstd, g, coef, None, True, True,
                                                  False, None)
                d = ctx.direct[bi]
                bi += 1
                if d is not None:
                    deliver(d[0], dw)
                    deliver(d[1], db)
                    dw = db = None
                grads += [dx, dw, db]
            else:
                C = ctx.plain[pi]
                pi += 1
                grads.append(dout[:, c0:c0 + C])
            c0 += C
        return (None, *grads)


def _plain_args(spec, args):
    """The argument (first tensor) of each piece, in piece order."""
    out, k = [], 0
    for item in spec.items:
        out.append(args[k])
        k += 3 if item is not None else 1
    return out


def bn_relu_concat(pieces) -> torch.Tensor:
    """``torch.cat`` over channels of ``pieces`` (tensors and :class:`Deferred` BN+ReLUs), with every
    deferred BN+ReLU written straight into its slice of the result when the HIP path covers the whole
    set (bf16 channels_last pieces of one N x H x W, channel offsets % 8, training-mode BNs with
    running statistics); otherwise the BNs are applied and the pieces concatenated by torch."""
    ok = CONCAT_ENABLED
    ref = None
    c0 = 0
    for p in (pieces if ok else ()):
        t = p.y if isinstance(p, Deferred) else p
        if ref is None:
            ref = t
        if (t.dtype != torch.bfloat16 or not t.is_cuda or t.shape[0] != ref.shape[0] or t.shape[2:] != ref.shape[2:]
                or c0 % 8):
            ok = False
            break
        if isinstance(p, Deferred):
            m = p.bn
            if not (m.training and m.track_running_stats and m.relu and m.momentum is not None
                    and _fusable(t, None) and type(m).forward is BatchNormAct2d.forward):
                ok = False
                break
        c0 += int(t.shape[1])
    if not ok or not any(isinstance(p, Deferred) for p in pieces):
        return torch.cat([p.materialize() if isinstance(p, Deferred) else p for p in pieces], 1)
    items, args = [], []
    for p in pieces:
        if isinstance(p, Deferred):
            items.append((p.bn, p.sums))
            args += [p.y, p.bn.weight, p.bn.bias]
        else:
            items.append(None)
            args.append(p)
    return _BNConcatFn.apply(_ConcatSpec(items, c0), *args)


class BatchNormAct2d(nn.BatchNorm2d):
    def __init__(self, num_features: int, relu: bool = True, eps: float = 1e-5, momentum: float = 0.1):
        super().__init__(num_features, eps=eps, momentum=momentum)
        self.relu = relu

    def _args(self):
        track = self.training and self.track_running_stats
        use_batch = self.training or self.running_mean is None
        stats = not self.training or self.track_running_stats
        return (self.weight, self.bias, self.running_mean if stats else None, self.running_var if stats else None,
                use_batch, self.momentum, self.eps), (self.num_batches_tracked if track else None)

    def forward(self, x, sums: Optional[torch.Tensor] = None, link: bool = False):
        """``sums``: batch statistics from the producing conv's epilogue (training only).
        ``link``: the output has exactly one consumer, a conv on the MFMA kernel (see bn_act)."""
        a, nbt = self._args()
        lw = self.stats_workspace(x.device) if (link and a[4] and self.track_running_stats) else None
        return bn_act(x, *a, relu=self.relu, num_batches_tracked=nbt, sums=sums if a[4] else None, link_ws=lw)

    def stats_workspace(self, dev) -> torch.Tensor:
        """Zeroed f64 [slots, 2, C] workspace a conv epilogue accumulates this BN's batch
        statistics into (consumed and re-zeroed by the BN kernels)."""
        ws = getattr(self, "_kf_sums", None)
        if ws is None or ws.device != dev:
            ws = torch.zeros(hip().conv_stat_slots * 2 * self.num_features, dtype=torch.float64, device=dev)
            self._kf_sums = ws
        return ws

    def forward_pool(self, x, sums: Optional[torch.Tensor] = None):
        """relu(bn(x)) followed by MaxPool2d(3, stride 2, padding 1), fused (``sums``: batch
        statistics from the producing conv's epilogue)."""
        assert self.relu
        a, nbt = self._args()
        return bn_act_pool(x, *a, num_batches_tracked=nbt, sums=sums if a[4] else None)


class BatchNormAddAct2d(BatchNormAct2d):
    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1):
        super().__init__(num_features, relu=True, eps=eps, momentum=momentum)

    def forward(self, x, res):
        a, nbt = self._args()
        return bn_act(x, *a, relu=True, res=res, num_batches_tracked=nbt)
