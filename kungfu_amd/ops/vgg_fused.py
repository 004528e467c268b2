"""VGG-16's feature stack (13 conv3x3+bias+ReLU, 5 max-pools) as ONE autograd node whose
every bias/ReLU lives inside a convolution or pool kernel.

Layered, each conv+bias+ReLU costs a separate in-place bias+ReLU pass over its output in
forward and a gate + bias-reduce pass over its output gradient in backward (``_BiasActFn``:
7.5 ms of a 38.9 ms step at batch 256, profiles/README.md).  Owning the whole stack, the
backward knows that the gradient of layer L's ReLU output is consumed only by layer L's
bias/ReLU, so it is produced already gated:

  forward   layer 0: library conv of the image + the in-place bias+ReLU pass (3 channels);
            layers 1..12: ``hip.conv(..., bias=b)`` -- relu(conv + b) in the MFMA epilogue;
            pools: ``hip.maxpool2x2_forward``.
  backward  pool after layer L: ``maxpool2x2_backward(gate_stats=...)`` gathers, gates by the
            window maximum > 0 and sums the bias gradient per channel;
            conv L+1 directly after layer L: its data gradient ``hip.conv(..., gate=True)``
            gates by layer L's output in the epilogue and sums the bias gradient there;
            weight gradients: ``ops.conv.wgrad`` (the row-image 3x3 kernel for <= 128
            channels, the tap-tiled split-K kernel above; MIOpen for the 3-channel image).

The bias gradients land in one zeroed f64 workspace (kStatSlots x 2 x C per layer, slot 0 row
used) and are folded per layer.  Numerics match the layered path: the same bf16 conv outputs
(bias added in f32 before the one rounding instead of after it), the same gated bf16 gradients.

Reference parity: BASELINE.md VGG16 rows (``benchmarks/system/result/sync-scalability.svg``);
the reference trains ``tf.keras.applications.VGG16`` with TF's stock kernels.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._lib import buf_ok, hip, hip_available
from .. import knobs

_ENABLED = knobs.get("KUNGFU_VGG_FUSED") != "0"

_CL = torch.channels_last


class _FeaturesFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pool_after: Tuple[bool, ...], *wb):
        H = hip()
        ws, bs = wb[0::2], wb[1::2]
        n = len(pool_after)
        x0 = x.to(torch.bfloat16).contiguous(memory_format=_CL)  # what autocast hands the first conv
        inputs: List[torch.Tensor] = [x0]
        pooled_src: List[torch.Tensor] = []  # ReLU outputs that feed a pool (the pool's x)
        y = F.conv2d(x0, ws[0], None, 1, 1).contiguous(memory_format=_CL)
        H.bias_act_forward_(y, bs[0].float().contiguous(), True)
        for L in range(n):
            if L > 0:
                y = H.conv(inputs[L], ws[L], 1, None, None, -1, bias=bs[L])
            if pool_after[L]:
                pooled_src.append(y)
                y = H.maxpool2x2_forward(y)
            if L + 1 < n:
                inputs.append(y)
        ctx.pool_after = pool_after
        ctx.n_in = len(inputs)
        ctx.save_for_backward(*inputs, *pooled_src, *ws)
        ctx.bias_dtype = bs[0].dtype
        return y

    @staticmethod
    def backward(ctx, g):
        from .conv import wgrad

        H = hip()
        pool_after = ctx.pool_after
        n = len(pool_after)
        saved = ctx.saved_tensors
        inputs = saved[:ctx.n_in]
        n_pool = sum(pool_after)
        pooled_src = list(saved[ctx.n_in:ctx.n_in + n_pool])
        ws = saved[ctx.n_in + n_pool:]
        slots = H.conv_stat_slots
        couts = [int(w.shape[0]) for w in ws]
        offs = [0]
        for c in couts:
            offs.append(offs[-1] + slots * 2 * c)
        stats = torch.zeros(offs[-1], dtype=torch.float64, device=g.device)
        st = [stats[offs[L]:offs[L + 1]] for L in range(n)]
        g = g.contiguous(memory_format=_CL)
        dws: List[torch.Tensor] = [None] * n  # type: ignore[list-item]
        dbs: List[torch.Tensor] = [None] * n  # type: ignore[list-item]
        for L in reversed(range(n)):
            if pool_after[L]:
                dz = H.maxpool2x2_backward(pooled_src.pop(), g, gate_stats=st[L])
            else:
                dz = g  # gated by conv L+1's data-gradient epilogue, bias sums in st[L]
            dbs[L] = st[L].view(slots, 2, couts[L])[:, 0].sum(0).to(ctx.bias_dtype)
            dws[L] = wgrad(dz, inputs[L], ws[L], 1, 1)
            if L > 0:
                wf = H.conv3x3_flip_weight(ws[L])
                if pool_after[L - 1]:
                    g = H.conv(dz, wf, 1)  # gradient of the pool output
                else:  # gradient of layer L-1's ReLU output (= this conv's input), gated
                    g = H.conv(dz, wf, 1, st[L - 1], None, -1, bn_x=inputs[L], gate=True)
        out = [None, None]
        for L in range(n):
            out += [dws[L], dbs[L]]
        return tuple(out)


class FusedVGGFeatures(nn.Sequential):
    """``nn.Sequential`` of ``Conv2dReLU`` / ``nn.Identity`` / ``MaxPool2x2`` (the module layout
    ``models.vgg`` builds, so state_dict keys are unchanged) whose forward runs the whole stack
    as one ``_FeaturesFn`` node when the MFMA path applies, and layer by layer otherwise."""

    def _plan(self) -> Tuple[List[nn.Conv2d], Tuple[bool, ...]]:
        from .conv import Conv2dReLU
        from .pool import MaxPool2x2

        convs: List[nn.Conv2d] = []
        pool_after: List[bool] = []
        for m in self:
            if isinstance(m, Conv2dReLU):
                convs.append(m)
                pool_after.append(False)
            elif isinstance(m, MaxPool2x2):
                if not pool_after or pool_after[-1]:
                    return [], ()
                pool_after[-1] = True
            elif not isinstance(m, nn.Identity):
                return [], ()
        return convs, tuple(pool_after)

    def _eligible(self, x: torch.Tensor, convs: Sequence[nn.Conv2d], pool_after: Sequence[bool] = ()) -> bool:
        if not convs or not x.is_cuda or not hip_available() or x.dim() != 4 or not _ENABLED:
            return False
        if not (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            return False
        # every layer's activations (N * H_l * W_l * its widest channel count, at ITS resolution: the
        # max-pools halve it) must stay below the conv kernels' 2 GiB buffer-resource range
        n, h, w = x.shape[0], x.shape[2], x.shape[3]
        for i, c in enumerate(convs):
            if not buf_ok(n * h * w * max(c.in_channels, c.out_channels)):
                return False
            if i < len(pool_after) and pool_after[i]:
                h, w = h // 2, w // 2
        H = hip()
        for i, c in enumerate(convs):
            if c.kernel_size != (3, 3) or c.stride != (1, 1) or c.padding != (1, 1) or c.groups != 1 or c.bias is None:
                return False
            if i > 0 and not H.conv3x3_supported(c.in_channels, c.out_channels, 1):
                return False
            if not H.bias_act_supported(c.out_channels):
                return False
        return True

    def forward(self, x):
        convs, pool_after = self._plan()
        if not self._eligible(x, convs, pool_after):
            return super().forward(x)
        from ..parallel.mixed import shadow

        wb = []
        for c in convs:
            w, b = shadow(c.weight), shadow(c.bias)
            if w.dtype != torch.bfloat16:
                w = w.to(torch.bfloat16)
            if b.dtype != torch.bfloat16:
                b = b.to(torch.bfloat16)
            wb += [w.contiguous(memory_format=_CL), b.contiguous()]
        return _FeaturesFn.apply(x, pool_after, *wb)
