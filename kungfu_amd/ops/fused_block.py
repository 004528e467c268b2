"""One autograd node per ResNet bottleneck block, sequenced by hand on the HIP kernels.

Why a block-level node: with one node per conv / BN, autograd materialises every
intermediate exactly as the modules produce it and sums the two gradients that reach
each block input (identity + conv1 data gradient) with a separate elementwise add
(16 per ResNet-50 step, 1.3 ms of 28 ms on MI355X, profiles/r7_*.md), and each BN
re-reads its input for batch statistics.  Owning the block's forward and backward
lets the MI355X kernels fuse across layer boundaries:

forward (training)
* every convolution (1x1 and 3x3, stride 1/2) runs on the MFMA implicit-GEMM kernel
  (csrc/kernels/conv.hip) whose epilogue also accumulates the per-channel
  sum / sum-of-squares of its bf16 output (slotted f64 atomics) -> the BN that follows
  skips its statistics pass and only folds the sums (``bn_forward(..., sums=)``);
* BN(+ReLU) and BN3 + residual + ReLU are the fused bn.hip kernels.

backward
* stride-1 data gradients are the same MFMA kernel on transposed/flipped weights, whose
  epilogue also accumulates the backward sums (sum dz, sum dz*x under the ReLU gate) of the
  BN that produced the conv input -> that BN's backward skips its reduction pass; stride-2
  data gradients (conv2 3x3 and the downsample 1x1 of layers 2-4) are parity-phase GEMMs on
  the same kernel (``conv_dgrad_s2``: each output pixel parity sees 1, 2 or 4 taps; the 1x1's
  even-pixel gradient is completed by conv1's data gradient, no zero fill); across
  blocks, the next block's conv1 data gradient does this for the previous block's BN3
  (``_TailSlot``);
* the block-input gradient is formed IN PLACE: conv1's data-gradient kernel
  accumulates into the identity gradient produced by the BN3+add+ReLU backward
  (or into the downsample branch's data gradient) -- no elementwise add, no extra
  pass over the largest activation of the block;
* weight gradients use the split-K MFMA kernel (``ops.conv.wgrad``, csrc/kernels/conv_wgrad.hip);
* BN gamma/beta gradients go to the flat space's gradient sink when registered
  (parallel/mixed.py), conv weight gradients flow to the bf16 shadow views.

Saved tensors are the same as per-layer autograd would keep (conv inputs, BN inputs,
per-channel coefficients, the 1-bit ReLU mask of the block tail).

No reference counterpart: the reference trains ``tf.keras.applications`` ResNet-50
with stock TF kernels (``benchmarks/system/benchmark_kungfu.py:96``).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.nn.functional as F

from .._lib import buf_ok, hip, hip_available
from ..parallel.mixed import deliver, direct_target, shadow

_ENABLED = os.environ.get("KUNGFU_FUSED_BLOCK", "1") != "0"


# Test hook (tests/test_gpu_engine.py): a list that every backward appends each BN's gradient inputs
# and its (dgamma, dbeta) to, so the fused BN-backward sums can be checked against an f64 reduction
# of the SAME bf16 tensors; None (the default) records nothing.
_CAPTURE = None


def _capture(bn, kind, dz, x, mean, invstd, gate, dg, db):
    """kind "relu": gate = the forward [scale; shift] (relu'(x*scale+shift)); "mask": gate = the
    1-bit ReLU mask; "plain": no gate (the downsample BN inside the residual add)."""
    _CAPTURE.append(dict(bn=bn, kind=kind, dz=dz.detach().clone(), x=x.detach().clone(), mean=mean.clone(),
                         invstd=invstd.clone(), gate=None if gate is None else gate.clone(),
                         dg=dg.detach().clone(), db=db.detach().clone()))


def set_enabled(on: bool) -> bool:
    global _ENABLED
    old, _ENABLED = _ENABLED, bool(on)
    return old


def _cl(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous(memory_format=torch.channels_last) else t.contiguous(memory_format=torch.channels_last)


def _sums(bn, dev) -> torch.Tensor:
    """Per-BN f64 statistics workspace (kept zeroed by the finalize kernel)."""
    ws = getattr(bn, "_kf_sums", None)
    if ws is None or ws.device != dev:
        ws = torch.zeros(hip().conv_stat_slots * 2 * bn.num_features, dtype=torch.float64, device=dev)
        bn._kf_sums = ws
    return ws


# _INLAUNCH_FIN (module attribute; the retired KUNGFU_BN_INLAUNCH_FIN): the statistics-producing conv finalizes its BN in its own launch
# (last-arriving workgroup, csrc/kernels/conv.hip bn_finalize_last; bit-identical).  Off by default:
# measured 0.55-1.25 ms/step SLOWER on ResNet-50 than the separate finalize launches (every
# workgroup must wait for its memory-side f64 slot atomics before it may arrive, and the arrivals
# and the last workgroup's fold sit on the launch's critical path), although dropping the finalize
# launches altogether would save 1.0 ms (KUNGFU_BN_SKIP_FINALIZE timing experiment).
_INLAUNCH_FIN = False  # BN finalize inside the statistics conv (r3: 0.55 ms/step slower); a switch for its test


def _kw(**kw):
    """The keyword arguments that are not None (older extension builds lack fin / pre)."""
    return {k: v for k, v in kw.items() if v is not None}


class _BNFinState:
    """Per-BN in-launch finalize state: the arrival counters and a ring of ``RING`` generations of
    (output buffers, device descriptor) -- the forward's mean / invstd / coefficients and the
    backward's dgamma / dbeta / coefficients live in persistent buffers the descriptors point at
    (packed once, rebuilt only when a pointer or the row count changes).  A generation is reused
    ``RING`` forwards later, so up to that many forwards may be outstanding before their backward."""
    RING = 4

    def __init__(self):
        self.key = None
        self.gen = 0
        self.fwd = self.bwd = None

    def _build(self, bn, gamma, beta, rows, dev):
        H = hip()
        C = bn.num_features
        f32 = dict(dtype=torch.float32, device=dev)
        self.arrive = torch.zeros(16, dtype=torch.int32, device=dev)
        self.fwd, self.bwd = [], []
        for _ in range(self.RING):
            mean, invstd, coef = torch.empty(C, **f32), torch.empty(C, **f32), torch.empty(2 * C, **f32)
            d = H.bn_fin_desc(1, [self.arrive, gamma, beta, mean, invstd, coef, bn.running_mean, bn.running_var,
                                  bn.num_batches_tracked], rows, float(bn.momentum), float(bn.eps), True).to(dev)
            self.fwd.append((d, [mean, invstd, coef]))
            dg, db, c3 = torch.empty(C, **f32), torch.empty(C, **f32), torch.empty(3 * C, **f32)
            d2 = H.bn_fin_desc(2, [self.arrive, gamma, mean, invstd, c3, dg, db], rows, 0.0, 0.0, True).to(dev)
            self.bwd.append((d2, [dg, db, c3]))

    def next_fwd(self, bn, gamma, beta, rows, dev):
        key = (gamma.data_ptr(), beta.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
               bn.num_batches_tracked.data_ptr(), int(rows), float(bn.momentum), float(bn.eps))
        if key != self.key:
            self._build(bn, gamma, beta, rows, dev)
            self.key = key
        g = self.gen
        self.gen = (g + 1) % self.RING
        return g


def _fin_state(bn) -> _BNFinState:
    st = getattr(bn, "_kf_fin", None)
    if st is None:
        st = bn._kf_fin = _BNFinState()
    return st


def _fin_fwd(bn, gamma, beta, rows, dev):
    """(conv kwargs, bn_forward pre, generation) for a forward statistics epilogue that finalizes
    in its own launch; the generation selects the backward buffers (:func:`_fin_bwd`)."""
    if not _INLAUNCH_FIN:
        return {}, None, None
    st = _fin_state(bn)
    g = st.next_fwd(bn, gamma, beta, rows, dev)
    d, pre = st.fwd[g]
    return dict(fin=d), pre, g


def _fin_bwd(bn, gen):
    """(fin descriptor, bn_backward pre) for the BN-backward-sums epilogue of the forward generation
    ``gen`` (None: finalize separately)."""
    if gen is None or not _INLAUNCH_FIN:
        return None, None
    d, pre = _fin_state(bn).bwd[gen]
    return d, pre


def _wgrad(dy, x, w, stride, pad):
    from .conv import wgrad

    return wgrad(dy, x, w, stride, pad)


class _FlipCache:
    """Data-gradient weights (``conv_flip_weight``) of every registered bf16 shadow conv
    weight of one flat space, produced by ONE multi-tensor kernel per shadow refresh
    (i.e. per step) on first use in backward, instead of one launch per convolution."""

    def __init__(self, space):
        self.space = space
        self.index = {}  # param index -> flipped tensor
        self.gen = -1

    def register(self, i: int, w: torch.Tensor):
        if i not in self.index:
            co, ci, kh, kw = w.shape
            self.index[i] = torch.empty((ci, co, kh, kw), dtype=torch.bfloat16, device=w.device).contiguous(
                memory_format=torch.channels_last)
            self.gen = -1

    def get(self, i: int) -> torch.Tensor:
        if self.gen != self.space.shadow_gen:
            idx = sorted(self.index)
            # linear weights [out, in] are 1x1 convolutions [out, in, 1, 1]: their flip is W^T
            ws = [self.space.shadow_view(j) for j in idx]
            ws = [w if w.dim() == 4 else w.view(w.shape[0], w.shape[1], 1, 1) for w in ws]
            hip().conv_flip_weights(ws, [self.index[j] for j in idx])
            self.gen = self.space.shadow_gen
        return self.index[i]


def _flip_cache(space) -> _FlipCache:
    c = getattr(space, "_kf_flip", None)
    if c is None:
        c = space._kf_flip = _FlipCache(space)
    return c


def _dgrad(dy, x, w, stride, pad, out: Optional[torch.Tensor] = None, flipped: Optional[torch.Tensor] = None,
           bn=None, out_mask: Optional[torch.Tensor] = None, acc_even: bool = False):
    """Data gradient on the MFMA kernels (accumulating into ``out`` if given).

    ``bn = (ws, bn_x, fcoef, mask)``: the result is the gradient of a BN(+ReLU) output whose
    input is ``bn_x``; the kernel epilogue also accumulates that BN's backward sums into
    ``ws`` (returns whether it did via ``_dgrad.fused``).
    ``out_mask`` (stride 1, with ``out``): accumulate into ``out * out_mask`` (1-bit ReLU mask).
    ``acc_even`` (stride 1, with ``out``): ``out`` holds a stride-2 1x1 data gradient at its even
    pixels only (``_dgrad_s2``); the other pixels are plainly stored.
    Stride 2 with an even input: parity-phase GEMMs (``conv_dgrad_s2``); odd inputs fall back
    to the library kernel."""
    H = hip()
    wt = flipped if flipped is not None else None
    if stride == 1:
        wt = wt if wt is not None else H.conv_flip_weight(w)
        _dgrad.fused = bn is not None
        if bn is not None:
            ws, bx, fc, mk = bn[:4]
            fin = bn[4] if len(bn) > 4 else None
            return H.conv(dy, wt, 1, ws, out, -1, bx, fc, mk, acc_mask=out_mask, acc_even=acc_even, **_kw(fin=fin))
        return H.conv(dy, wt, 1, None, out, acc_mask=out_mask, acc_even=acc_even)
    assert out_mask is None and not acc_even
    ks = w.shape[2]
    if stride == 2 and out is None and _even_s2(x, dy, ks):
        wt = wt if wt is not None else H.conv_flip_weight(w)
        if ks == 3 and bn is not None:
            ws, bx, fc, mk = bn[:4]
            fin = bn[4] if len(bn) > 4 else None
            _dgrad.fused = True
            return H.conv_dgrad_s2(dy, wt, 3, ws, bx, fc, mk, **_kw(fin=fin))
        _dgrad.fused = False
        dx = H.conv_dgrad_s2(dy, wt, ks)
        if ks == 1:  # odd pixels get no gradient from a 1x1 stride-2 conv
            dx.view(dx.shape[0], dx.shape[1], dx.shape[2] // 2, 2, dx.shape[3] // 2, 2)[:, :, :, 1:, :, :].zero_()
            dx.view(dx.shape[0], dx.shape[1], dx.shape[2] // 2, 2, dx.shape[3] // 2, 2)[:, :, :, 0, :, 1:].zero_()
        return dx
    _dgrad.fused = False
    dx = torch.ops.aten.convolution_backward(dy, x, w, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1,
                                             [True, False, False])[0]
    if out is not None:
        out.add_(dx)
        return out
    return _cl(dx)


def _even_s2(x, dy, ks) -> bool:
    """Stride-2 data gradient on the parity-phase kernels: the input is exactly twice the output."""
    return (x.shape[2] == 2 * dy.shape[2] and x.shape[3] == 2 * dy.shape[3] and ks in (1, 3)
            and hip().conv_supported(dy.shape[1], x.shape[1], ks, 1))


def _dgrad_s2_even(dy, x, w, flipped=None):
    """Stride-2 1x1 data gradient written at the even pixels only (the caller completes the
    tensor with a stride-1 data gradient ``_dgrad(..., out=dx, acc_even=True)``)."""
    H = hip()
    wt = flipped if flipped is not None else H.conv_flip_weight(w)
    return H.conv_dgrad_s2(dy, wt, 1)


class _TailSlot:
    """Link from a block's output to the NEXT block's backward: that block's conv1 data
    gradient IS the gradient of this output, so its epilogue can also produce this block's
    BN3 backward sums (sum dz, sum dz*y3 under the 1-bit ReLU mask).  ``dx_ptr`` lets this
    block's backward check that the gradient it receives is exactly that tensor (no other
    consumer added to it); otherwise the sums are discarded and recomputed."""
    __slots__ = ("ws", "y3", "mask", "ready", "dx_ptr", "fin", "pre")

    def __init__(self, ws, y3, mask, fin=None, pre=None):
        self.ws, self.y3, self.mask = ws, y3, mask
        self.ready = False
        self.dx_ptr = 0
        self.fin, self.pre = fin, pre  # in-launch finalize of this block's BN3 backward (see _fin_bwd)


class _Spec:
    """Static description of one block (modules for running stats / workspaces)."""
    __slots__ = ("bns", "stride", "ds", "dtypes", "direct", "wsrc")

    def __init__(self, bns, stride, ds):
        self.bns, self.stride, self.ds = bns, stride, ds
        self.dtypes = None
        self.direct = None
        self.wsrc = None  # per conv: (flip cache, param index) for bf16 shadow weights, else None


class _BottleneckFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec: _Spec, x, *params):
        H = hip()
        dev = x.device
        ws = [p for p in params]
        ws_bf = [w if w.dtype == torch.bfloat16 else w.to(torch.bfloat16) for w in ws[0::3]]
        ws_bf = [_cl(w) for w in ws_bf]
        gam, bet = ws[1::3], ws[2::3]
        s = spec.stride
        outs = []

        pres = [None] * len(spec.bns)

        def bn(i, y, res, relu, res_coef=None, apply=True):
            m = spec.bns[i]
            return H.bn_forward(y, res, gam[i], bet[i], m.running_mean, m.running_var, m.momentum, m.eps, True, relu,
                                m.num_batches_tracked, _sums(m, dev), res_coef=res_coef, apply=apply, **_kw(pre=pres[i]))

        gens = [None] * len(spec.bns)

        def conv(i, inp, w_, st_):
            # the conv's statistics epilogue also finalizes BN i in its own launch (_fin_fwd)
            oh = (inp.shape[2] - 1) // st_ + 1
            ow = (inp.shape[3] - 1) // st_ + 1
            kw, pres[i], gens[i] = _fin_fwd(spec.bns[i], gam[i], bet[i], inp.shape[0] * oh * ow, dev)
            return H.conv(inp, w_, st_, _sums(spec.bns[i], dev), **kw)

        y1 = conv(0, x, ws_bf[0], 1)
        z1, m1, i1, c1, _ = bn(0, y1, None, True)
        y2 = conv(1, z1, ws_bf[1], s)
        z2, m2, i2, c2, _ = bn(1, y2, None, True)
        y3 = conv(2, z2, ws_bf[2], 1)
        if spec.ds:
            # the downsample BN is folded into the tail's residual read (coefficients only here):
            # out = relu(bn3(y3) + bn_d(yd)) without materialising bn_d(yd)
            yd = conv(3, x, ws_bf[3], s)
            _, md, idd, cd, _ = bn(3, yd, None, False, apply=False)
            out, m3, i3, c3, mask3 = bn(2, y3, yd, True, res_coef=cd)
        else:
            yd = md = idd = cd = None
            out, m3, i3, c3, mask3 = bn(2, y3, x, True)
        # cross-block BN3 backward fusion: the previous block's tail (if x is its output)
        ctx.prev = getattr(x, "_kf_tail", None)
        fin3, pre3 = _fin_bwd(spec.bns[2], gens[2])
        ctx.tail = _TailSlot(_sums(spec.bns[2], dev), y3, mask3, fin3, pre3)
        ctx.gens = gens
        ctx.spec = spec
        ctx.wdtypes = [w.dtype for w in ws[0::3]]
        ctx.save_for_backward(x, y1, z1, y2, z2, y3, yd, *ws_bf, *gam, m1, i1, c1, m2, i2, c2, m3, i3, c3, mask3,
                              md, idd, cd)
        return out

    @staticmethod
    def backward(ctx, dout):
        H = hip()
        spec = ctx.spec
        nb = 4 if spec.ds else 3
        t = list(ctx.saved_tensors)
        x, y1, z1, y2, z2, y3, yd = t[:7]
        w = t[7:7 + nb]
        g = t[7 + nb:7 + 2 * nb]
        (m1, i1, c1, m2, i2, c2, m3, i3, c3, mask3, md, idd, cd) = t[7 + 2 * nb:]
        s = spec.stride
        dout = _cl(dout)
        fl = [None] * nb
        if spec.wsrc is not None:
            for k, src in enumerate(spec.wsrc):
                if src is not None:
                    fl[k] = src[0].get(src[1])
        dbn = [None] * nb  # (dgamma, dbeta)
        dw = [None] * nb
        # (the conv weight gradients on a side stream measured slower twice: eager 1.2 % in r3, as
        # hipGraph branches 20.44 -> 21.05 ms/step in r6t4 -- removed, round 6)
        wgrad = _wgrad

        ws = [_sums(b, dout.device) for b in spec.bns]
        tail = ctx.tail
        use3 = tail.ready and dout.data_ptr() == tail.dx_ptr
        if tail.ready and not use3:
            tail.ws.zero_()  # sums of a gradient that is not the one we got: discard
            tail.pre = None  # (its in-launch finalize re-zeroed the slots; the coefficients are stale)
        pre3 = tail.pre if use3 else None
        tail.ready, tail.y3, tail.mask, tail.fin, tail.pre = False, None, None, None, None
        # identity block whose output gradient is our own buffer (the next block's conv1 data
        # gradient): the residual gradient dout * relu' is never written -- conv1's data
        # gradient below accumulates into dout in place, masking it on the fly
        in_place = use3 and not spec.ds
        # downsample block: the residual gradient also feeds the downsample BN, whose backward
        # sums are accumulated by this same pass (that BN then skips its reduce)
        dy3, didt, dg3, db3 = H.bn_backward(dout, y3, m3, i3, g[2], c3, mask3, True, True, not in_place,
                                            ws[2] if use3 else None, dres_x=yd if spec.ds else None,
                                            dres_sums=ws[3] if spec.ds else None, **_kw(pre=pre3))
        dbn[2] = (dg3, db3)
        if _CAPTURE is not None:
            _capture(spec.bns[2], "mask", dout, y3, m3, i3, mask3, dg3, db3)
        fin2, pre2 = _fin_bwd(spec.bns[1], ctx.gens[1])
        dz2 = _dgrad(dy3, z2, w[2], 1, 0, flipped=fl[2], bn=(ws[1], y2, c2, None, fin2))
        dw[2] = wgrad(dy3, z2, w[2], 1, 0)
        dy2, _, dg2, db2 = H.bn_backward(dz2, y2, m2, i2, g[1], c2, None, True, True, False, ws[1], **_kw(pre=pre2))
        dbn[1] = (dg2, db2)
        if _CAPTURE is not None:
            _capture(spec.bns[1], "relu", dz2, y2, m2, i2, c2, dg2, db2)
        fin1, pre1 = _fin_bwd(spec.bns[0], ctx.gens[0])
        dz1 = _dgrad(dy2, z1, w[1], s, 1, flipped=fl[1], bn=(ws[0], y1, c1, None, fin1))
        fused1 = _dgrad.fused
        dw[1] = wgrad(dy2, z1, w[1], s, 1)
        dy1, _, dg1, db1 = H.bn_backward(dz1, y1, m1, i1, g[0], c1, None, True, True, False,
                                         ws[0] if fused1 else None, **_kw(pre=pre1 if fused1 else None))
        dbn[0] = (dg1, db1)
        if _CAPTURE is not None:
            _capture(spec.bns[0], "relu", dz1, y1, m1, i1, c1, dg1, db1)
        acc_even = False
        if spec.ds:
            dyd, _, dgd, dbd = H.bn_backward(didt, yd, md, idd, g[3], cd, None, False, True, False, ws[3])
            dbn[3] = (dgd, dbd)
            if _CAPTURE is not None:
                _capture(spec.bns[3], "plain", didt, yd, md, idd, None, dgd, dbd)
            if s == 2 and _even_s2(x, dyd, 1):
                # even pixels only; conv1's data gradient below stores the odd ones
                dx = _dgrad_s2_even(dyd, x, w[3], flipped=fl[3])
                acc_even = True
            else:
                dx = _dgrad(dyd, x, w[3], s, 0, flipped=fl[3])
            dw[3] = wgrad(dyd, x, w[3], s, 0)
        elif in_place:
            dx = dout  # raw output gradient; masked by mask3 inside conv1's data-gradient epilogue
        else:
            dx = didt  # the identity gradient: conv1's data gradient is accumulated into it
        om = mask3 if in_place else None
        prev = ctx.prev
        if prev is not None and prev.y3 is not None and prev.y3.shape == dx.shape:
            # conv1's data gradient completes the gradient of the previous block's output:
            # its epilogue also accumulates that block's BN3 backward sums
            dx = _dgrad(dy1, x, w[0], 1, 0, out=dx, flipped=fl[0], bn=(prev.ws, prev.y3, None, prev.mask, prev.fin),
                        out_mask=om, acc_even=acc_even)
            prev.ready, prev.dx_ptr = True, dx.data_ptr()
        else:
            dx = _dgrad(dy1, x, w[0], 1, 0, out=dx, flipped=fl[0], out_mask=om, acc_even=acc_even)
        dw[0] = wgrad(dy1, x, w[0], 1, 0)
        grads: List[Optional[torch.Tensor]] = []
        for i in range(nb):
            gw = dw[i]
            if gw.dtype != ctx.wdtypes[i]:
                gw = gw.to(ctx.wdtypes[i])
            dgm, dbt = dbn[i]
            tgt = spec.direct[i] if spec.direct is not None else None
            if tgt is not None:
                deliver(tgt[0], dgm)
                deliver(tgt[1], dbt)
                dgm = dbt = None
            grads += [gw, dgm, dbt]
        return (None, dx, *grads)


def eligible(block, x: torch.Tensor) -> bool:
    if not (_ENABLED and block.training and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    if not x.is_contiguous(memory_format=torch.channels_last) or not hip_available():
        return False
    # every activation of the block (at most N*H*W * its widest channel count) must stay below
    # the conv kernels' 2 GiB buffer-resource range; larger batches take the layered path
    widest = max(block.conv1.in_channels, block.conv3.out_channels, block.conv1.out_channels)
    if not buf_ok(x.numel() // x.shape[1] * widest):
        return False
    H = hip()
    convs = [block.conv1, block.conv2, block.conv3] + ([block.downsample[0]] if block.downsample is not None else [])
    for c in convs:
        if c.bias is not None or c.groups != 1 or c.dilation != (1, 1):
            return False
        if not H.conv_supported(c.in_channels, c.out_channels, c.kernel_size[0], c.stride[0]):
            return False
    if block.conv2.kernel_size != (3, 3) or block.conv2.padding != (1, 1):
        return False
    if block.downsample is not None and block.downsample[0].kernel_size != (1, 1):
        return False
    bns = [block.bn1, block.bn2, block.bn3] + ([block.downsample[1]] if block.downsample is not None else [])
    for b in bns:
        if not (b.track_running_stats and b.momentum is not None and b.affine):
            return False
        if not H.bn_supported_channels(b.num_features):
            return False
    return True


def bottleneck_forward(block, x: torch.Tensor) -> torch.Tensor:
    """Training forward of a ResNet ``Bottleneck`` (fused tail) as one autograd node."""
    ds = block.downsample is not None
    convs = [block.conv1, block.conv2, block.conv3] + ([block.downsample[0]] if ds else [])
    bns = [block.bn1, block.bn2, block.bn3] + ([block.downsample[1]] if ds else [])
    spec = getattr(block, "_kf_spec", None)
    if spec is None or spec.ds != ds:
        spec = _Spec(bns, block.conv2.stride[0], ds)
        block._kf_spec = spec
    params = []
    direct = []
    wsrc = []
    for c, b in zip(convs, bns):
        w = shadow(c.weight)
        params += [w, b.weight, b.bias]
        tw, tb = direct_target(b.weight), direct_target(b.bias)
        direct.append((tw, tb) if tw is not None and tb is not None else None)
        tc = direct_target(c.weight)
        if tc is not None and w is not c.weight and w.dtype == torch.bfloat16:
            fc = _flip_cache(tc[0])
            fc.register(tc[1], w)
            wsrc.append((fc, tc[1]))
        else:
            wsrc.append(None)
    spec.direct = direct if any(d is not None for d in direct) else None
    spec.wsrc = wsrc if any(v is not None for v in wsrc) else None
    out = _BottleneckFn.apply(spec, x, *params)
    if out.grad_fn is not None:
        out._kf_tail = out.grad_fn.tail  # the next block's backward fills our BN3 sums
    return out
