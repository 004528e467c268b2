"""Inception-v3 (the reference's third headline model),
299x299 input, no auxiliary head (training throughput benchmark form)."""
import torch
import torch.nn as nn
import torch.nn.functional as F


# set by inception_v3(fused_bn=True) while the model is being built
_FUSED_BN = [False]


class BasicConv2d(nn.Module):
    """conv -> BN -> ReLU.  With ``fused_bn`` the BN+ReLU is the HIP ``BatchNormAct2d``
    (same parameters and state_dict keys), which runs its kernels for the channel counts
    it supports (64, 128, ...) and the torch composition for the others (80, 192, ...)."""

    def __init__(self, cin, cout, pool_after_conv: bool = False, **kw):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, bias=False, **kw)
        # branch-pool form: conv1x1(avg_pool3x3(x)) == avg_pool3x3(conv1x1(x)) exactly (both
        # linear, no conv bias, count_include_pad pads with zeros either way); pooling the
        # cout-channel conv output instead of the cin-channel input moves 4-10x fewer bytes
        self.pool_after_conv = pool_after_conv
        self.fused = _FUSED_BN[0]
        if self.fused:
            from ..ops.fused_bn import BatchNormAct2d

            self.bn = BatchNormAct2d(cout, relu=True, eps=0.001)
        else:
            self.bn = nn.BatchNorm2d(cout, eps=0.001)

    def forward(self, x, link: bool = False, defer: bool = False):
        """``link``: this output's only consumer is another BasicConv2d's (or a sibling group's)
        stride-1 conv -- its data-gradient epilogue then produces this BN's backward sums.
        ``defer`` (fused training path): return a :class:`~kungfu_amd.ops.fused_bn.Deferred` BN+ReLU
        (conv output + BN) for a concatenation to apply straight into its channel slice."""
        defer = defer and self.fused and self.training and self.bn.track_running_stats
        if self.fused and not self.pool_after_conv and self.training and self.bn.track_running_stats:
            # MFMA conv whose epilogue accumulates the BN batch statistics: the BN skips its
            # statistics pass (ops/conv.py conv2d_stats; None if the shape is not on the kernel)
            from ..ops.conv import conv2d_stats
            from ..parallel.mixed import shadow

            c = self.conv
            w = shadow(c.weight)
            from ..ops import stem as stem_ops

            if stem_ops.stem3_eligible(c, x):
                # the 3-channel image stem (Conv2d_1a) on stem3.hip: MFMA conv + BN-statistics epilogue
                # straight from the f32 image (no cast pass, no MIOpen, no BN statistics pass)
                ws = self.bn.stats_workspace(x.device)
                y = stem_ops.stem3_conv(c, x, w, ws)
                if defer:
                    from ..ops.fused_bn import Deferred

                    return Deferred(y, self.bn, ws)
                return self.bn(y, sums=ws, link=link)
            if w.dtype == torch.bfloat16 and x.dtype == torch.bfloat16:
                ws = self.bn.stats_workspace(x.device)
                y = conv2d_stats(x, w, c.stride, c.padding, ws, master=c.weight)
                if y is not None:
                    if defer:
                        from ..ops.fused_bn import Deferred

                        return Deferred(y, self.bn, ws)
                    return self.bn(y, sums=ws, link=link)
        y = self.conv(x)
        if self.pool_after_conv:
            if self.fused:  # HIP 3x3/s1/p1 stencil (forward and backward)
                from ..ops.pool import avg_pool3x3s1

                y = avg_pool3x3s1(y)
            else:
                y = F.avg_pool2d(y, 3, 1, 1)
        if defer:
            from ..ops.fused_bn import Deferred

            return Deferred(y, self.bn)
        if self.fused:
            return self.bn(y, link=link)
        return F.relu(self.bn(y), inplace=True)


def _chain(x, mods, link_last: bool = False, defer_last: bool = True):
    """``mods[-1](...mods[0](x))`` for BasicConv2d modules: every output but the last has the next
    conv as its only consumer (BN-sums link, see BasicConv2d.forward).  ``defer_last``: the last
    BN+ReLU is left to the block's concatenation (:func:`~kungfu_amd.ops.fused_bn.bn_relu_concat`)."""
    for i, m in enumerate(mods):
        nxt = mods[i + 1] if i + 1 < len(mods) else None
        # stride-1 consumers, and 3x3 stride-2 ones (parity-phase data gradient), produce the BN sums
        lk = link_last if nxt is None else (nxt.conv.stride in (1, (1, 1)) or nxt.conv.kernel_size == (3, 3))
        x = m(x, link=lk, defer=defer_last and nxt is None)
    return x


def _cat(pieces):
    """An Inception block's channel concatenation: the deferred branch BN+ReLUs write straight into
    their slices (fused model), else torch.cat."""
    from ..ops.fused_bn import bn_relu_concat

    return bn_relu_concat(pieces)


def _heads(x, mods, links=None, defer=None):
    """``[m(x) for m in mods]`` for BasicConv2d modules that all read ``x`` (an Inception block's
    branch heads).  Fused training path: their convolutions are ONE autograd node on the MFMA
    kernel (``ops.conv.sibling_convs``: the branch gradients of x are accumulated by the conv
    epilogue instead of autograd adds), each conv's epilogue producing its BN's statistics
    (the pool branch pools the conv output first, so its BN computes its own).  ``defer[i]``: head i's
    BN+ReLU is left to the block's concatenation (a Deferred is returned)."""
    m0 = mods[0]
    if (len(mods) > 1 and m0.fused and m0.training and x.dtype == torch.bfloat16
            and all(m.bn.track_running_stats for m in mods)):
        from ..ops.conv import sibling_convs

        st = [None if m.pool_after_conv else m.bn.stats_workspace(x.device) for m in mods]
        ys = sibling_convs(x, [m.conv for m in mods], st)
        if ys is not None:
            from ..ops.pool import avg_pool3x3s1

            from ..ops.fused_bn import Deferred

            lks = links or [False] * len(mods)
            dfs = defer or [False] * len(mods)
            out = []
            for m, y, s, lk, df in zip(mods, ys, st, lks, dfs):
                if m.pool_after_conv:
                    y = avg_pool3x3s1(y)
                out.append(Deferred(y, m.bn, s) if df else m.bn(y, sums=s, link=lk))
            return out
    return [m(x, link=lk, defer=df) for m, lk, df in zip(mods, links or [False] * len(mods),
                                                           defer or [False] * len(mods))]


def _pool_module():
    """The stem's MaxPool2d(3, 2): HIP kernels (byte argmax, gather backward) in the fused model."""
    if _FUSED_BN[0]:
        from ..ops.pool import MaxPool3x3s2

        return MaxPool3x3s2()
    return nn.MaxPool2d(3, 2)


def _max_pool3s2(x, fused: bool):
    """F.max_pool2d(x, 3, 2); in the fused model on the HIP kernels when the input qualifies."""
    if not fused:
        return F.max_pool2d(x, 3, 2)
    from ..ops.pool import max_pool3x3s2

    return max_pool3x3s2(x)


def _branch_pool(cin, cout):
    """BasicConv2d applied to avg_pool2d(x, 3, 1, 1) (the Inception pool branch)."""
    assert cout <= cin
    return BasicConv2d(cin, cout, pool_after_conv=True, kernel_size=1)


class InceptionA(nn.Module):
    def __init__(self, cin, pool_features):
        super().__init__()
        self.b1 = BasicConv2d(cin, 64, kernel_size=1)
        self.b5 = nn.Sequential(BasicConv2d(cin, 48, kernel_size=1), BasicConv2d(48, 64, kernel_size=5, padding=2))
        self.b3 = nn.Sequential(BasicConv2d(cin, 64, kernel_size=1), BasicConv2d(64, 96, kernel_size=3, padding=1),
                                BasicConv2d(96, 96, kernel_size=3, padding=1))
        self.bp = _branch_pool(cin, pool_features)

    def forward(self, x):
        o1, t5, t3, op = _heads(x, [self.b1, self.b5[0], self.b3[0], self.bp], [False, True, True, False],
                                [True, False, False, True])
        return _cat([o1, self.b5[1](t5, defer=True), _chain(t3, list(self.b3[1:])), op])


class InceptionB(nn.Module):
    def __init__(self, cin):
        super().__init__()
        self.fused = _FUSED_BN[0]
        self.b3 = BasicConv2d(cin, 384, kernel_size=3, stride=2)
        self.bd = nn.Sequential(BasicConv2d(cin, 64, kernel_size=1), BasicConv2d(64, 96, kernel_size=3, padding=1),
                                BasicConv2d(96, 96, kernel_size=3, stride=2))

    def forward(self, x):
        return _cat([self.b3(x, defer=True), _chain(x, list(self.bd)), _max_pool3s2(x, self.fused)])


class InceptionC(nn.Module):
    def __init__(self, cin, c7):
        super().__init__()
        self.b1 = BasicConv2d(cin, 192, kernel_size=1)
        self.b7 = nn.Sequential(BasicConv2d(cin, c7, kernel_size=1),
                                BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3)),
                                BasicConv2d(c7, 192, kernel_size=(7, 1), padding=(3, 0)))
        self.bd = nn.Sequential(BasicConv2d(cin, c7, kernel_size=1),
                                BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0)),
                                BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3)),
                                BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0)),
                                BasicConv2d(c7, 192, kernel_size=(1, 7), padding=(0, 3)))
        self.bp = _branch_pool(cin, 192)

    def forward(self, x):
        o1, t7, td, op = _heads(x, [self.b1, self.b7[0], self.bd[0], self.bp], [False, True, True, False],
                                [True, False, False, True])
        return _cat([o1, _chain(t7, list(self.b7[1:])), _chain(td, list(self.bd[1:])), op])


class InceptionD(nn.Module):
    def __init__(self, cin):
        super().__init__()
        self.fused = _FUSED_BN[0]
        self.b3 = nn.Sequential(BasicConv2d(cin, 192, kernel_size=1), BasicConv2d(192, 320, kernel_size=3, stride=2))
        self.b7 = nn.Sequential(BasicConv2d(cin, 192, kernel_size=1),
                                BasicConv2d(192, 192, kernel_size=(1, 7), padding=(0, 3)),
                                BasicConv2d(192, 192, kernel_size=(7, 1), padding=(3, 0)),
                                BasicConv2d(192, 192, kernel_size=3, stride=2))

    def forward(self, x):
        t3, t7 = _heads(x, [self.b3[0], self.b7[0]], [False, True])
        return _cat([self.b3[1](t3, defer=True), _chain(t7, list(self.b7[1:])), _max_pool3s2(x, self.fused)])


class InceptionE(nn.Module):
    def __init__(self, cin):
        super().__init__()
        self.b1 = BasicConv2d(cin, 320, kernel_size=1)
        self.b3_1 = BasicConv2d(cin, 384, kernel_size=1)
        self.b3_2a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.b3_2b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.bd_1 = BasicConv2d(cin, 448, kernel_size=1)
        self.bd_2 = BasicConv2d(448, 384, kernel_size=3, padding=1)
        self.bd_3a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.bd_3b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.bp = _branch_pool(cin, 192)

    def forward(self, x):
        # b3 / bd feed one sibling group each (a single autograd consumer): linked
        o1, b3, bd, op = _heads(x, [self.b1, self.b3_1, self.bd_1, self.bp], [False, True, True, False],
                                [True, False, False, True])
        bd = self.bd_2(bd, link=True)
        both = [True, True]
        return _cat([o1] + _heads(b3, [self.b3_2a, self.b3_2b], defer=both) + _heads(bd, [self.bd_3a, self.bd_3b], defer=both)
                    + [op])


class InceptionV3(nn.Module):
    def __init__(self, num_classes: int = 1000):
        super().__init__()
        pool = _pool_module
        self.stem = nn.Sequential(
            BasicConv2d(3, 32, kernel_size=3, stride=2), BasicConv2d(32, 32, kernel_size=3),
            BasicConv2d(32, 64, kernel_size=3, padding=1), pool(),
            BasicConv2d(64, 80, kernel_size=1), BasicConv2d(80, 192, kernel_size=3), pool())
        self.blocks = nn.Sequential(
            InceptionA(192, 32), InceptionA(256, 64), InceptionA(288, 64), InceptionB(288),
            InceptionC(768, 128), InceptionC(768, 160), InceptionC(768, 160), InceptionC(768, 192),
            InceptionD(768), InceptionE(1280), InceptionE(2048))
        self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        st = self.stem
        # conv -> conv links inside the stem (the pools consume stem[2] / stem[5])
        x = st[3](_chain(x, [st[0], st[1], st[2]], defer_last=False))
        x = self.blocks(st[6](_chain(x, [st[4], st[5]], defer_last=False)))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def inception_v3(fused_bn: bool = False, **kw):
    _FUSED_BN[0] = bool(fused_bn)
    try:
        return InceptionV3(**kw)
    finally:
        _FUSED_BN[0] = False
