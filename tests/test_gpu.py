"""GPU tests (run with -m gpu on an MI355X).  Every numerics test compares a
HIP kernel with a float32 PyTorch reference of the same op."""
import os
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

from conftest import ROOT, kungfu_run, worker

pytestmark = pytest.mark.gpu

needs_gpu = pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")


@pytest.fixture(scope="module")
def H():
    from kungfu_amd._lib import hip

    return hip()


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()


@needs_gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n", [1, 1000, (1 << 20) + 3])
def test_reduce_kernel(H, dtype, n):
    x = torch.randn(n, device="cuda").to(dtype)
    y = torch.randn(n, device="cuda").to(dtype)
    z = torch.empty_like(x)
    for op, f in [(0, torch.add), (1, torch.minimum), (2, torch.maximum), (3, torch.mul)]:
        H.reduce(z, x, y, op)
        torch.testing.assert_close(z.float(), f(x.float(), y.float()).to(dtype).float(), rtol=0, atol=0)


@needs_gpu
@pytest.mark.parametrize("nesterov", [False, True])
def test_fused_sgd_matches_torch(H, nesterov):
    from kungfu_amd.optimizers import FusedSGD
    from kungfu_amd.parallel.flat import FlatParamSpace

    torch.manual_seed(0)
    m1 = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 5)).cuda()
    m2 = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 5)).cuda()
    m2.load_state_dict(m1.state_dict())
    m2 = m2.to(memory_format=torch.channels_last)
    o1 = torch.optim.SGD(m1.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=nesterov)
    o2 = FusedSGD(FlatParamSpace(m2.parameters()), lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=nesterov)
    for _ in range(3):
        x = torch.randn(4, 3, 8, 8, device="cuda")
        for m, o in [(m1, o1), (m2, o2)]:
            o.zero_grad()
            m(x).square().mean().backward()
            o.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)  # NCHW vs NHWC conv algos round differently


@needs_gpu
def test_fused_adam_matches_torch(H):
    from kungfu_amd.optimizers import FusedAdam
    from kungfu_amd.parallel.flat import FlatParamSpace

    torch.manual_seed(0)
    m1 = torch.nn.Linear(37, 11).cuda()
    m2 = torch.nn.Linear(37, 11).cuda()
    m2.load_state_dict(m1.state_dict())
    o1 = torch.optim.AdamW(m1.parameters(), lr=1e-2, weight_decay=0.01)
    o2 = FusedAdam(FlatParamSpace(m2.parameters()), lr=1e-2, weight_decay=0.01, adamw=True)
    for _ in range(4):
        x = torch.randn(8, 37, device="cuda")
        for m, o in [(m1, o1), (m2, o2)]:
            o.zero_grad()
            m(x).square().sum().backward()
            o.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


@needs_gpu
def test_norms_variance_axpby(H):
    n = (1 << 21) + 5
    a, b = torch.randn(n, device="cuda"), torch.randn(n, device="cuda")
    s = H.sumsq2(a, b)
    ref = torch.stack([a.double().pow(2).sum(), b.double().pow(2).sum()])
    assert _rel(s.double(), ref) < 1e-5
    sb = H.sumsq2(a.bfloat16(), None)
    assert abs(sb[0].item() / a.bfloat16().double().pow(2).sum().item() - 1) < 1e-5
    s1 = torch.randn(n, device="cuda")
    s2 = s1 * s1 + torch.rand(n, device="cuda")
    v = H.variance(s1, s2, 0.25)
    vr = (s2.double() * 0.25 - (s1.double() * 0.25) ** 2).abs().sum()
    assert abs(v.item() / vr.item() - 1) < 1e-4
    offs = torch.tensor([0, 10, 1000, 100000, n], dtype=torch.int64, device="cuda")
    sv = H.seg_variance(s1, s2, offs, 0.5).item()
    d = s2.double() * 0.5 - (s1.double() * 0.5) ** 2
    svr = sum(d[offs[i]:offs[i + 1]].norm().item() for i in range(4))
    assert abs(sv / svr - 1) < 1e-4
    y, x, z = torch.randn(n, device="cuda"), torch.randn(n, device="cuda"), torch.empty(n, device="cuda")
    y0 = y.clone()
    H.axpby(y, x, z, 0.9, 0.1)
    torch.testing.assert_close(y, 0.9 * y0 + 0.1 * x)
    torch.testing.assert_close(z, y)


@needs_gpu
def test_gns_update_device(H):
    st = torch.zeros(4, device="cuda")
    sq_small, sq_big = torch.tensor([4.0], device="cuda"), torch.tensor([1.0], device="cuda")
    H.gns_update(sq_small, sq_big, 32.0, 256.0, 0.6, st)
    G = (256 * 1.0 - 32 * 4.0) / (256 - 32)
    S = (4.0 - 1.0) / (1 / 32 - 1 / 256)
    assert abs(st[2].item() - S / G) / (S / G) < 1e-5 and st[3].item() == 1


@needs_gpu
def test_pack_unpack(H):
    from kungfu_amd.ops import defuse, fuse

    ts = [torch.randn(k, device="cuda") for k in [3, 100, 4097, 1, 65536]]
    flat = fuse(ts, scale=2.0)
    torch.testing.assert_close(flat, torch.cat(ts) * 2)
    outs = [torch.empty_like(t) for t in ts]
    defuse(flat, outs, scale=0.5)
    for t, o in zip(ts, outs):
        torch.testing.assert_close(o, t)
    flat16 = fuse(ts, dtype=torch.bfloat16)
    torch.testing.assert_close(flat16.float(), torch.cat(ts).bfloat16().float())


@needs_gpu
@pytest.mark.parametrize("shape", [(4, 64, 16, 16), (8, 256, 14, 14), (2, 2048, 7, 7), (3, 128, 5, 9),
                                   # Inception-v3 channel counts (C/8 not a power of two)
                                   (4, 80, 17, 17), (4, 192, 9, 9), (2, 448, 8, 8), (3, 32, 13, 11),
                                   (2, 48, 10, 10), (2, 96, 7, 9), (2, 160, 6, 6), (2, 320, 5, 5),
                                   (2, 384, 5, 7)])
@pytest.mark.parametrize("relu,with_res", [(True, False), (True, True), (False, False)])
def test_fused_bn(shape, relu, with_res):
    import torch.nn.functional as F

    from kungfu_amd.ops.fused_bn import bn_act

    torch.manual_seed(1)
    N, C, Hh, W = shape
    x = (torch.randn(shape, device="cuda") * 2 + 0.5).bfloat16().to(memory_format=torch.channels_last)
    res = torch.randn_like(x) if with_res else None
    w, b = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    rm2, rv2 = rm.clone(), rv.clone()
    xr = x.detach().float().requires_grad_()
    wr, br = w.clone().requires_grad_(), b.clone().requires_grad_()
    resr = res.detach().float().requires_grad_() if with_res else None
    yr = F.batch_norm(xr, rm2, rv2, wr, br, True, 0.1, 1e-5)
    if with_res:
        yr = yr + resr
    if relu:
        yr = F.relu(yr)
    xa, wa, ba = x.detach().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    resa = res.detach().requires_grad_() if with_res else None
    ya = bn_act(xa, wa, ba, rm, rv, True, 0.1, 1e-5, relu=relu, res=resa)
    g = torch.randn_like(yr)
    yr.backward(g)
    ya.backward(g.bfloat16().to(memory_format=torch.channels_last))
    for a, r in [(ya, yr), (xa.grad, xr.grad), (wa.grad, wr.grad), (ba.grad, br.grad), (rm, rm2), (rv, rv2)]:
        assert _rel(a, r) < 3e-2
    if with_res:
        assert _rel(resa.grad, resr.grad) < 3e-2


@needs_gpu
@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (2, 64, 15, 17), (3, 128, 8, 8)])
def test_fused_bn_relu_maxpool(shape):
    """Stem BN+ReLU+MaxPool(3,2,1) (one forward pass, gather backward) vs f32 torch."""
    import torch.nn.functional as F

    from kungfu_amd.ops.fused_bn import BatchNormAct2d, bn_act_pool

    torch.manual_seed(2)
    N, C, Hh, W = shape
    x = (torch.randn(shape, device="cuda") * 2 + 0.3).bfloat16().to(memory_format=torch.channels_last)
    w, b = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    w[::7] *= -1  # negative gamma: max must be taken after the affine map
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    rm2, rv2 = rm.clone(), rv.clone()
    xr = x.detach().float().requires_grad_()
    wr, br = w.clone().requires_grad_(), b.clone().requires_grad_()
    yr = F.max_pool2d(F.relu(F.batch_norm(xr, rm2, rv2, wr, br, True, 0.1, 1e-5)), 3, 2, 1)
    xa, wa, ba = x.detach().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    nbt = torch.zeros((), dtype=torch.long, device="cuda")
    ya = bn_act_pool(xa, wa, ba, rm, rv, True, 0.1, 1e-5, num_batches_tracked=nbt)
    assert ya.shape == yr.shape and ya.is_contiguous(memory_format=torch.channels_last)
    g = torch.randn_like(yr)
    yr.backward(g)
    ya.backward(g.bfloat16().to(memory_format=torch.channels_last))
    for a, r in [(ya, yr), (xa.grad, xr.grad), (wa.grad, wr.grad), (ba.grad, br.grad), (rm, rm2), (rv, rv2)]:
        assert _rel(a, r) < 3e-2
    assert int(nbt) == 1
    m = BatchNormAct2d(C).cuda().eval()
    torch.testing.assert_close(m.forward_pool(x).float(), F.max_pool2d(m(x), 3, 2, 1).float())


@needs_gpu
def test_fused_bn_num_batches_tracked():
    from kungfu_amd.ops.fused_bn import BatchNormAct2d, BatchNormAddAct2d

    x = torch.randn(2, 64, 8, 8, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    m1, m2 = BatchNormAct2d(64).cuda(), BatchNormAddAct2d(64).cuda()
    for _ in range(3):
        m1(x)
        m2(x, x)
    assert int(m1.num_batches_tracked) == 3 and int(m2.num_batches_tracked) == 3


@needs_gpu
def test_rccl_single_rank_and_ops():
    import kungfu_amd as kf
    from kungfu_amd.parallel.comm import get_device_comm

    kf.init()
    torch.cuda.set_device(0)
    t = torch.arange(1000, device="cuda", dtype=torch.float32)
    torch.testing.assert_close(kf.ops.all_reduce(t), t)
    b = kf.ops.broadcast(t)
    torch.testing.assert_close(b, t)
    g = kf.ops.all_gather(t[:10])
    assert g.shape == (1, 10)
    comm = get_device_comm()
    out = torch.empty(10, device="cuda")
    comm.reduce_scatter(t[:10].clone(), out)
    torch.cuda.synchronize()
    torch.testing.assert_close(out, t[:10])


@needs_gpu
def test_resnet_step_ssgd_fused_vs_plain():
    """One ResNet-18 step through the engine (fused BN + flat SGD) vs plain torch."""
    import torch.nn.functional as F

    import kungfu_amd as kf
    from kungfu_amd.models import resnet18

    kf.init()
    torch.manual_seed(0)
    m1 = resnet18(fused_bn=False).cuda().to(memory_format=torch.channels_last)
    m2 = resnet18(fused_bn=True).cuda().to(memory_format=torch.channels_last)
    m2.load_state_dict(m1.state_dict())
    o1 = torch.optim.SGD(m1.parameters(), lr=0.05, momentum=0.9)
    o2 = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m2.parameters(), lr=0.05, momentum=0.9))
    x = torch.randn(8, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (8,), device="cuda")
    losses = []
    for m, o in [(m1, o1), (m2, o2)]:
        ls = []
        for _ in range(3):
            o.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            o.step()
            ls.append(loss.item())
        losses.append(ls)
    # step 1 runs on identical weights; the next steps memorise the 8-image batch (loss 6.8 ->
    # ~0.3 at lr 0.05), which amplifies bf16 rounding and MIOpen's own run-to-run differences:
    # compare them loosely and require the same trajectory shape
    (a0, b0), rest = (losses[0][0], losses[1][0]), list(zip(losses[0][1:], losses[1][1:]))
    assert abs(a0 - b0) < 0.02 * abs(a0) + 0.02, losses
    for a, b in rest:
        assert abs(a - b) < 0.3 * abs(a) + 0.1, losses
    assert losses[1][-1] < losses[1][0] and losses[0][-1] < losses[0][0], losses


@needs_gpu
@pytest.mark.parametrize("shape", [(2, 64, 56, 64, 1), (2, 128, 28, 256, 2), (3, 256, 14, 128, 1), (2, 512, 7, 512, 1),
                                   (1, 64, 9, 128, 2), (2, 192, 5, 64, 1)])
def test_conv3x3_mfma_matches_torch(shape):
    """MFMA implicit-GEMM 3x3 conv (fwd, dgrad via flipped weights, wgrad) vs f32 torch."""
    import torch.nn.functional as F

    from kungfu_amd.ops.conv import _Conv3x3Fn, eligible

    torch.manual_seed(4)
    N, C, Hh, K, s = shape
    x = (torch.randn(N, C, Hh, Hh + 1, device="cuda")).bfloat16().to(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 3, 3, device="cuda") * 0.05).bfloat16().to(memory_format=torch.channels_last)
    assert eligible(x, w, s, 1, 1, 1)
    xr, wr = x.float().requires_grad_(), w.float().requires_grad_()
    yr = F.conv2d(xr, wr, stride=s, padding=1)
    xa, wa = x.detach().requires_grad_(), w.detach().requires_grad_()
    ya = _Conv3x3Fn.apply(xa, wa, s)
    assert ya.shape == yr.shape and ya.is_contiguous(memory_format=torch.channels_last)
    g = torch.randn_like(yr)
    yr.backward(g)
    ya.backward(g.bfloat16().to(memory_format=torch.channels_last))
    for a, r in [(ya, yr), (xa.grad, xr.grad), (wa.grad, wr.grad)]:
        assert ((a.float() - r).norm() / r.norm()).item() < 1e-2


@needs_gpu
def test_conv_over_2gib_falls_back():
    """the conv kernels' buffer-resource staging addresses < 2 GiB per operand; larger
    inputs must not be routed to them (they used to raise inside forward) but fall back."""
    import torch.nn.functional as F

    from kungfu_amd.ops.conv import conv3x3, eligible, rect_eligible

    x = torch.zeros(1, 64, 4096, 4100, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    assert x.numel() * 2 >= 1 << 31
    w = (torch.randn(64, 64, 3, 3, device="cuda") * 0.05).bfloat16().to(memory_format=torch.channels_last)
    assert not eligible(x, w, 1, 1, 1, 1) and not rect_eligible(x, w, 1, 1, 1, 1)
    xs = x[:, :, :64, :64]
    assert eligible(xs.contiguous(memory_format=torch.channels_last), w, 1, 1, 1, 1)
    x[:, :, 5:9, 7:11] = 1.0
    y = conv3x3(x, w, 1)
    ref = F.conv2d(x[:, :, :16, :16].float(), w.float(), padding=1)
    assert y.shape == (1, 64, 4096, 4100)
    assert ((y[:, :, 1:15, 1:15].float() - ref[:, :, 1:15, 1:15]).norm() / ref.norm()).item() < 1e-2
    del x, y
    torch.cuda.empty_cache()


@needs_gpu
@pytest.mark.parametrize("shape", [(3, 64, 9, 11, 256, 1, 1), (2, 256, 14, 14, 64, 1, 1), (2, 128, 15, 13, 512, 1, 2),
                                   (2, 64, 10, 12, 64, 3, 1), (3, 128, 9, 9, 256, 3, 2), (1, 512, 7, 7, 512, 3, 1),
                                   (2, 192, 6, 5, 128, 3, 1), (1, 64, 4, 130, 128, 3, 1), (2, 128, 5, 64, 64, 3, 1),
                                   (3, 64, 9, 28, 64, 3, 1)])
def test_conv_wgrad_mfma_matches_torch(H, shape):
    """Split-K MFMA weight gradient (every tile variant, several split counts, bf16 and
    f32-accumulate outputs) vs the f32 torch weight gradient."""
    N, C, Hh, Ww, K, ks, s = shape
    pad = (ks - 1) // 2
    torch.manual_seed(5)
    x = torch.randn(N, C, Hh, Ww, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    OH, OW = (Hh + 2 * pad - ks) // s + 1, (Ww + 2 * pad - ks) // s + 1
    dy = torch.randn(N, K, OH, OW, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_weight(x.float(), (K, C, ks, ks), dy.float(), stride=s, padding=pad)
    nrm = ref.norm()
    for v in range(H.conv_wgrad_variants()):
        try:
            H.conv_wgrad_plan(N, Hh, Ww, C, K, ks, s, v, -1)
        except Exception:
            continue  # tile does not divide the channels
        for sp in (1, 3, -1):
            got = H.conv_wgrad(dy, x, ks, s, variant=v, splits=sp)
            assert got.shape == ref.shape and got.is_contiguous(memory_format=torch.channels_last)
            assert ((got.float() - ref).norm() / nrm).item() < 1e-2, (v, sp)
    base = torch.randn(K, C, ks, ks, device="cuda").to(memory_format=torch.channels_last)
    acc = base.clone()
    H.conv_wgrad(dy, x, ks, s, out=acc, accumulate=True)
    assert ((acc - base - ref).norm() / nrm).item() < 1e-4
    from kungfu_amd.ops.conv import wgrad

    w = torch.empty(K, C, ks, ks, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    assert ((wgrad(dy, x, w, s, pad).float() - ref).norm() / nrm).item() < 1e-2


@needs_gpu
def test_conv_wgrad_batch_chunks(H, monkeypatch):
    """Weight gradients past the kernel's per-launch pixel limit (VGG-16's 224x224 layers at
    256 images) are summed over batch chunks into one f32 gradient; the limit is lowered here
    so the chunked path runs on a small shape (5 images, 2 per chunk)."""
    import kungfu_amd.ops.conv as kconv

    torch.manual_seed(6)
    N, C, Hh, Ww, K = 5, 64, 20, 20, 128
    x = torch.randn(N, C, Hh, Ww, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    dy = torch.randn(N, K, Hh, Ww, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_weight(x.float(), (K, C, 3, 3), dy.float(), stride=1, padding=1)
    w = torch.empty(K, C, 3, 3, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    monkeypatch.setattr(kconv, "_WGRAD_MAX_PIXELS", 2 * Hh * Ww + 1)
    got = kconv.wgrad(dy, x, w, 1, 1)
    assert got.dtype == torch.bfloat16 and got.shape == ref.shape
    assert ((got.float() - ref).norm() / ref.norm()).item() < 1e-2


@needs_gpu
@pytest.mark.parametrize("shape", [(2, 224, 224), (3, 37, 45), (1, 16, 9), (8, 64, 64)])
@pytest.mark.parametrize("xdtype", [torch.float32, torch.bfloat16])
def test_stem_conv_matches_torch(H, shape, xdtype):
    """MFMA stem 7x7/2 conv (pad-4 + cast, fused BN statistics) and its split-K weight
    gradient vs f32 torch."""
    import torch.nn.functional as F

    from kungfu_amd.ops.stem import stem_conv

    N, Hh, Ww = shape
    torch.manual_seed(6)
    x = torch.randn(N, 3, Hh, Ww, device="cuda").to(xdtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).bfloat16().contiguous(memory_format=torch.channels_last)
    ref = F.conv2d(x.bfloat16().float(), w.float(), stride=2, padding=3)
    stats = torch.zeros(H.conv_stat_slots * 2 * 64, dtype=torch.float64, device="cuda")
    wr = w.detach().requires_grad_()
    y = stem_conv(x, wr, stats)
    assert y.shape == ref.shape and y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    assert ((y.float() - ref).norm() / ref.norm()).item() < 1e-2
    st = stats.view(H.conv_stat_slots, 2, 64).sum(0)
    yf = y.float()
    assert torch.allclose(st[0], yf.sum((0, 2, 3)).double(), rtol=1e-3, atol=1e-2)
    assert torch.allclose(st[1], (yf * yf).sum((0, 2, 3)).double(), rtol=1e-3, atol=1e-2)
    dy = torch.randn_like(ref).bfloat16().contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    dref = torch.nn.grad.conv2d_weight(x.bfloat16().float(), w.shape, dy.float(), stride=2, padding=3)
    assert wr.grad.shape == w.shape
    assert ((wr.grad.float() - dref).norm() / dref.norm()).item() < 1e-2
    for sp in (1, 7):
        dw = H.stem_wgrad(dy, H.stem_pad4(x), sp)
        assert ((dw.float() - dref).norm() / dref.norm()).item() < 1e-2


@needs_gpu
@pytest.mark.parametrize("shape", [(4, 64, 64), (2, 37, 50), (2, 224, 224)])
def test_stem_block_fused_backward_matches_fp32(shape):
    """conv7x7/2 -> BN -> ReLU -> MaxPool as one node (the weight-gradient kernel forms the BN
    input gradient while staging: pool gather + ReLU gate + BN backward, never materialised):
    outputs, running stats and the weight / gamma / beta gradients vs an f32 torch reference, no
    worse than the layered path; gamma / beta bit-identical to the layered path (same statistics
    kernels) and the weight gradient within bf16 rounding of it (the same f32 dx expression)."""
    import torch.nn.functional as F

    from kungfu_amd.ops.fused_bn import BatchNormAct2d
    from kungfu_amd.ops.stem import stem_block, stem_conv

    N, Hh, Ww = shape
    torch.manual_seed(7)
    x = torch.randn(N, 3, Hh, Ww, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w0 = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).bfloat16().contiguous(memory_format=torch.channels_last)
    g0 = torch.rand(64, device="cuda") + 0.5
    b0 = torch.randn(64, device="cuda") * 0.1

    def make():
        bn = BatchNormAct2d(64).cuda()
        with torch.no_grad():
            bn.weight.copy_(g0)
            bn.bias.copy_(b0)
        return bn, w0.clone().requires_grad_()

    # f32 reference
    bn_r, w_r = make()
    y_r = F.max_pool2d(F.relu(F.batch_norm(F.conv2d(x.float(), w_r.float(), stride=2, padding=3), bn_r.running_mean,
                                           bn_r.running_var, bn_r.weight, bn_r.bias, True, 0.1, 1e-5)), 3, 2, 1)
    dy = torch.randn_like(y_r)
    y_r.backward(dy)
    # fused node
    from kungfu_amd.ops.fused_block import _sums

    bn_f, w_f = make()
    y_f = stem_block(x, w_f, bn_f, _sums(bn_f, x.device))
    y_f.backward(dy.bfloat16().contiguous(memory_format=torch.channels_last))
    # layered HIP path (stem conv node + BN-pool node), the statistics from the conv epilogue as well
    bn_l, w_l = make()
    s_l = _sums(bn_l, x.device)
    y_l = bn_l.forward_pool(stem_conv(x, w_l, s_l), sums=s_l)
    y_l.backward(dy.bfloat16().contiguous(memory_format=torch.channels_last))

    def r(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm()).item()

    assert r(y_f, y_r) < 2e-2
    assert r(bn_f.running_mean, bn_r.running_mean) < 1e-2 and r(bn_f.running_var, bn_r.running_var) < 1e-2
    assert int(bn_f.num_batches_tracked) == 1
    for a, b, c, what in [(w_f.grad, w_l.grad, w_r.grad, "w"), (bn_f.weight.grad, bn_l.weight.grad, bn_r.weight.grad,
                                                                  "gamma"),
                          (bn_f.bias.grad, bn_l.bias.grad, bn_r.bias.grad, "beta")]:
        ef, el = r(a, c), r(b, c)
        assert ef <= max(1.5 * el, 2e-2), (what, ef, el)
    assert torch.equal(bn_f.weight.grad, bn_l.weight.grad) and torch.equal(bn_f.bias.grad, bn_l.bias.grad)
    assert r(w_f.grad, w_l.grad) < 2e-3, r(w_f.grad, w_l.grad)


@needs_gpu
def test_grad_accumulate_multi_tensor(H):
    """_hip.grad_accumulate (flat += bf16/f32 sources, batched tables) vs torch f32."""
    torch.manual_seed(3)
    sizes = [1, 7, 64, 1000, 8192 * 3 + 5, 70000] + [33] * 60  # > one 48-entry table
    srcs, offs, off = [], [], 0
    for i, n in enumerate(sizes):
        dt = torch.bfloat16 if i % 3 else torch.float32
        srcs.append(torch.randn(n, device="cuda").to(dt))
        offs.append(off)
        off += (n + 63) // 64 * 64
    flat = torch.randn(off, device="cuda")
    ref = flat.clone()
    for s, o in zip(srcs, offs):
        ref[o:o + s.numel()] += 0.5 * s.float()
    H.grad_accumulate(flat, srcs, offs, 0.5)
    torch.testing.assert_close(flat, ref, rtol=1e-6, atol=1e-6)
    # channels_last 4-D source lands in memory order
    w = torch.randn(16, 8, 3, 3, device="cuda").to(memory_format=torch.channels_last).bfloat16()
    flat2 = torch.zeros(w.numel(), device="cuda")
    H.grad_accumulate(flat2, [w], [0])
    torch.testing.assert_close(flat2, w.permute(0, 2, 3, 1).reshape(-1).float())


@needs_gpu
def test_resnet_ssgd_bf16_shadow_matches_autocast():
    """bf16 shadow weights + direct bucket gradients vs stock autocast: same forward
    loss (to conv-algorithm rounding) and first-step gradients within the run-to-run noise of the
    stock path itself (MIOpen's weight-gradient kernels are not bitwise deterministic)."""
    import torch.nn.functional as F

    import kungfu_amd as kf
    from kungfu_amd.models import resnet18
    from kungfu_amd.parallel.mixed import enable_bf16_shadow

    kf.init()
    x = torch.randn(8, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (8,), device="cuda")

    def run(shadow):
        torch.manual_seed(0)
        m = resnet18(fused_bn=True).cuda().to(memory_format=torch.channels_last)
        o = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9))
        if shadow:
            assert enable_bf16_shadow(m, o) > 20
        ls, g0 = [], None
        for s in range(3):
            o.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            if s == 0:
                g0 = o.space.flat_grad.clone()
            o.step()
            ls.append(loss.item())
        return ls, g0

    from kungfu_amd.ops import conv as conv_ops

    old = conv_ops.set_enabled(False)  # isolate the shadow/direct-gradient path from the conv kernels
    try:
        l_a, g_a = run(False)
        l_b, g_b = run(False)
        l_s, g_s = run(True)
    finally:
        conv_ops.set_enabled(old)
    # same math; conv kernels may pick other tiles/split-K for a differently aligned weight view
    assert abs(l_s[0] - l_a[0]) <= max(2 * abs(l_b[0] - l_a[0]), 1e-3 * abs(l_a[0])), (l_a, l_b, l_s)
    def fro(a, b):
        return ((a.double() - b.double()).norm() / b.double().norm()).item()

    # MIOpen's split-K kernels are not deterministic and ResNet-18 at batch 8 amplifies it: two
    # stock runs measured 0.6 %-9 % apart (tools/diag/diag_bwd_det.py, also on the pre-r12 build)
    noise = fro(g_b, g_a)
    assert fro(g_s, g_a) < max(3 * noise, 0.12), (noise, fro(g_s, g_a))
    # later steps memorise the 8-image batch: same trajectory shape, loose values
    for a, b in zip(l_a[1:], l_s[1:]):
        assert abs(a - b) < 0.3 * abs(a) + 0.1, (l_a, l_s)
    assert l_s[-1] < l_s[0], l_s


@needs_gpu
def test_ssgd_engine_two_ranks_one_gpu_host_staged():
    """Bucketed S-SGD with 2 ranks sharing the GPU (host-staged collectives): replicas
    stay identical through broadcast + averaged gradients + auto-ordered buckets."""
    r = kungfu_run(2, [worker("ssgd_gpu.py")], timeout=400, extra=["-allow-xgmi"],
                   env={"KUNGFU_FORCE_DEVICE": "0", "KUNGFU_GPU_DATAPLANE": "host"})
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count("SSGD_GPU_OK") == 2, r.stdout[-4000:]


@needs_gpu
def test_bench_torchrun_two_ranks_one_gpu_host_staged():
    """bench.py through torch.distributed.run with 2 ranks (the driver's multi-GPU
    launch path), host-staged collectives so both ranks can share one GPU."""
    import json

    env = dict(os.environ, KUNGFU_FORCE_DEVICE="0", KUNGFU_GPU_DATAPLANE="host", PYTHONPATH=ROOT)
    from conftest import free_port_block

    port = free_port_block(2)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "16"],
                       cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["value"] > 0 and res["config"]["parallelism"] == "dp2"
    assert res["verify"]["comm_ranks"] == 2 and res["verify"]["comm_plane"] == "host", res["verify"]
    assert res["verify"]["replicas_consistent"] is True, res["verify"]


@needs_gpu
def test_pair_averaging_ipc_two_procs_one_gpu():
    """Two peers on ONE GPU: the HIP-IPC device model store (one-sided pulls)."""
    r = kungfu_run(2, [worker("pair_gpu.py")], timeout=300, extra=["-allow-xgmi"],
                   env={"KUNGFU_FORCE_DEVICE": "0", "KUNGFU_GPU_DATAPLANE": "host"})
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count("PAIR_GPU_OK") == 2, r.stdout[-4000:]


@needs_gpu
def test_pair_averaging_skewed_peers_no_torn_reads():
    """One peer sleeps between steps while the other rewrites its snapshot ring flat out:
    every accepted pull is a complete snapshot (uniform model invariant)."""
    r = kungfu_run(2, [worker("pair_stress.py")], timeout=300, extra=["-allow-xgmi"],
                   env={"KUNGFU_FORCE_DEVICE": "0", "KUNGFU_GPU_DATAPLANE": "host"})
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count("PAIR_STRESS_OK") == 2, r.stdout[-4000:]


@needs_gpu
def test_smoke_entry():
    r = subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; g.smoke()"], cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0 and "smoke ok" in r.stdout, r.stdout[-3000:]


@needs_gpu
def test_bench_json():
    import json

    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "2", "--batch", "64"], cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    for k in ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"]:
        assert k in d
    assert d["value"] > 0 and d["n_gpus"] == 1


@needs_gpu
@pytest.mark.parametrize("cin,stride,ds,nblk", [(256, 1, False, 1), (64, 1, True, 1), (256, 2, True, 1),
                                                (64, 1, True, 3), (256, 2, True, 2)])
def test_fused_bottleneck_matches_fp32(cin, stride, ds, nblk):
    """One-node bottleneck (MFMA convs with BN-statistics epilogue, in-place residual
    gradient) vs the float32 PyTorch composition of the same block; its error must be
    within the bf16 error of the per-layer bf16 path (autocast + fused BN modules)."""
    import copy

    import torch.nn as nn

    from kungfu_amd.models.resnet import Bottleneck, conv1x1
    from kungfu_amd.ops import fused_block
    from kungfu_amd.ops.fused_bn import BatchNormAct2d

    torch.manual_seed(0)
    planes = 64
    norm = lambda c, relu: BatchNormAct2d(c, relu=relu)  # noqa: E731
    down = nn.Sequential(conv1x1(cin, planes * 4, stride), BatchNormAct2d(planes * 4, relu=False)) if ds else None
    blocks = [Bottleneck(cin, planes, stride, down, norm=norm, fused_tail=True)]
    # following identity blocks: their conv1 data gradients also produce the previous
    # block's BN3 backward sums (cross-block fusion)
    blocks += [Bottleneck(planes * 4, planes, 1, None, norm=norm, fused_tail=True) for _ in range(nblk - 1)]
    blk = nn.Sequential(*blocks).cuda().to(memory_format=torch.channels_last)
    for m in blk.modules():
        if isinstance(m, nn.BatchNorm2d):
            nn.init.uniform_(m.weight, 0.5, 1.5)
            nn.init.uniform_(m.bias, -0.2, 0.2)
    ref, lay = copy.deepcopy(blk), copy.deepcopy(blk)
    x = torch.randn(4, cin, 16, 16, device="cuda").to(memory_format=torch.channels_last)
    gout = torch.randn(4, planes * 4, 16 // stride, 16 // stride, device="cuda")

    def run(mod, xin, fused, autocast):
        xin = xin.detach().clone().requires_grad_(True)
        old = fused_block.set_enabled(fused)
        try:
            if fused:
                assert fused_block.eligible(mod[0], xin)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
                out = mod(xin)
            (out.float() * gout).sum().backward()
        finally:
            fused_block.set_enabled(old)
        return out, xin.grad

    xb = x.bfloat16()
    out_f, gx_f = run(blk, xb, True, False)
    out_r, gx_r = run(ref, xb.float(), False, False)
    out_l, gx_l = run(lay, xb, False, True)

    def r(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm()).item()

    def close(a, b, c, what, floor):
        ef, el = r(a, c), r(b, c)
        assert ef <= max(1.5 * el, floor), (what, ef, el)

    close(out_f, out_l, out_r, "out", 1e-2)
    close(gx_f, gx_l, gx_r, "dx", 2e-2)
    for (n, p), (_, q), (_, l) in zip(blk.named_parameters(), ref.named_parameters(), lay.named_parameters()):
        assert p.grad is not None, n
        close(p.grad, l.grad, q.grad, n, 2e-2)
    for (n, b), (_, c) in zip(blk.named_buffers(), ref.named_buffers()):
        if b.dtype.is_floating_point:
            assert r(b, c) < 1e-2, (n, r(b, c))
        else:
            assert int(b) == int(c) == 1, n


@needs_gpu
@pytest.mark.parametrize("cin,stride,ds,nblk", [(256, 1, False, 2), (64, 1, True, 3), (256, 2, True, 2),
                                                (512, 2, True, 2)])
def test_fused_bottleneck_inlaunch_finalize_bit_identical(cin, stride, ds, nblk, monkeypatch):
    """BN finalize folded into the statistics-producing conv's own launch (the last-arriving
    workgroup folds the slots, conv.hip bn_finalize_last) vs the separate finalize launches:
    the same f64 sums in the same order through the same code, so outputs, every gradient,
    running statistics and num_batches_tracked must be bit-identical -- over two steps (the
    slots and arrival counters must be left zeroed for the next use)."""
    import copy

    import torch.nn as nn

    from kungfu_amd.models.resnet import Bottleneck, conv1x1
    from kungfu_amd.ops import fused_block
    from kungfu_amd.ops.fused_bn import BatchNormAct2d

    torch.manual_seed(1)
    planes = 64 if cin <= 256 else 128
    norm = lambda c, relu: BatchNormAct2d(c, relu=relu)  # noqa: E731
    down = nn.Sequential(conv1x1(cin, planes * 4, stride), BatchNormAct2d(planes * 4, relu=False)) if ds else None
    blocks = [Bottleneck(cin, planes, stride, down, norm=norm, fused_tail=True)]
    blocks += [Bottleneck(planes * 4, planes, 1, None, norm=norm, fused_tail=True) for _ in range(nblk - 1)]
    blk = nn.Sequential(*blocks).cuda().to(memory_format=torch.channels_last)
    for m in blk.modules():
        if isinstance(m, nn.BatchNorm2d):
            nn.init.uniform_(m.weight, 0.5, 1.5)
            nn.init.uniform_(m.bias, -0.2, 0.2)
    other = copy.deepcopy(blk)
    hw = 28
    res = []
    for mod, on in ((blk, False), (other, True)):
        monkeypatch.setattr(fused_block, "_INLAUNCH_FIN", on)
        outs = []
        for step in range(2):
            torch.manual_seed(100 + step)
            x = torch.randn(8, cin, hw, hw, device="cuda").bfloat16().to(memory_format=torch.channels_last)
            gout = torch.randn(8, planes * 4, hw // stride, hw // stride, device="cuda")
            xin = x.clone().requires_grad_(True)
            assert fused_block.eligible(mod[0], xin)
            out = mod(xin)
            (out.float() * gout).sum().backward()
            outs += [out.detach().clone(), xin.grad.clone()]
        outs += [p.grad.clone() for p in mod.parameters()] + [b.clone() for b in mod.buffers()]
        res.append(outs)
    for i, (a, b) in enumerate(zip(*res)):
        assert torch.equal(a, b), i
    for m in other.modules():  # the in-launch finalize left its workspaces zeroed
        if getattr(m, "_kf_fin", None) is not None:
            assert int(m._kf_fin.arrive.abs().sum()) == 0
        if getattr(m, "_kf_sums", None) is not None:
            assert float(m._kf_sums.abs().sum()) == 0.0


@needs_gpu
def test_resnet50_fused_block_step_matches_layerwise():
    """ResNet-50 S-SGD steps (bf16 shadow weights) with one-node fused bottlenecks: the
    first-step loss is as close to the float32 model as the per-layer bf16 path's, and
    training proceeds (finite, decreasing loss)."""
    import torch.nn.functional as F

    import kungfu_amd as kf
    from kungfu_amd.models import resnet50
    from kungfu_amd.ops import fused_block
    from kungfu_amd.parallel.mixed import enable_bf16_shadow

    kf.init()
    x = torch.randn(16, 3, 96, 96, device="cuda").to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (16,), device="cuda")

    def run(mode):
        torch.manual_seed(0)
        m = resnet50(fused_bn=True).cuda().to(memory_format=torch.channels_last)
        o = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9))
        if mode != "fp32":
            enable_bf16_shadow(m, o)
        old = fused_block.set_enabled(mode == "fused")
        ls = []
        try:
            for _ in range(5):
                o.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode != "fp32"):
                    loss = F.cross_entropy(m(x).float(), y)
                loss.backward()
                o.step()
                ls.append(loss.item())
        finally:
            fused_block.set_enabled(old)
        return ls

    l_r, l_l, l_f = run("fp32"), run("layer"), run("fused")
    assert abs(l_f[0] - l_r[0]) <= max(1.5 * abs(l_l[0] - l_r[0]), 0.02 * abs(l_r[0])), (l_r, l_l, l_f)
    assert all(map(lambda v: v == v and abs(v) < 1e4, l_f)), l_f
    assert l_f[-1] < l_f[0], l_f


@needs_gpu
def test_device_graph_allreduce_two_ranks():
    """KungFu strategy graphs executed on the device plane (RCCL send/recv rounds + K1)
    with 2 ranks sharing the GPU as a real RCCL communicator (KUNGFU_RCCL_COLOCATE)."""
    r = kungfu_run(2, [worker("graph_gpu.py")], timeout=300, extra=["-allow-xgmi"],
                   env={"KUNGFU_FORCE_DEVICE": "0", "KUNGFU_RCCL_COLOCATE": "1", "NCCL_SOCKET_IFNAME": "lo"})
    if "GRAPH_GPU_SKIP" in r.stdout:
        pytest.skip("RCCL refuses 2 ranks on one GPU: " + r.stdout[-300:])
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count("GRAPH_GPU_OK") == 2, r.stdout[-4000:]


@needs_gpu
def test_device_graph_allreduce_two_ranks_host_staged():
    """The device graph plane's round plans + device K1 reduce with 2 ranks on one GPU
    (host transfers), every strategy, graph-mode S-SGD, and device strategy statistics."""
    r = kungfu_run(2, [worker("graph_gpu.py")], timeout=300,
                   env={"KUNGFU_FORCE_DEVICE": "0", "KUNGFU_GPU_DATAPLANE": "host"})
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count("GRAPH_GPU_OK") == 2, r.stdout[-4000:]


@needs_gpu
def test_inception_fused_bn_matches_torch_bn():
    """Inception-v3 with the HIP BN+ReLU (the channel counts it supports) against the stock
    BatchNorm2d+ReLU model with the same weights, layer by layer on the same inputs (bf16
    autocast, training mode): end-to-end outputs of a random-init 47-layer net amplify bf16
    rounding differences chaotically (tools/diag/diag_inception_bn.py: 4e-3 per layer, 0.5 at the
    logits), so the per-layer error is what is pinned.  Plus one layer's backward."""
    from kungfu_amd.models import get_model
    from kungfu_amd.models.inception import BasicConv2d

    torch.manual_seed(7)
    ref = get_model("inception_v3").cuda().to(memory_format=torch.channels_last)
    fused = get_model("inception_v3", fused_bn=True).cuda().to(memory_format=torch.channels_last)
    fused.load_state_dict(ref.state_dict())
    x = torch.randn(4, 3, 128, 128, device="cuda").to(memory_format=torch.channels_last)
    acts = []
    hooks = [mod.register_forward_hook(lambda mo, i, o, n=n: acts.append((n, i[0].detach(), o.detach())))
             for n, mod in ref.named_modules() if isinstance(mod, BasicConv2d)]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref(x)
    for h in hooks:
        h.remove()
    fmods = dict(fused.named_modules())
    n_fused = 0
    for n, i0, o0 in acts:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            o1 = fmods[n](i0)
        n_fused += int(o0.shape[1] % 8 == 0)
        assert ((o1.float() - o0.float()).norm() / o0.float().norm()).item() < 1e-2, n
    assert n_fused >= 90  # every BN of the net (C % 8 == 0) takes the HIP kernels
    # backward of one fused layer (32 -> 64, 3x3) on the same input and upstream gradient
    r, f = ref.stem[2], fmods["stem.2"]
    xi = torch.randn(4, 32, 40, 40, device="cuda").to(memory_format=torch.channels_last)
    gy = torch.randn(4, 64, 40, 40, device="cuda").to(memory_format=torch.channels_last)
    grads = []
    for m in (r, f):
        xx = xi.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(xx)
        y.float().backward(gy)
        grads.append([xx.grad.float()] + [p.grad.float() for p in m.parameters()])
    for a, b in zip(*grads):
        assert ((b - a).norm() / a.norm()).item() < 2e-2
    assert torch.allclose(f.bn.running_mean, r.bn.running_mean, rtol=1e-2, atol=1e-3)


@needs_gpu
@pytest.mark.parametrize("C", [64, 128, 512])
@pytest.mark.parametrize("relu", [True, False])
def test_bias_act_matches_torch(H, C, relu):
    """Fused conv bias (+ReLU) forward (in place) and backward (gated gradient + bias
    gradient) vs f32 torch."""
    torch.manual_seed(8)
    y0 = torch.randn(3, C, 17, 19, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    b = torch.randn(C, device="cuda")
    ref = y0.float() + b.view(1, -1, 1, 1)
    ref = ref.clamp_min(0) if relu else ref
    y = y0.clone()
    H.bias_act_forward_(y, b, relu)
    assert ((y.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    dy = torch.randn_like(y0)
    dz, db = H.bias_act_backward(dy, y, relu)
    gate = (y.float() > 0) if relu else torch.ones_like(ref, dtype=torch.bool)
    dz_ref = dy.float() * gate
    assert torch.equal(dz.float(), dz_ref.bfloat16().float())
    db_ref = dz_ref.sum(dim=(0, 2, 3))
    assert ((db - db_ref).norm() / db_ref.norm()).item() < 1e-4
    # deterministic (fixed-order partial sums, no atomics), also over a many-block grid
    dz2, db2 = H.bias_act_backward(dy, y, relu)
    assert torch.equal(db, db2) and torch.equal(dz, dz2)
    big = torch.randn(64, C, 28, 28, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    dyb = torch.randn_like(big)
    _, d1 = H.bias_act_backward(dyb, big, relu)
    _, d2 = H.bias_act_backward(dyb, big, relu)
    gb = (big.float() > 0) if relu else torch.ones_like(big, dtype=torch.bool)
    ref_b = (dyb.float() * gb).double().sum(dim=(0, 2, 3))
    assert torch.equal(d1, d2) and ((d1.double() - ref_b).norm() / ref_b.norm()).item() < 1e-5


@needs_gpu
def test_vgg_fused_conv_relu_matches_stock():
    """VGG-16 with Conv2dReLU (MFMA conv + fused bias/ReLU pass) vs the stock conv -> ReLU
    model: per-layer outputs on the same bf16 inputs, and one layer's gradients."""
    from kungfu_amd.models import get_model
    from kungfu_amd.ops.conv import Conv2dReLU

    import kungfu_amd.ops.conv as kconv

    torch.manual_seed(9)
    # bf16 parameters so the fused model takes the MFMA + bias/ReLU path without the shadow engine
    ref = get_model("vgg16").cuda().to(memory_format=torch.channels_last)
    fused = get_model("vgg16", fused_bn=True).cuda().to(memory_format=torch.channels_last)
    fused.load_state_dict(ref.state_dict())
    ref, fused = ref.bfloat16(), fused.bfloat16()
    calls = []
    orig = kconv._BiasActFn.apply
    kconv._BiasActFn.apply = lambda *a: calls.append(1) or orig(*a)
    n = 0
    for i, m in enumerate(fused.features):
        if not isinstance(m, Conv2dReLU) or m.in_channels % 64:
            continue
        r = ref.features[i]
        x = torch.randn(2, m.in_channels, 20, 20, device="cuda").bfloat16().to(memory_format=torch.channels_last)
        gy = torch.randn(2, m.out_channels, 20, 20, device="cuda").to(memory_format=torch.channels_last)
        outs = []
        for mod, act in ((r, True), (m, False)):
            xx = x.clone().requires_grad_(True)
            mod.zero_grad()
            y = mod(xx)
            y = torch.relu(y) if act else y
            y.float().backward(gy)
            outs.append([y.detach().float(), xx.grad.float(), mod.weight.grad.float(), mod.bias.grad.float()])
        for a, c in zip(*outs):
            assert ((c - a).norm() / a.norm()).item() < 2e-2, i
        n += 1
    del kconv._BiasActFn.apply  # back to the inherited Function.apply
    assert n == 12 and len(calls) == 12


@needs_gpu
@pytest.mark.parametrize("shape", [(2, 64, 224, 224), (3, 512, 14, 14), (2, 8, 6, 10)])
def test_maxpool2x2_matches_torch(H, shape):
    """2x2/s2 max-pool forward and gradient (argmax recomputed from x, ties included: the
    ReLU'd input has many all-zero windows) vs torch's max-pool on the same bf16 values."""
    import torch.nn.functional as F

    from kungfu_amd.ops.pool import max_pool2x2

    torch.manual_seed(10)
    x = torch.randn(*shape, device="cuda").clamp_min(0).bfloat16().to(memory_format=torch.channels_last)
    dy = torch.randn(shape[0], shape[1], shape[2] // 2, shape[3] // 2, device="cuda").bfloat16().to(
        memory_format=torch.channels_last)
    xr = x.float().requires_grad_(True)
    yr = F.max_pool2d(xr, 2, 2)
    yr.backward(dy.float())
    xa = x.clone().requires_grad_(True)
    ya = max_pool2x2(xa)
    ya.backward(dy)
    assert torch.equal(ya.float(), yr.detach())
    assert torch.equal(xa.grad.float(), xr.grad)


@needs_gpu
def test_conv_relu_first_layer_autocast():
    """Conv2dReLU on an f32 image under bf16 autocast (library conv, then the fused bias+ReLU
    pass) vs the stock conv -> ReLU: output, input gradient and parameter gradients."""
    import kungfu_amd.ops.conv as kconv

    torch.manual_seed(11)
    ref = torch.nn.Conv2d(3, 64, 3, padding=1).cuda().to(memory_format=torch.channels_last)
    m = kconv.Conv2dReLU(3, 64, 3, padding=1).cuda().to(memory_format=torch.channels_last)
    m.load_state_dict(ref.state_dict())
    x = torch.randn(2, 3, 32, 32, device="cuda").to(memory_format=torch.channels_last)
    gy = torch.randn(2, 64, 32, 32, device="cuda").to(memory_format=torch.channels_last)
    outs = []
    for mod, act in ((ref, True), (m, False)):
        xx = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = mod(xx)
            y = torch.relu(y) if act else y
        y.float().backward(gy)
        outs.append([y.detach().float(), xx.grad.float(), mod.weight.grad.float(), mod.bias.grad.float()])
    for a, c in zip(*outs):
        assert ((c - a).norm() / a.norm()).item() < 2e-2


@needs_gpu
def test_relu_and_maxpool_propagate_nan(H):
    """the fused ReLU and the 2x2 max-pool keep a NaN (torch.relu / max_pool2d do),
    so a diverging loss surfaces on the fused VGG path too."""
    import torch.nn.functional as F

    from kungfu_amd.ops.pool import max_pool2x2

    y = torch.randn(2, 64, 4, 6, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    y[0, 3, 1, 2] = float("nan")
    y[1, 10, 0, 0] = float("nan")
    b = torch.zeros(64, device="cuda")
    z = y.clone()
    H.bias_act_forward_(z, b, True)
    assert torch.isnan(z[0, 3, 1, 2]) and torch.isnan(z[1, 10, 0, 0])
    assert torch.equal(torch.isnan(z), torch.isnan(torch.relu(y)))
    x = torch.randn(2, 64, 8, 8, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    x[0, 5, 3, 3] = float("nan")  # bottom-right of its window: a strict '>' would drop it
    x[1, 7, 0, 1] = float("nan")
    ref = F.max_pool2d(x.float(), 2, 2)
    got = max_pool2x2(x)
    assert torch.equal(torch.isnan(got.float()), torch.isnan(ref))
    assert torch.equal(torch.nan_to_num(got.float(), nan=7.0), torch.nan_to_num(ref, nan=7.0))


@needs_gpu
@pytest.mark.parametrize("shape,pad", [((2, 64, 147, 147), 0), ((2, 192, 71, 71), 0), ((3, 288, 35, 35), 0),
                                       ((2, 40, 9, 10), 0), ((2, 16, 12, 11), 1)])
def test_maxpool3x3s2_matches_torch(shape, pad):
    """3x3/s2 max-pool (byte argmax + gather backward) vs torch's max-pool on the same bf16
    values: identical outputs and gradients (ties: first maximum, like torch)."""
    import torch.nn.functional as F

    from kungfu_amd.ops.pool import max_pool3x3s2

    torch.manual_seed(12)
    x = torch.randn(*shape, device="cuda").clamp_min(0).bfloat16().to(memory_format=torch.channels_last)
    xr = x.float().cpu().contiguous().requires_grad_(True)  # CPU NCHW reference
    yr = F.max_pool2d(xr, 3, 2, pad)
    dy = torch.randn_like(yr).bfloat16().cuda().to(memory_format=torch.channels_last)
    yr.backward(dy.float().cpu())
    xa = x.clone().requires_grad_(True)
    ya = max_pool3x3s2(xa, pad)
    ya.backward(dy)
    assert torch.equal(ya.float().cpu(), yr.detach())
    assert ((xa.grad.float().cpu() - xr.grad).abs().max() <= 2e-2 * xr.grad.abs().max()).item()


@needs_gpu
@pytest.mark.parametrize("shape", [(2, 32, 35, 35), (2, 192, 17, 17), (3, 320, 8, 8), (2, 8, 3, 5)])
def test_avgpool3x3s1_matches_torch(shape):
    import torch.nn.functional as F

    from kungfu_amd.ops.pool import avg_pool3x3s1

    torch.manual_seed(13)
    x = torch.randn(*shape, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    dy = torch.randn(*shape, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    # reference in float64 on the CPU (NCHW): on this ROCm build the GPU NHWC avg_pool2d
    # BACKWARD returns the gradient shifted by the padding (tools/diag/dbg_avgpool.py: its dx(0,0)
    # equals the true dx(1,1)), so torch-on-GPU cannot be the reference for the gradient
    xr = x.double().cpu().contiguous().requires_grad_(True)
    yr = F.avg_pool2d(xr, 3, 1, 1)
    yr.backward(dy.double().cpu().contiguous())
    xa = x.clone().requires_grad_(True)
    ya = avg_pool3x3s1(xa)
    ya.backward(dy)
    assert _rel(ya.cpu(), yr) < 1e-2 and _rel(xa.grad.cpu(), xr.grad) < 1e-2


@needs_gpu
@pytest.mark.parametrize("H,C,K,stride,ks", [(56, 64, 256, 1, 1), (28, 128, 512, 1, 1), (28, 64, 128, 1, 3),
                                            (56, 256, 512, 2, 1)])
def test_conv_persistent_stats_epilogue(H, C, K, stride, ks):
    """Large-M convolutions take the persistent-block path of the statistics epilogue (one
    atomic flush per block, stats accumulated across m-tiles): output vs torch, and the
    per-channel sum / sum of squares vs float64 sums of that output."""
    import torch.nn.functional as F

    torch.manual_seed(14)
    N = 64
    x = torch.randn(N, C, H, H, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    w = (torch.randn(K, C, ks, ks, device="cuda") * 0.05).bfloat16().to(memory_format=torch.channels_last)
    st = torch.zeros(H_slots() * 2 * K, dtype=torch.float64, device="cuda")
    from kungfu_amd._lib import hip

    y = hip().conv(x, w, stride, st, None, -1)
    ref = F.conv2d(x.float(), w.float(), stride=stride, padding=(ks - 1) // 2)
    assert _rel(y, ref) < 1e-2
    sums = st.view(-1, 2, K).sum(0)
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, K)
    torch.testing.assert_close(sums[0], yd.sum(0), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(sums[1], (yd * yd).sum(0), rtol=1e-6, atol=1e-3)


def H_slots():
    from kungfu_amd._lib import hip

    return hip().conv_stat_slots


@needs_gpu
@pytest.mark.parametrize("N,OH,K,C", [(4, 7, 128, 64), (8, 14, 256, 128), (2, 28, 512, 256), (16, 4, 64, 192)])
def test_conv_dgrad_s2_matches_torch(N, OH, K, C):
    """Stride-2 data gradients on the parity-phase MFMA kernels vs the float32 torch data
    gradient: 3x3/pad 1 (four phases, every pixel; with the BN-backward sums epilogue vs
    float64 sums of the gated gradient) and 1x1 (even pixels) completed by a stride-1 1x1 data
    gradient accumulated with acc_even (the ResNet downsample block's block-input gradient)."""
    import torch.nn.functional as F

    from kungfu_amd._lib import hip

    H = hip()
    torch.manual_seed(21)
    dy = torch.randn(N, K, OH, OH, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(N, C, 2 * OH, 2 * OH, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    for ks in (3, 1):
        w = (torch.randn(K, C, ks, ks, device="cuda") * 0.05).bfloat16().to(memory_format=torch.channels_last)
        ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [2, 2], [(ks - 1) // 2] * 2,
                                                  [1, 1], False, [0, 0], 1, [True, False, False])[0]
        wt = H.conv_flip_weight(w)
        if ks == 3:
            dx = H.conv_dgrad_s2(dy, wt, 3)
            assert _rel(dx, ref) < 1e-2, ks
            # BN backward sums of a BN+ReLU whose input is bx, forward coefficients fc
            bx = torch.randn_like(x)
            fc = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2])
            st = torch.zeros(H_slots() * 2 * C, dtype=torch.float64, device="cuda")
            dx2 = H.conv_dgrad_s2(dy, wt, 3, st, bx, fc)
            assert torch.equal(dx2, dx)
            xd = bx.double().permute(0, 2, 3, 1).reshape(-1, C)
            gd = dx.double().permute(0, 2, 3, 1).reshape(-1, C)
            on = (bx.float().permute(0, 2, 3, 1).reshape(-1, C) * fc[:C] + fc[C:]) > 0
            dz = torch.where(on, gd, torch.zeros_like(gd))
            sums = st.view(-1, 2, C).sum(0)
            torch.testing.assert_close(sums[0], dz.sum(0), rtol=1e-5, atol=1e-2)
            torch.testing.assert_close(sums[1], (dz * xd).sum(0), rtol=1e-5, atol=1e-2)
        else:
            dx = H.conv_dgrad_s2(dy, wt, 1)
            ev = dx[:, :, 0::2, 0::2]
            assert _rel(ev, ref[:, :, 0::2, 0::2]) < 1e-2
            # complete it: + the stride-1 1x1 data gradient of a second conv over all pixels
            dy1 = torch.randn(N, K, 2 * OH, 2 * OH, device="cuda").bfloat16().to(memory_format=torch.channels_last)
            w1 = (torch.randn(K, C, 1, 1, device="cuda") * 0.05).bfloat16().to(memory_format=torch.channels_last)
            ref1 = F.conv_transpose2d(dy1.float(), w1.float())
            out = H.conv(dy1, H.conv_flip_weight(w1), 1, None, dx, acc_even=True)
            assert out.data_ptr() == dx.data_ptr()
            assert _rel(out, ref + ref1) < 1e-2


@needs_gpu
@pytest.mark.parametrize("N,DH,DW,K,C,pad", [(4, 25, 25, 384, 288, 0), (4, 25, 25, 96, 96, 0), (3, 12, 12, 320, 192, 0),
                                             (3, 13, 11, 64, 40, 1), (2, 9, 10, 128, 64, 0)])
def test_conv_dgrad_s2_any_size_matches_torch(N, DH, DW, K, C, pad):
    """Stride-2 3x3 data gradient for ANY input size / padding 0|1 and channel counts % 8
    (Inception's 25x25 -> 12x12 pad-0 layers): four parity phases of different sizes vs the
    float32 torch data gradient, and with the BN-backward sums epilogue."""
    from kungfu_amd._lib import hip

    H = hip()
    torch.manual_seed(23)
    OH, OW = (DH + 2 * pad - 3) // 2 + 1, (DW + 2 * pad - 3) // 2 + 1
    dy = torch.randn(N, K, OH, OW, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(N, C, DH, DW, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 3, 3, device="cuda") * 0.05).bfloat16().to(memory_format=torch.channels_last)
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [2, 2], [pad, pad],
                                              [1, 1], False, [0, 0], 1, [True, False, False])[0]
    wt = H.conv_flip_weight(w)
    dx = H.conv_dgrad_s2(dy, wt, 3, dh=DH, dw=DW, pad=pad)
    assert dx.shape == ref.shape
    assert _rel(dx, ref) < 1e-2
    bx = torch.randn_like(x)
    fc = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2])
    st = torch.zeros(H_slots() * 2 * C, dtype=torch.float64, device="cuda")
    dx2 = H.conv_dgrad_s2(dy, wt, 3, st, bx, fc, None, -1, DH, DW, pad)
    assert torch.equal(dx2, dx)
    xd = bx.double().permute(0, 2, 3, 1).reshape(-1, C)
    gd = dx.double().permute(0, 2, 3, 1).reshape(-1, C)
    on = (bx.float().permute(0, 2, 3, 1).reshape(-1, C) * fc[:C] + fc[C:]) > 0
    dz = torch.where(on, gd, torch.zeros_like(gd))
    sums = st.view(-1, 2, C).sum(0)
    torch.testing.assert_close(sums[0], dz.sum(0), rtol=1e-5, atol=1e-2)
    torch.testing.assert_close(sums[1], (dz * xd).sum(0), rtol=1e-5, atol=1e-2)


@needs_gpu
@pytest.mark.parametrize("N,Hh,C,K", [(3, 12, 64, 64), (2, 10, 64, 128), (2, 9, 128, 256), (1, 8, 256, 512)])
def test_conv_bias_relu_and_gate_epilogues(H, N, Hh, C, K):
    """conv epilogues of the fused VGG stack: relu(conv + bias) vs f32 torch; the ReLU-gated
    data gradient (conv * (y_prev > 0)) bit-exact vs the plain kernel output masked, and its
    per-channel sums (the bias gradient) vs f64 sums."""
    import torch.nn.functional as F

    torch.manual_seed(31)
    cl = lambda t: t.contiguous(memory_format=torch.channels_last)  # noqa: E731
    x = cl(torch.randn(N, C, Hh, Hh, device="cuda")).bfloat16()
    w = cl(torch.randn(K, C, 3, 3, device="cuda") * 0.05).bfloat16()
    b = (torch.randn(K, device="cuda") * 0.5).bfloat16()
    y = H.conv(x, w, 1, bias=b)
    ref = F.relu(F.conv2d(x.float(), w.float(), padding=1) + b.float().view(1, -1, 1, 1))
    assert _rel(y, ref) < 1e-2
    assert (y.float() >= 0).all()
    yprev = cl(F.relu(torch.randn(N, K, Hh, Hh, device="cuda"))).bfloat16()
    st = torch.zeros(H.conv_stat_slots * 2 * K, dtype=torch.float64, device="cuda")
    dz = H.conv(x, w, 1, st, None, -1, bn_x=yprev, gate=True)
    plain = H.conv(x, w, 1)
    exp = torch.where(yprev > 0, plain, torch.zeros_like(plain))
    torch.testing.assert_close(dz.float(), exp.float(), rtol=0, atol=0)
    sums = st.view(-1, 2, K)[:, 0].sum(0)
    torch.testing.assert_close(sums, exp.double().sum((0, 2, 3)), rtol=1e-6, atol=1e-3)


@needs_gpu
@pytest.mark.parametrize("C", [64, 128, 512])
def test_maxpool2x2_gate_backward(H, C):
    """2x2 max-pool backward with the ReLU gate of its input and the per-channel gradient sums
    (VGG's conv -> ReLU -> pool): bit-exact vs the plain gather masked by x > 0."""
    torch.manual_seed(32)
    cl = lambda t: t.contiguous(memory_format=torch.channels_last)  # noqa: E731
    x = cl(torch.relu(torch.randn(3, C, 10, 12, device="cuda"))).bfloat16()
    x[:, :, :4] = 0  # whole windows of zeros: the ReLU gate closes
    dy = cl(torch.randn(3, C, 5, 6, device="cuda")).bfloat16()
    st = torch.zeros(H.conv_stat_slots * 2 * C, dtype=torch.float64, device="cuda")
    dx = H.maxpool2x2_backward(x, dy, gate_stats=st)
    plain = H.maxpool2x2_backward(x, dy)
    exp = torch.where(x > 0, plain, torch.zeros_like(plain))
    torch.testing.assert_close(dx.float(), exp.float(), rtol=0, atol=0)
    torch.testing.assert_close(st.view(-1, 2, C)[:, 0].sum(0), exp.double().sum((0, 2, 3)), rtol=1e-6, atol=1e-3)


@needs_gpu
def test_vgg16_fused_stack_matches_layered():
    """VGG-16 with its feature stack as one fused autograd node (bias/ReLU in the conv and pool
    kernels) vs the same modules run layer by layer (Conv2dReLU + MaxPool2x2), both under bf16
    autocast, each measured against an f32 run of the same weights: at random init the early
    layers' gradients are tiny and carry ~5-45 % bf16 noise on EITHER path (the layered path
    differs that much from itself between runs), so the fused path must be as close to f32 as
    the layered one, not bit-equal to it."""
    from kungfu_amd.models.vgg import vgg16
    from kungfu_amd.ops.vgg_fused import FusedVGGFeatures

    torch.manual_seed(33)
    m = vgg16(fused_bn=True).cuda().to(memory_format=torch.channels_last).eval()  # no dropout masks
    x = torch.randn(4, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
    tgt = torch.randint(0, 1000, (4,), device="cuda")

    def run(fused, amp=True):
        m.zero_grad(set_to_none=True)
        orig = FusedVGGFeatures.forward
        if not fused:
            FusedVGGFeatures.forward = torch.nn.Sequential.forward
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                out = m(x)
                loss = torch.nn.functional.cross_entropy(out.float(), tgt)
            loss.backward()
        finally:
            FusedVGGFeatures.forward = orig
        return out.float().detach(), {k: p.grad.detach().float().clone() for k, p in m.named_parameters()}

    o1, g1 = run(True)
    o0, g0 = run(False)
    of, gf = run(False, amp=False)
    rel = lambda a, b: ((a - b).norm() / (b.norm() + 1e-12)).item()  # noqa: E731
    assert rel(o1, of) < 1.5 * rel(o0, of) + 1e-3
    for k in gf:
        e1, e0 = rel(g1[k], gf[k]), rel(g0[k], gf[k])
        assert e1 < 1.5 * e0 + 0.02, (k, e1, e0)


@needs_gpu
def test_conv_flip_weights_multi_matches_single(H):
    """Multi-tensor weight flip (tiled transpose, one launch for many layers, incl. channel
    counts that are not multiples of the 64x64 tile) == w.flip(2, 3).transpose(0, 1)."""
    torch.manual_seed(34)
    shapes = [(64, 64, 3), (256, 64, 1), (64, 256, 1), (512, 128, 3), (96, 40, 3), (8, 200, 1)]
    srcs = [torch.randn(co, ci, k, k, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            for co, ci, k in shapes]
    dsts = [torch.empty(ci, co, k, k, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
            for co, ci, k in shapes]
    H.conv_flip_weights(srcs, dsts)
    for w, d in zip(srcs, dsts):
        torch.testing.assert_close(d, w.flip(2, 3).transpose(0, 1), rtol=0, atol=0)


@needs_gpu
@pytest.mark.parametrize("S,p", [(128, 0.0), (64, 0.0), (128, 0.1), (64, 0.25)])
def test_fused_attention_matches_fp32(S, p):
    """Fused self-attention (csrc/kernels/attention.hip) forward and dq/dk/dv vs an f32 torch
    composition with the SAME dropout mask (the kernels' counter hash, reproduced by
    ops.attention.dropout_keep)."""
    from kungfu_amd.ops.attention import _AttnFn, dropout_keep

    torch.manual_seed(41)
    B, H = 3, 4
    qkv = (torch.randn(B, S, 3 * H * 64, device="cuda") * 1.5).bfloat16().requires_grad_(True)
    seed = 12345
    out = _AttnFn.apply(qkv, H, p, seed)
    gout = torch.randn_like(out)
    out.backward(gout)
    x = qkv.detach().float().requires_grad_(True)
    q, k, v = x.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
    P = torch.softmax(q @ k.transpose(-1, -2) / 8.0, dim=-1)
    from kungfu_amd.ops import dropout_seed

    keep = dropout_keep(dropout_seed.effective(seed), B, H, S, p, device="cuda")
    if p > 0:
        frac = keep.float().mean().item()
        assert abs(frac - (1 - p)) < 0.01, frac
    Pd = P * keep / (1 - p)
    ref = (Pd @ v).transpose(1, 2).reshape(B, S, H * 64)
    ref.backward(gout.float())
    assert _rel(out, ref) < 2e-2
    assert _rel(qkv.grad, x.grad) < 3e-2
    for t in range(3):  # q, k, v blocks separately
        a = qkv.grad.view(B, S, 3, H * 64)[:, :, t]
        r = x.grad.view(B, S, 3, H * 64)[:, :, t]
        assert ((a.float() - r).norm() / r.norm()).item() < 2e-2, t


@needs_gpu
@pytest.mark.parametrize("T,i,o", [(1000, 768, 768), (4096, 768, 3072), (333, 128, 64)])
def test_linear_mfma_wgrad_matches_fp32(T, i, o):
    """ops.linear: F.linear forward, weight gradient on the split-K MFMA kernel (a linear
    layer's dW is the 1x1-conv weight gradient over tokens), data and bias gradients via torch;
    all vs f32 torch."""
    from kungfu_amd.ops.linear import eligible, linear

    torch.manual_seed(42)
    x = torch.randn(2, T, i, device="cuda").bfloat16().requires_grad_(True)
    w = (torch.randn(o, i, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    b = torch.randn(o, device="cuda").bfloat16().requires_grad_(True)
    assert eligible(x, w)
    y = linear(x, w, b)
    g = torch.randn_like(y)
    y.backward(g)
    xf, wf, bf = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yf = torch.nn.functional.linear(xf, wf, bf)
    yf.backward(g.float())
    for a, r in ((y, yf), (x.grad, xf.grad), (w.grad, wf.grad), (b.grad, bf.grad)):
        assert a.dtype == torch.bfloat16
        assert ((a.float() - r).norm() / r.norm()).item() < 1e-2


@needs_gpu
@pytest.mark.parametrize("N,C,Hh", [(8, 2048, 7), (3, 64, 5), (2, 768, 8)])
def test_global_avg_pool_matches_torch(N, C, Hh):
    """Global average pool (ResNet / Inception head) on pool.hip vs the float32 torch mean, and
    its backward (dy / HW broadcast to every pixel) vs autograd of the float32 mean."""
    from kungfu_amd.ops.pool import global_avg_pool

    torch.manual_seed(5)
    x = torch.randn(N, C, Hh, Hh, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    xa = x.clone().requires_grad_(True)
    y = global_avg_pool(xa)
    assert y.grad_fn is not None and "GlobalAvgPool" in type(y.grad_fn).__name__
    xr = x.float().requires_grad_(True)
    yr = xr.mean((2, 3))
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(N, C, device="cuda").bfloat16()
    y.backward(dy)
    yr.backward(dy.float())
    assert xa.grad.is_contiguous(memory_format=torch.channels_last)
    assert _rel(xa.grad, xr.grad) < 1e-2


@needs_gpu
@pytest.mark.parametrize("kh,kw,ph,pw,stride,C,K,Hh", [(1, 7, 0, 3, 1, 128, 192, 12), (7, 1, 3, 0, 1, 192, 128, 12),
                                                       (1, 3, 0, 1, 1, 384, 384, 5), (3, 1, 1, 0, 1, 384, 384, 5),
                                                       (5, 5, 2, 2, 1, 64, 64, 9), (3, 3, 0, 0, 2, 192, 320, 12),
                                                       (3, 3, 0, 0, 1, 64, 128, 10), (1, 1, 0, 0, 1, 768, 192, 12),
                                                       # channel counts off the 64 grid (zero-padded K / N)
                                                       (3, 3, 0, 0, 1, 80, 192, 12), (5, 5, 2, 2, 1, 48, 64, 9),
                                                       (1, 1, 0, 0, 1, 192, 48, 12), (3, 3, 1, 1, 1, 96, 96, 10),
                                                       (1, 7, 0, 3, 1, 160, 160, 12), (3, 3, 0, 0, 2, 288, 384, 12),
                                                       (3, 3, 0, 0, 1, 32, 32, 13)])
def test_conv_rect_matches_torch(kh, kw, ph, pw, stride, C, K, Hh):
    """Inception-v3 windows on the MFMA kernel (``ops.conv._ConvRectFn``): forward with the
    BN-statistics epilogue, data and weight gradients (``conv_wgrad_rect`` for the windows /
    channel counts the ResNet planner does not take), all vs the float32 torch convolution;
    the statistics vs float64 sums of the bf16 output."""
    import torch.nn.functional as F

    from kungfu_amd.ops.conv import conv2d_stats, rect_eligible

    torch.manual_seed(33)
    N = 4
    x = torch.randn(N, C, Hh, Hh, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    w = (torch.randn(K, C, kh, kw, device="cuda") * 0.05).bfloat16().to(memory_format=torch.channels_last)
    assert rect_eligible(x, w, stride, (ph, pw), 1, 1)
    st = torch.zeros(H_slots() * 2 * K, dtype=torch.float64, device="cuda")
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = conv2d_stats(xa, wa, stride, (ph, pw), st)
    xr, wr = x.float().requires_grad_(True), w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=stride, padding=(ph, pw))
    assert y.shape == yr.shape and _rel(y, yr) < 1e-2
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, K)
    sums = st.view(-1, 2, K).sum(0)
    torch.testing.assert_close(sums[0], yd.sum(0), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(sums[1], (yd * yd).sum(0), rtol=1e-6, atol=1e-3)
    dy = torch.randn_like(yr)
    y.backward(dy.bfloat16().contiguous(memory_format=torch.channels_last))
    yr.backward(dy)
    assert _rel(xa.grad, xr.grad) < 2e-2
    assert _rel(wa.grad, wr.grad) < 2e-2


@needs_gpu
@pytest.mark.parametrize("cin,cout,kw", [(128, 192, dict(kernel_size=(1, 7), padding=(0, 3))),
                                         (768, 192, dict(kernel_size=1)),
                                         (448, 384, dict(kernel_size=3, padding=1)),
                                         (192, 320, dict(kernel_size=3, stride=2)),
                                         (48, 64, dict(kernel_size=5, padding=2)),
                                         (768, 160, dict(kernel_size=1))])
def test_inception_basicconv_mfma_stats_path(monkeypatch, cin, cout, kw):
    """Inception BasicConv2d on the MFMA conv with the BN-statistics epilogue (the path taken
    with bf16 shadow weights) vs the stock conv + BatchNorm2d + ReLU module in float32:
    output, input / weight / gamma / beta gradients and the running statistics."""
    import copy

    import kungfu_amd.parallel.mixed as mixed
    from kungfu_amd.models import inception as inc

    torch.manual_seed(12)
    inc._FUSED_BN[0] = True
    try:
        fused = inc.BasicConv2d(cin, cout, **kw).cuda().to(memory_format=torch.channels_last)
    finally:
        inc._FUSED_BN[0] = False
    ref = inc.BasicConv2d(cin, cout, **kw).cuda().to(memory_format=torch.channels_last)
    ref.load_state_dict(fused.state_dict())
    with torch.no_grad():
        fused.bn.weight.uniform_(0.5, 1.5)
        fused.bn.bias.uniform_(-0.2, 0.2)
        ref.bn.weight.copy_(fused.bn.weight)
        ref.bn.bias.copy_(fused.bn.bias)
    # the bf16 compute weight the shadow machinery would hand over (a differentiable cast here)
    monkeypatch.setattr(mixed, "shadow", lambda p: p.bfloat16().contiguous(memory_format=torch.channels_last))
    lay = copy.deepcopy(ref)  # stock conv + BN in bf16 autocast: the bf16 error baseline
    x = torch.randn(4, cin, 12, 12, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    xf, xr, xl = x.clone().requires_grad_(True), x.float().requires_grad_(True), x.clone().requires_grad_(True)
    y = fused(xf)
    assert fused.bn._kf_sums is not None  # the statistics came from the conv epilogue
    yr = ref(xr)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        yl = lay(xl)

    def nrel(a, b):  # norm-relative: bf16 activations through a BN backward
        return ((a.float() - b.float()).norm() / b.float().norm()).item()

    def close(a, l, r, what):
        assert nrel(a, r) <= max(1.5 * nrel(l, r), 1e-2), (what, nrel(a, r), nrel(l, r))

    close(y, yl, yr, "out")
    g = torch.randn_like(yr)
    y.float().backward(g)
    yr.backward(g)
    yl.float().backward(g)
    close(xf.grad, xl.grad, xr.grad, "dx")
    for (n, p), (_, q), (_, l) in zip(fused.named_parameters(), ref.named_parameters(), lay.named_parameters()):
        close(p.grad, l.grad, q.grad, n)
    assert torch.allclose(fused.bn.running_mean, ref.bn.running_mean, rtol=1e-2, atol=1e-3)
    assert torch.allclose(fused.bn.running_var, ref.bn.running_var, rtol=1e-2, atol=1e-3)
    assert int(fused.bn.num_batches_tracked) == 1


@needs_gpu
def test_sibling_convs_match_torch(monkeypatch):
    """Inception branch heads as one autograd node (``ops.conv.sibling_convs``): outputs, the
    input gradient (the siblings' data gradients chained by the accumulate epilogue) and the
    weight gradients vs float32 torch convolutions of the same input."""
    import torch.nn as nn
    import torch.nn.functional as F

    import kungfu_amd.parallel.mixed as mixed
    from kungfu_amd.ops.conv import sibling_convs

    torch.manual_seed(17)
    monkeypatch.setattr(mixed, "shadow", lambda p: p.bfloat16().contiguous(memory_format=torch.channels_last))
    convs = [nn.Conv2d(192, 64, 1, bias=False), nn.Conv2d(192, 48, 1, bias=False),
             nn.Conv2d(192, 96, (1, 3), padding=(0, 1), bias=False), nn.Conv2d(192, 64, 3, padding=1, bias=False)]
    convs = [c.cuda().to(memory_format=torch.channels_last) for c in convs]
    x = torch.randn(4, 192, 12, 12, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    xa, xr = x.clone().requires_grad_(True), x.float().requires_grad_(True)
    st = [torch.zeros(H_slots() * 2 * c.out_channels, dtype=torch.float64, device="cuda") for c in convs]
    ys = sibling_convs(xa, convs, st)
    assert ys is not None and len(ys) == 4
    gs = [torch.randn(4, c.out_channels, 12, 12, device="cuda") for c in convs]
    wr = [c.weight.detach().bfloat16().float().requires_grad_(True) for c in convs]
    yr = [F.conv2d(xr, w, padding=c.padding) for w, c in zip(wr, convs)]
    for y, r, s, c in zip(ys, yr, st, convs):
        assert _rel(y, r) < 1e-2
        sums = s.view(-1, 2, c.out_channels).sum(0)
        torch.testing.assert_close(sums[0], y.double().sum((0, 2, 3)), rtol=1e-6, atol=1e-3)
    sum((y.float() * g).sum() for y, g in zip(ys, gs)).backward()
    sum((y * g).sum() for y, g in zip(yr, gs)).backward()
    assert _rel(xa.grad, xr.grad) < 2e-2
    for c, w in zip(convs, wr):
        assert _rel(c.weight.grad, w.grad) < 2e-2


@needs_gpu
def test_inception_bn_link_chain(monkeypatch):
    """BasicConv2d -> BasicConv2d chain with the BN link (the second conv's data-gradient
    epilogue produces the first BN's backward sums; that BN skips its reduction pass) vs the
    stock modules in float32, against the bf16 autocast baseline error."""
    import copy

    import kungfu_amd.ops.fused_bn as fbn
    import kungfu_amd.parallel.mixed as mixed
    from kungfu_amd.models import inception as inc

    torch.manual_seed(19)
    inc._FUSED_BN[0] = True
    try:
        fused = [inc.BasicConv2d(64, 96, kernel_size=3, padding=1), inc.BasicConv2d(96, 160, kernel_size=(1, 7),
                                                                                    padding=(0, 3))]
    finally:
        inc._FUSED_BN[0] = False
    fused = [m.cuda().to(memory_format=torch.channels_last) for m in fused]
    ref = [inc.BasicConv2d(64, 96, kernel_size=3, padding=1), inc.BasicConv2d(96, 160, kernel_size=(1, 7),
                                                                              padding=(0, 3))]
    ref = [m.cuda().to(memory_format=torch.channels_last) for m in ref]
    for f, r in zip(fused, ref):
        with torch.no_grad():
            f.bn.weight.uniform_(0.5, 1.5)
            f.bn.bias.uniform_(-0.2, 0.2)
        r.load_state_dict(f.state_dict())
    lay = copy.deepcopy(ref)
    monkeypatch.setattr(mixed, "shadow", lambda p: p.bfloat16().contiguous(memory_format=torch.channels_last))
    used = []
    orig = fbn.hip

    class _Spy:
        def __getattr__(self, n):
            f = getattr(orig(), n)
            if n != "bn_backward":
                return f

            def wrapped(*a, **k):
                used.append(len(a) > 10 and a[10] is not None)
                return f(*a, **k)
            return wrapped

    monkeypatch.setattr(fbn, "hip", lambda: _Spy())
    x = torch.randn(4, 64, 14, 14, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    xf, xr, xl = x.clone().requires_grad_(True), x.float().requires_grad_(True), x.clone().requires_grad_(True)
    y = inc._chain(xf, fused, defer_last=False)
    assert getattr(fused[0].bn, "_kf_sums", None) is not None
    yr = ref[1](ref[0](xr))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        yl = lay[1](lay[0](xl))
    g = torch.randn_like(yr)
    y.float().backward(g)
    yr.backward(g)
    yl.float().backward(g)
    assert used == [False, True]  # the second layer's BN reduces itself, the first takes the linked sums

    def nrel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm()).item()

    assert nrel(xf.grad, xr.grad) <= max(1.5 * nrel(xl.grad, xr.grad), 1e-2)
    for mf, mr, ml in zip(fused, ref, lay):
        for (n, p), (_, q), (_, l) in zip(mf.named_parameters(), mr.named_parameters(), ml.named_parameters()):
            assert nrel(p.grad, q.grad) <= max(1.5 * nrel(l.grad, q.grad), 1e-2), n
    assert all(float(m.bn._kf_sums.abs().sum()) == 0.0 for m in fused)  # workspaces re-zeroed


@needs_gpu
@pytest.mark.parametrize("C,off,tot", [(64, 64, 288), (96, 128, 288), (192, 576, 768), (48, 0, 256)])
def test_bn_backward_channel_slice_grad(H, C, off, tot):
    """BN backward reading its output gradient as a channel slice of a wider channels-last tensor
    (the gradient of an Inception concatenation) in place: bit-identical to the contiguous copy."""
    torch.manual_seed(23)
    x = torch.randn(4, C, 9, 11, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    w, b = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    y, mean, invstd, coef, _ = H.bn_forward(x, None, w, b, rm, rv, 0.1, 1e-3, True, True)
    big = torch.randn(4, tot, 9, 11, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    dy = big[:, off:off + C]
    assert not dy.is_contiguous(memory_format=torch.channels_last)
    a = H.bn_backward(dy, x, mean, invstd, w, coef, None, True, True, False)
    r = H.bn_backward(dy.contiguous(memory_format=torch.channels_last), x, mean, invstd, w, coef, None, True, True,
                      False)
    for u, v in zip(a, r):
        if u is not None and u.numel():
            assert torch.equal(u, v)


@needs_gpu
@pytest.mark.parametrize("T,O", [(16384, 768), (16384, 3072), (300, 2304), (5, 64)])
def test_colsum_matches_torch(H, T, O):
    """Bias-gradient column sums (norms.hip) vs the float64 torch sum, f32 and bf16 outputs,
    and run-to-run bit equality (deterministic two-stage reduction)."""
    torch.manual_seed(29)
    x = torch.randn(T, O, device="cuda").bfloat16()
    ref = x.double().sum(0)
    a = H.colsum(x, torch.float32)
    torch.testing.assert_close(a.double(), ref, rtol=1e-4, atol=1e-3)
    assert torch.equal(a, H.colsum(x, torch.float32))
    b = H.colsum(x, torch.bfloat16)
    assert b.dtype == torch.bfloat16 and torch.allclose(b.double(), ref, rtol=1e-2, atol=1e-1)


@needs_gpu
@pytest.mark.parametrize("batch_fin", [False, True])
@pytest.mark.parametrize("block", ["A", "B", "C", "D", "E"])
def test_inception_bn_concat_matches_cat(block, batch_fin, monkeypatch):
    """Inception blocks whose branch BN+ReLUs write straight into their slice of the
    concatenation (ops.fused_bn.bn_relu_concat) against the same blocks with the BNs applied
    separately and torch.cat: outputs, block-input and parameter gradients, running stats
    (including num_batches_tracked).  ``batch_fin``: the concatenation's BN finalizes (forward
    and backward) batched into one launch each (bn_finalize_multi / bn_backward_multi)."""
    import copy

    from kungfu_amd.models import inception as inc
    from kungfu_amd.ops import fused_bn

    torch.manual_seed(5)
    inc._FUSED_BN[0] = True
    try:
        mk = {"A": (lambda: inc.InceptionA(64, 32), 64, 13), "B": (lambda: inc.InceptionB(96), 96, 13),
              "C": (lambda: inc.InceptionC(192, 64), 192, 9), "D": (lambda: inc.InceptionD(128), 128, 9),
              "E": (lambda: inc.InceptionE(192), 192, 5)}[block]
        m0 = mk[0]().cuda().to(memory_format=torch.channels_last)
    finally:
        inc._FUSED_BN[0] = False
    for mod in m0.modules():
        if isinstance(mod, inc.BasicConv2d):
            mod.conv.to(torch.bfloat16)  # bf16 conv weights: the MFMA conv + BN-statistics path
    m1 = copy.deepcopy(m0)
    x = torch.randn(4, mk[1], mk[2], mk[2], device="cuda").bfloat16().to(memory_format=torch.channels_last)
    res = []
    g = None
    # batch_fin: the batched concatenation against the unbatched one (same kernels, same order of
    # additions: equal up to the convolutions' atomics), else the concatenation against torch.cat
    runs = ((copy.deepcopy(m0), True, False), (m1, True, True)) if batch_fin else ((m0, False, False), (m1, True, False))
    for m, on, bf in runs:
        monkeypatch.setattr(fused_bn, "CONCAT_ENABLED", on)
        monkeypatch.setattr(fused_bn, "_BATCH_FIN", bf)
        xx = x.clone().requires_grad_(True)
        y = m(xx)
        if on:
            assert y.grad_fn is not None and "BNConcat" in type(y.grad_fn).__name__
        if g is None:
            g = torch.randn_like(y.float()).bfloat16()
        y.backward(g)
        res.append((y.detach().float(), xx.grad.float(), [p.grad.float() for p in m.parameters()],
                    [b.clone() for b in m.buffers()]))
    (y0, gx0, gp0, b0), (y1, gx1, gp1, b1) = res
    # batched vs unbatched: the same math, but the batched finalize kernel's coefficients may differ
    # in the last float bit (FMA contraction), which flips the bf16 rounding of some gradient elements
    # (r4t25: 1.0e-3 / 1.5e-3 on blocks B / E, 0 elsewhere)
    tol = 3e-3 if batch_fin else 1e-3
    assert torch.equal(y0, y1)
    assert ((gx1 - gx0).norm() / gx0.norm()).item() < tol
    for a, b in zip(gp0, gp1):
        assert ((b - a).norm() / a.norm().clamp_min(1e-12)).item() < tol
    for a, b in zip(b0, b1):
        assert torch.equal(a, b)


@needs_gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_bert_layer_bias_link_matches_colsum(p, monkeypatch):
    """The out-projection / FC2 bias gradients produced by the consuming AddLayerNorm's backward
    (column sums of the residual gradient it writes, ops.linear.BiasLink) vs the linear layer's own
    column-sum pass: same forward, same gradients (bias gradients to bf16 rounding)."""
    import copy

    from kungfu_amd.models.bert import BertLayer
    from kungfu_amd.ops import layernorm

    torch.manual_seed(3)
    layer = BertLayer(dropout=p).cuda()
    for m in (layer.qkv, layer.out, layer.fc1, layer.fc2):
        m.to(torch.bfloat16)
        torch.nn.init.normal_(m.bias, std=0.02)
    other = copy.deepcopy(layer)
    x = torch.randn(4, 128, 768, device="cuda").bfloat16()
    g = torch.randn(4, 128, 768, device="cuda").bfloat16()
    orig = layernorm.add_layer_norm
    res = []
    for mod, link in ((layer, True), (other, False)):
        if not link:
            monkeypatch.setattr(layernorm, "add_layer_norm",
                                lambda *a, **k: orig(*a, **{**k, "bias_link": False}) if "bias_link" in k
                                else orig(*a[:7]))
        torch.manual_seed(11)
        xx = x.clone().requires_grad_(True)
        y = mod(xx)
        y.backward(g)
        res.append((y.detach(), xx.grad, {n: q.grad.float() for n, q in mod.named_parameters()}))
    (y0, gx0, gp0), (y1, gx1, gp1) = res
    assert torch.equal(y0, y1)
    assert torch.equal(gx0, gx1)
    for n in gp0:
        a, b = gp0[n], gp1[n]
        if n in ("out.bias", "fc2.bias"):
            assert ((a - b).norm() / b.norm()).item() < 1e-2, n
        else:
            assert torch.equal(a, b), n


@needs_gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_bert_layer_residual_link_matches_autograd_add(p, monkeypatch):
    """The skip-input gradient handed from each AddLayerNorm's backward to the consuming linear's
    data-gradient GEMM (``addmm``, ops.linear.ResidualLink) vs autograd's separate add: same forward,
    gradients equal to bf16 rounding (one rounding of dx instead of two), and the link is consumed."""
    import copy

    from kungfu_amd.models.bert import BertLayer
    from kungfu_amd.ops import linear as lin

    torch.manual_seed(3)
    layer = BertLayer(dropout=p).cuda()
    for m in (layer.qkv, layer.out, layer.fc1, layer.fc2):
        m.to(torch.bfloat16)
    other = copy.deepcopy(layer)
    for mod in (layer, other):  # the engine's linear (what the bf16-shadow models run)
        for m in (mod.qkv, mod.out, mod.fc1, mod.fc2):
            m.forward = (lambda mm: (lambda t: lin.linear(t, mm.weight, mm.bias)))(m)
    x = torch.randn(4, 128, 768, device="cuda").bfloat16()
    g = torch.randn(4, 128, 768, device="cuda").bfloat16()
    res = []
    for mod, link in ((layer, True), (other, False)):
        monkeypatch.setattr(lin, "_RES_LINK", link)
        torch.manual_seed(11)
        xx = x.clone().requires_grad_(True)
        y = mod(xx)
        rl = getattr(xx, "_kf_rlink", None)
        assert (rl is not None and rl.armed) == link
        y.backward(g)
        assert rl is None or rl.value is None  # handed over and consumed
        res.append((y.detach(), xx.grad.float(), {n: q.grad.float() for n, q in mod.named_parameters()}))
    (y0, gx0, gp0), (y1, gx1, gp1) = res
    assert torch.equal(y0, y1)
    assert ((gx0 - gx1).norm() / gx1.norm()).item() < 1e-2
    for n in gp0:
        a, b = gp0[n], gp1[n]
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)).item() < 2e-2, n


@needs_gpu
@pytest.mark.parametrize("T,O", [(16384, 3072), (1000, 776), (37, 64)])
def test_gelu_backward_colsum_matches_torch(T, O):
    """Fused erf-GELU backward + column sums (norms.hip) vs torch's GELU backward on the same bf16
    inputs and an f64 column sum of its bf16 result."""
    from kungfu_amd._lib import hip

    torch.manual_seed(9)
    u = (torch.randn(T, O, device="cuda") * 2).bfloat16()
    dy = torch.randn(T, O, device="cuda").bfloat16()
    du, db = hip().gelu_backward_colsum(dy, u, torch.float32)
    ref = torch.ops.aten.gelu_backward(dy, u)
    assert ((du.float() - ref.float()).abs() > 0).float().mean().item() < 1e-3  # same math, ~1-ulp differences
    assert ((du.float() - ref.float()).norm() / ref.float().norm()).item() < 1e-3
    torch.testing.assert_close(db.double(), du.double().sum(0), rtol=1e-4, atol=1e-3)
    _, db16 = hip().gelu_backward_colsum(dy, u, torch.bfloat16)
    assert db16.dtype == torch.bfloat16 and ((db16.float() - db).abs() <= db.abs() * 8e-3 + 1e-3).all()


@needs_gpu
def test_comm_emulate_kernel_paces_and_keeps_bucket(H):
    """comm_emu.hip (bench.py --emulate-comm): resident for AT LEAST the modelled time (its waves
    spin on the wall clock until each slice is due -- a one-sided bound: an upper bound would time
    the box's load), copies the requested bytes into the scratch half, never
    writes the bucket."""
    b = torch.randn(4 << 20, device="cuda")  # 16 MiB
    keep = b.clone()
    scratch = torch.zeros_like(b)
    s = torch.cuda.current_stream()
    H.comm_emulate(b, scratch, 1 << 20, 16, 0.0001, s.cuda_stream)  # first launch: code-object load (r4t21: +0.5 ms)
    torch.cuda.synchronize()
    scratch.zero_()
    for secs in (0.0005, 0.004):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        H.comm_emulate(b, scratch, int(b.numel() * 4 * 1.75), 16, secs, s.cuda_stream)
        en.record()
        en.synchronize()
        ms = st.elapsed_time(en)
        assert ms > secs * 1e3 * 0.95, (secs, ms)
    assert torch.equal(b, keep)
    assert torch.equal(scratch, b)  # 1.75 passes cover every element at least once


@needs_gpu
def test_bench_emulate_comm_model():
    """bench.py --emulate-comm 8: every bucket all-reduce becomes the emulator on the comm
    stream; the JSON labels the number a MODEL and reports the emulator's parameters."""
    import json

    e = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "2", "--batch", "32",
                        "--emulate-comm", "8", "--emulate-ctas", "8"], cwd=ROOT, env=e, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["metric"].startswith("MODEL") and res["vs_baseline"] is None, res["metric"]
    em = res["config"]["comm"]["emulated"]
    # calls are counted when the Python step runs: the eager warm-up steps and the capture (the
    # graph replays relaunch the captured emulator kernels without Python)
    hg = res["config"]["hip_graph"]
    total = res["steps"] + res["warmup"]
    eager = total if not hg else total - hg["replays"] + (1 if hg["captured"] else 0)
    assert em["ranks"] == 8 and em["ctas"] == 8 and em["calls"] >= eager * res["config"]["comm"]["buckets"], em
    assert res["config"]["comm"]["comm_plane"] == "emulate"


@needs_gpu
@pytest.mark.parametrize("n,h,w,k,s,p", [(3, 37, 37, 3, 2, 0), (2, 29, 31, 3, 1, 1), (2, 33, 33, 4, 2, 1),
                                         (4, 20, 18, 2, 1, 0), (256, 224, 224, 3, 2, 0)])
def test_stem3_forward_and_wgrad_match_fp32(H, n, h, w, k, s, p):
    """stem3.hip (Inception's Conv2d_1a on MFMA: <= 4x4 window, 3 -> 32 channels): forward from the f32
    image and from bf16, the BN-statistics epilogue, and the deterministic weight gradient -- vs the
    float32 torch convolution of the same bf16-rounded operands."""
    torch.manual_seed(n * 7 + k)
    x = torch.randn(n, 3, h, w, device="cuda").contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(32, 3, k, k, device="cuda") * 0.3).bfloat16().contiguous(memory_format=torch.channels_last)
    xb = x.bfloat16()
    ref = F.conv2d(xb.float(), wt.float(), stride=s, padding=p)
    wp = H.stem3_pack_weight(wt)
    slots = H.conv_stat_slots
    for src in (x, xb):
        st = torch.zeros(slots * 2 * 32, dtype=torch.float64, device="cuda")
        y = H.stem3_forward(src, wp, k, k, s, p, p, st)
        assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
        err = (y.float() - ref).abs().max().item()
        assert err <= 2 ** -7 * ref.abs().max().item() + 1e-3, err
        yd = y.double()
        sums = st.view(slots, 2, 32).sum(0)
        # per-lane partial sums are f32 (as in conv.hip's statistics epilogue), folded in f64
        torch.testing.assert_close(sums[0], yd.sum(dim=(0, 2, 3)), rtol=1e-5, atol=1e-2)
        torch.testing.assert_close(sums[1], (yd * yd).sum(dim=(0, 2, 3)), rtol=1e-5, atol=1e-2)
    dy = torch.randn_like(ref).bfloat16().contiguous(memory_format=torch.channels_last)
    dw = H.stem3_wgrad(dy, xb, k, k, s, p, p, out_f32=True)
    dref = torch.nn.grad.conv2d_weight(xb.float(), wt.shape, dy.float(), stride=s, padding=p)
    assert dw.shape == dref.shape
    assert ((dw - dref).norm() / dref.norm()).item() < 1e-5
    assert torch.equal(dw, H.stem3_wgrad(dy, xb, k, k, s, p, p, out_f32=True))  # no atomics: reproducible
    assert ((H.stem3_wgrad(dy, x, k, k, s, p, p, out_f32=True) - dw).norm() / dw.norm()).item() < 1e-6  # f32 image
    dwb = H.stem3_wgrad(dy, xb, k, k, s, p, p)
    assert dwb.dtype == torch.bfloat16 and torch.equal(dwb, dw.bfloat16())


@needs_gpu
def test_inception_stem_runs_on_stem3(monkeypatch):
    """The fused Inception-v3 takes its 3-channel Conv2d_1a through stem3.hip (not MIOpen): forward +
    backward of a small batch calls it once and produces finite gradients for its weight."""
    import kungfu_amd as kf
    from kungfu_amd.models.inception import inception_v3
    from kungfu_amd.ops import stem as stem_ops
    from kungfu_amd.parallel.mixed import enable_bf16_shadow

    kf.init()
    calls = []
    orig = stem_ops.stem3_conv

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(stem_ops, "stem3_conv", spy)
    torch.manual_seed(0)
    m = inception_v3(fused_bn=True).cuda().to(memory_format=torch.channels_last)
    opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.01),
                                                named_parameters=m.named_parameters())
    enable_bf16_shadow(m, opt)
    x = torch.randn(4, 3, 224, 224, device="cuda").to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (4,), device="cuda")
    opt.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        F.cross_entropy(m(x).float(), y).backward()
    opt.reducer.synchronize()
    assert calls == [1]
    i = opt.space.names.index("stem.0.conv.weight")
    g = opt.space.grad_view(i)
    assert torch.isfinite(g).all() and g.abs().sum() > 0
