"""The 224x256 conv tile (csrc/kernels/conv_kernel.hpp variant 8: 28 LDS-DMA pieces of A over 8
waves, the last round partial) against float32 torch references, on 1x1 and 3x3 shapes with the
epilogues the ResNet bottleneck uses: plain, forward BN statistics, BN-backward sums, accumulate
into the masked residual gradient; M not a multiple of the tile included."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
needs_gpu = pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()


def _hip():
    from kungfu_amd._lib import hip

    return hip()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@needs_gpu
@pytest.mark.parametrize("N,H,C,K,ks", [(4, 14, 256, 256, 3), (3, 14, 1024, 256, 1), (2, 9, 64, 512, 1),
                                        (5, 7, 512, 256, 3)])
def test_conv_tile_224_matches_torch(N, H, C, K, ks):
    torch.manual_seed(71)
    Hh = _hip()
    x = _cl(torch.randn(N, C, H, H, device="cuda")).bfloat16()
    w = _cl(torch.randn(K, C, ks, ks, device="cuda") * 0.05).bfloat16()
    ref = F.conv2d(x.float(), w.float(), padding=(ks - 1) // 2)
    y = Hh.conv(x, w, 1, None, None, 8)
    assert _rel(y, ref) < 1e-2
    assert torch.equal(y, Hh.conv(x, w, 1, None, None, 7))  # same K order as the 256x256 tile
    st = torch.zeros(Hh.conv_stat_slots * 2 * K, dtype=torch.float64, device="cuda")
    y2 = Hh.conv(x, w, 1, st, None, 8)
    assert torch.equal(y, y2)
    yd = y2.double().permute(0, 2, 3, 1).reshape(-1, K)
    sums = st.view(-1, 2, K).sum(0)
    torch.testing.assert_close(sums[0], yd.sum(0), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(sums[1], (yd * yd).sum(0), rtol=1e-6, atol=1e-3)


@needs_gpu
@pytest.mark.parametrize("N,H,C,K", [(4, 14, 256, 256), (3, 7, 256, 512)])
def test_conv_tile_224_backward_epilogues(N, H, C, K):
    """BN-backward sums from the forward coefficients, and accumulation into an existing gradient
    through its 1-bit ReLU mask plus BN-backward bits (the identity block's conv1 data gradient)."""
    torch.manual_seed(72)
    Hh = _hip()
    x = _cl(torch.randn(N, C, H, H, device="cuda")).bfloat16()
    w = _cl(torch.randn(K, C, 1, 1, device="cuda") * 0.05).bfloat16()
    ref = F.conv2d(x.float(), w.float())
    bx = _cl(torch.randn(N, K, H, H, device="cuda")).bfloat16()
    fc = torch.cat([torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.2])
    st = torch.zeros(Hh.conv_stat_slots * 2 * K, dtype=torch.float64, device="cuda")
    st7 = torch.zeros_like(st)
    y = Hh.conv(x, w, 1, st, None, 8, bn_x=bx, bn_fcoef=fc)
    y7 = Hh.conv(x, w, 1, st7, None, 7, bn_x=bx, bn_fcoef=fc)
    assert _rel(y, ref) < 1e-2 and torch.equal(y, y7)
    xd = bx.double().permute(0, 2, 3, 1).reshape(-1, K)
    gd = y.double().permute(0, 2, 3, 1).reshape(-1, K)
    dz = torch.where((xd * fc[:K].double() + fc[K:].double()) > 0, gd, torch.zeros_like(gd))
    for t in (st, st7):  # f32 partials per tile: the two tilings agree with f64 sums, not bit for bit
        torch.testing.assert_close(t.view(-1, 2, K).sum(0)[0], dz.sum(0), rtol=1e-6, atol=1e-3)
        torch.testing.assert_close(t.view(-1, 2, K).sum(0)[1], (dz * xd).sum(0), rtol=1e-6, atol=1e-3)
    # accumulate into old * amask (+ BN-backward bits)
    old = _cl(torch.randn(N, K, H, H, device="cuda")).bfloat16()
    amask = torch.randint(0, 256, (old.numel() // 8,), dtype=torch.uint8, device="cuda")
    bmask = torch.randint(0, 256, (old.numel() // 8,), dtype=torch.uint8, device="cuda")
    outs = []
    for v in (8, 7):
        o = old.clone()
        s2 = torch.zeros_like(st)
        Hh.conv(x, w, 1, s2, o, v, bn_x=bx, bn_mask=bmask, acc_mask=amask)
        outs.append((o, s2))
    assert torch.equal(outs[0][0], outs[1][0])
    o = outs[0][0]
    ref_o = (old.float().permute(0, 2, 3, 1).reshape(-1, 8) *
             ((amask.view(-1, 1) >> torch.arange(8, device="cuda")) & 1).float()).reshape(N, H, H, K).permute(0, 3, 1, 2)
    assert _rel(o, ref_o + ref) < 2e-2
    torch.testing.assert_close(outs[0][1].view(-1, 2, K).sum(0), outs[1][1].view(-1, 2, K).sum(0), rtol=1e-5,
                               atol=1e-2)
