"""Row-image stride-1 3x3 convolution (csrc/kernels/conv_kernel.hpp conv_rows_kernel, variants
20-23 of the conv binding) against float32 torch references: the output, the forward BN
statistics epilogue (vs float64 sums of the output) and the BN-backward-sums epilogue (vs float64
sums of the gated gradient), on shapes whose tiles straddle image boundaries and end past M."""
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


# (variant, N, H, Cin, Cout): 20 / 23 need Cin = 64 (one image buffer); odd N and small maps put
# image boundaries and the end of M inside tiles
CASES = [(20, 3, 56, 64, 64), (20, 5, 9, 64, 64), (23, 3, 56, 64, 64), (23, 2, 13, 64, 128), (24, 3, 56, 64, 64),
         (25, 3, 56, 64, 64), (25, 2, 13, 64, 128),
         (21, 3, 28, 128, 128), (21, 5, 14, 256, 256), (21, 3, 7, 512, 512), (21, 2, 11, 192, 128),
         (22, 3, 28, 128, 128), (22, 4, 7, 512, 512), (22, 3, 10, 64, 256)]


@needs_gpu
@pytest.mark.parametrize("variant,N,H,C,K", CASES)
def test_conv_rows_forward_stats(variant, N, H, C, K):
    torch.manual_seed(61)
    Hh = _hip()
    x = _cl(torch.randn(N, C, H, H, device="cuda")).bfloat16()
    w = _cl(torch.randn(K, C, 3, 3, device="cuda") * 0.05).bfloat16()
    ref = F.conv2d(x.float(), w.float(), padding=1)
    y = Hh.conv(x, w, 1, None, None, variant)
    assert _rel(y, ref) < 1e-2
    st = torch.zeros(Hh.conv_stat_slots * 2 * K, dtype=torch.float64, device="cuda")
    y2 = Hh.conv(x, w, 1, st, None, variant)
    assert torch.equal(y, y2)
    sums = st.view(-1, 2, K).sum(0)
    yd = y2.double().permute(0, 2, 3, 1).reshape(-1, K)
    torch.testing.assert_close(sums[0], yd.sum(0), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(sums[1], (yd * yd).sum(0), rtol=1e-6, atol=1e-3)


@needs_gpu
@pytest.mark.parametrize("variant,N,H,C,K", [(20, 3, 56, 64, 64), (23, 2, 13, 128, 64), (21, 3, 28, 128, 128),
                                             (21, 5, 14, 256, 256), (22, 4, 7, 512, 512), (22, 3, 10, 256, 64)])
def test_conv_rows_data_gradient_bn_sums(variant, N, H, C, K):
    """The stride-1 data gradient (the conv on flipped weights) with the BN-backward-sums epilogue
    of the BN(+ReLU) whose input is bn_x: dz = grad * relu'(bn_x * scale + shift)."""
    torch.manual_seed(62)
    Hh = _hip()
    dy = _cl(torch.randn(N, K, H, H, device="cuda")).bfloat16()
    w = _cl(torch.randn(K, C, 3, 3, device="cuda") * 0.05).bfloat16()
    wt = Hh.conv_flip_weight(w)
    bx = _cl(torch.randn(N, C, H, H, device="cuda")).bfloat16()
    fc = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2])
    st = torch.zeros(Hh.conv_stat_slots * 2 * C, dtype=torch.float64, device="cuda")
    dx = Hh.conv(dy, wt, 1, st, None, variant, bn_x=bx, bn_fcoef=fc)
    ref = torch.nn.grad.conv2d_input(bx.shape, w.float(), dy.float(), padding=1)
    assert _rel(dx, ref) < 1e-2
    if K == 64:  # one channel chunk: the tap-wise kernel sums in the same order -> same bits
        assert torch.equal(dx, Hh.conv(dy, wt, 1, None, None, 2))
    xd = bx.double().permute(0, 2, 3, 1).reshape(-1, C)
    gd = dx.double().permute(0, 2, 3, 1).reshape(-1, C)
    on = (xd * fc[:C].double() + fc[C:].double()) > 0
    dz = torch.where(on, gd, torch.zeros_like(gd))
    sums = st.view(-1, 2, C).sum(0)
    torch.testing.assert_close(sums[0], dz.sum(0), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(sums[1], (dz * xd).sum(0), rtol=1e-6, atol=1e-3)


@needs_gpu
def test_conv_rows_rejects_unsupported():
    Hh = _hip()
    x = _cl(torch.randn(2, 128, 8, 8, device="cuda")).bfloat16()
    w = _cl(torch.randn(128, 128, 3, 3, device="cuda") * 0.05).bfloat16()
    with pytest.raises(Exception):
        Hh.conv(x, w, 1, None, None, 20)  # Cin != 64 on the one-buffer variant
    with pytest.raises(Exception):
        Hh.conv(x, w, 2, None, None, 21)  # stride 2
