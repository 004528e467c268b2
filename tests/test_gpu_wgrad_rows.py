"""Row-image weight gradient for stride-1 KH x KW windows and channel counts % 8
(csrc/kernels/conv_wgrad.hip wgrad_rows_rect_kernel, ``conv_wgrad_rect(..., variant=6)`` on 64-channel
tiles; ``variant=8..12``: segments sized for the fewest staged rows, a 2-4 stage LDS ring, 32- or
64-channel tiles, dw-layout split partials) against an fp32 PyTorch reference of the same weight
gradient."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


CASES = [
    # N, H, W, Cin, Cout, kh, kw, ph, pw
    (4, 25, 25, 48, 64, 5, 5, 2, 2),
    (4, 25, 25, 96, 96, 3, 3, 1, 1),
    (4, 25, 25, 64, 96, 3, 3, 1, 1),
    (3, 12, 12, 160, 192, 1, 7, 0, 3),
    (3, 12, 12, 192, 160, 7, 1, 3, 0),
    (2, 54, 54, 80, 192, 3, 3, 0, 0),
    (2, 70, 70, 32, 64, 3, 3, 1, 1),     # OW >= 64: two segments per row, the second partial
    (2, 71, 71, 32, 32, 3, 3, 0, 0),
    (5, 9, 9, 24, 40, 3, 3, 1, 1),       # channel counts below one tile
    (16, 25, 25, 48, 64, 5, 5, 2, 2),    # many segments: split-K + reduce
    (2, 111, 111, 32, 32, 3, 3, 0, 0),   # Conv2d_2a's 109-wide rows: 32-tile segments of R > 1 rows
]


@pytest.mark.parametrize("variant", [6, 8, 9, 10, 11, 12, 13])
@pytest.mark.parametrize("N,H,W,cin,cout,kh,kw,ph,pw", CASES)
def test_wgrad_rows_rect_matches_fp32(N, H, W, cin, cout, kh, kw, ph, pw, variant):
    from kungfu_amd._lib import hip

    Hh = hip()
    assert Hh.conv_wgrad_rows_rect_supported(N, H, W, cin, cout, kh, kw, ph, pw, 1)
    torch.manual_seed(11)
    x = _cl(torch.randn(N, cin, H, W, device="cuda").bfloat16())
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    dy = _cl(torch.randn(N, cout, oh, ow, device="cuda").bfloat16())
    dw = Hh.conv_wgrad_rect(dy, x, kh, kw, 1, ph, pw, variant)
    assert torch.equal(dw, Hh.conv_wgrad_rect(dy, x, kh, kw, 1, ph, pw, variant))  # no atomics: reproducible
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, kh, kw), dy.float(), 1, (ph, pw))
    assert dw.shape == ref.shape
    rel = ((dw.float() - ref).norm() / ref.norm()).item()
    assert rel < 1e-2, rel
    # and the tap-tiled kernel agrees (same f32 accumulation, different order)
    dw2 = Hh.conv_wgrad_rect(dy, x, kh, kw, 1, ph, pw)
    assert ((dw.float() - dw2.float()).norm() / ref.norm()).item() < 1e-2


S2_CASES = [
    # N, H, W, Cin, Cout, kh, kw, ph, pw: Inception's stride-2 narrow layers (Mixed_6a / 7a), small N
    (4, 25, 25, 96, 96, 3, 3, 0, 0),
    (4, 12, 12, 192, 320, 3, 3, 0, 0),
    (3, 12, 12, 192, 192, 3, 3, 0, 0),
    (2, 33, 31, 32, 48, 3, 3, 1, 1),
    (2, 20, 20, 40, 24, 5, 5, 2, 2),
]


@pytest.mark.parametrize("variant", [8, 11, 12, 13])
@pytest.mark.parametrize("N,H,W,cin,cout,kh,kw,ph,pw", S2_CASES)
def test_wgrad_rows_rect_stride2_matches_fp32(N, H, W, cin, cout, kh, kw, ph, pw, variant):
    """The segment-sized ring variants on stride 2: output (r, c) reads image row 2r + kh, column 2c + kw."""
    from kungfu_amd._lib import hip

    Hh = hip()
    assert Hh.conv_wgrad_rows_rect_supported(N, H, W, cin, cout, kh, kw, ph, pw, 2)
    torch.manual_seed(12)
    x = _cl(torch.randn(N, cin, H, W, device="cuda").bfloat16())
    oh, ow = (H + 2 * ph - kh) // 2 + 1, (W + 2 * pw - kw) // 2 + 1
    dy = _cl(torch.randn(N, cout, oh, ow, device="cuda").bfloat16())
    dw = Hh.conv_wgrad_rect(dy, x, kh, kw, 2, ph, pw, variant)
    assert torch.equal(dw, Hh.conv_wgrad_rect(dy, x, kh, kw, 2, ph, pw, variant))
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, kh, kw), dy.float(), 2, (ph, pw))
    rel = ((dw.float() - ref).norm() / ref.norm()).item()
    assert rel < 1e-2, rel


def test_wgrad_rows_rect_auto_picks():
    """conv_wgrad_rows_rect_auto on Inception-v3's narrow shapes (batch 256): host-side rule."""
    from kungfu_amd._lib import hip

    Hh = hip()
    assert Hh.conv_wgrad_rows_rect_auto(256, 111, 111, 32, 32, 3, 3, 0, 0, 1) == 8
    assert Hh.conv_wgrad_rows_rect_auto(256, 12, 12, 128, 128, 1, 7, 0, 3, 1) == 6
    assert Hh.conv_wgrad_rows_rect_auto(256, 54, 54, 80, 192, 3, 3, 0, 0, 1) == 11
    assert Hh.conv_wgrad_rows_rect_auto(256, 25, 25, 96, 96, 3, 3, 1, 1, 1) == 12
    assert Hh.conv_wgrad_rows_rect_auto(256, 25, 25, 96, 96, 3, 3, 0, 0, 2) == 10
    assert Hh.conv_wgrad_rows_rect_auto(256, 25, 25, 288, 384, 3, 3, 0, 0, 2) == 8
    assert Hh.conv_wgrad_rows_rect_auto(256, 12, 12, 192, 320, 3, 3, 0, 0, 2) == 12
