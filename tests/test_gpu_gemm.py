"""Linear-layer GEMM on the MFMA kernel (csrc/kernels/conv.hip launch_gemm) with its epilogues,
against plain PyTorch fp32 references of the same ops."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _hip():
    from kungfu_amd._lib import hip

    return hip()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("M,K,N", [(4096, 768, 2304), (1000, 768, 768), (2048, 3072, 768), (520, 256, 192)])
@pytest.mark.parametrize("variant", [-1, 0, 1, 2, 3])
def test_gemm_plain_bias_gelu(M, K, N, variant):
    H = _hip()
    if variant in (0, 3) and N % 256:
        pytest.skip("256-wide tile")
    torch.manual_seed(3)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    ref = x.float() @ w.float().t()
    y = H.gemm(x, w, variant=variant)[0]
    assert y.shape == (M, N) and _rel(y, ref) < 1e-2
    yb = H.gemm(x, w, b, variant=variant)[0]
    assert _rel(yb, ref + b.float()) < 1e-2
    g, u = H.gemm(x, w, b, True, variant=variant)
    assert _rel(u, ref + b.float()) < 1e-2
    # gelu applied to the bf16 pre-activation, as torch's bf16 F.gelu does
    assert _rel(g, F.gelu(u.float())) < 1e-2
    assert (g.float() - F.gelu(u.float())).abs().max().item() < 0.05


@pytest.mark.parametrize("M,K,N", [(4096, 3072, 768), (1000, 768, 3072), (520, 768, 64)])
def test_gemm_gelu_grad_and_bias_sums(M, K, N):
    """dy @ W with the GELU-gradient gate of the pre-activation u and the column sums of the
    gated result (the bias gradient of the layer that produced u)."""
    H = _hip()
    torch.manual_seed(5)
    dy = torch.randn(M, K, device="cuda").bfloat16()
    wt = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    u = (torch.randn(M, N, device="cuda") * 2).bfloat16()
    st = torch.zeros(H.conv_stat_slots * 2 * N, dtype=torch.float64, device="cuda")
    du = H.gemm(dy, wt, gelu_u=u, stats=st)[0]
    uf = u.float().requires_grad_(True)
    F.gelu(uf).backward(dy.float() @ wt.float().t())
    assert _rel(du, uf.grad) < 1.5e-2
    db = st.view(H.conv_stat_slots, 2, N)[:, 0].sum(0)
    # sums of the bf16 outputs the kernel wrote
    assert _rel(db, du.double().sum(0)) < 1e-5
    assert _rel(db, uf.grad.double().sum(0)) < 2e-2


def test_gemm_accumulate():
    H = _hip()
    torch.manual_seed(7)
    x = torch.randn(3000, 768, device="cuda").bfloat16()
    w = (torch.randn(768, 768, device="cuda") / 28).bfloat16()
    out = torch.randn(3000, 768, device="cuda").bfloat16()
    ref = out.float() + x.float() @ w.float().t()
    y = H.gemm(x, w, out=out)[0]
    assert y.data_ptr() == out.data_ptr() and _rel(out, ref) < 1e-2
