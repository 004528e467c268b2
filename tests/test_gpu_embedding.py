"""Embedding gradient by the HIP scatter-add (csrc/kernels/flat_ops.hip embedding_bwd_kernel,
kungfu_amd/ops/embedding.py) against torch's fp32 embedding backward."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dy_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("V,D,shape", [(30522, 768, (32, 128)), (512, 768, (128,)), (2, 64, (4, 16)), (2, 768, (128, 128)),
                                   (97, 4, (3, 5)), (30522, 768, (7, 33))])
def test_embedding_backward_matches_torch(V, D, shape, dy_dtype):
    from kungfu_amd._lib import hip

    g = torch.Generator(device="cuda").manual_seed(3)
    ids = torch.randint(0, V, shape, device="cuda", generator=g)
    if V > 1000:
        ids[0, :64] = 7  # heavy repeats: many atomics on one row
    if V == 2:  # BERT segment ids: long runs of one row
        ids = (torch.arange(shape[-1], device="cuda") >= shape[-1] // 2).long().expand(*shape).contiguous()
    dy = torch.randn(*shape, D, device="cuda", generator=g).to(dy_dtype)
    grad = torch.zeros(V, D, device="cuda")
    hip().embedding_backward(grad, ids.reshape(-1), dy)
    w = torch.zeros(V, D, device="cuda", requires_grad=True)
    F.embedding(ids, w).backward(dy.float())
    # f32 atomics: the summation order is run-dependent.  A row hit n times carries ~eps * sqrt(n) * |row sum|
    # of order noise (BERT segment ids: 8,192 hits per row, sums ~90 -> ~5e-4), so the tolerance scales with it
    n = int(torch.bincount(ids.reshape(-1).clamp_min(0), minlength=V).max())
    atol = max(1e-4, 4e-7 * n ** 0.5 * float(w.grad.abs().max()))
    torch.testing.assert_close(grad, w.grad, rtol=1e-5, atol=atol)


def test_embedding_backward_skips_out_of_range_ids():
    from kungfu_amd._lib import hip

    ids = torch.tensor([0, 5, -1, 9, 2], device="cuda")
    dy = torch.ones(5, 8, device="cuda")
    grad = torch.zeros(4, 8, device="cuda")
    hip().embedding_backward(grad, ids, dy)
    assert grad[0].eq(1).all() and grad[2].eq(1).all() and grad[1].eq(0).all() and grad[3].eq(0).all()


def test_embedding_op_autograd_and_graph_replay():
    """ops.embedding gives torch's gradients, and a captured forward+backward replays with new ids."""
    from kungfu_amd.ops.embedding import embedding

    V, D = 1000, 128
    w = torch.randn(V, D, device="cuda", requires_grad=True)
    ids = torch.randint(0, V, (8, 64), device="cuda")
    (embedding(ids, w) * 2).sum().backward()
    ref = torch.zeros(V, D, device="cuda")
    ref.index_add_(0, ids.reshape(-1), torch.full((ids.numel(), D), 2.0, device="cuda"))
    torch.testing.assert_close(w.grad, ref)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            w.grad = None
            embedding(ids, w).sum().backward()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    w.grad = None
    with torch.cuda.graph(gr):
        embedding(ids, w).sum().backward()
    for _ in range(3):
        ids.copy_(torch.randint(0, V, (8, 64), device="cuda"))
        gr.replay()
        torch.cuda.synchronize()
        ref = torch.zeros(V, D, device="cuda")
        ref.index_add_(0, ids.reshape(-1), torch.ones(ids.numel(), D, device="cuda"))
        torch.testing.assert_close(w.grad, ref)


@pytest.mark.parametrize("R,V", [(2560, 30522), (7, 2), (33, 1000)])
def test_fused_cross_entropy_matches_torch(R, V):
    """ops.xent.cross_entropy (csrc/kernels/xent.hip) vs F.cross_entropy on the f32 copy of the same
    bf16 logits: loss to f32 rounding, logit gradient to one bf16 rounding; ignore_index rows."""
    from kungfu_amd.ops.xent import cross_entropy

    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.randn(R, V, device="cuda", generator=g) * 4).bfloat16().requires_grad_(True)
    lab = torch.randint(0, V, (R,), device="cuda", generator=g)
    lab[::5] = -100
    loss = cross_entropy(x, lab)
    loss.backward(torch.tensor(3.0, device="cuda"))
    xr = x.detach().float().requires_grad_(True)
    ref = F.cross_entropy(xr, lab)
    ref.backward(torch.tensor(3.0, device="cuda"))
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad.float(), xr.grad.bfloat16().float(), rtol=1e-2, atol=1e-6)
    assert x.grad[::5].abs().sum().item() == 0.0


@pytest.mark.parametrize("R,V", [(2560, 30522), (33, 1000), (9, 13)])
def test_fused_cross_entropy_padded_rows(R, V):
    """The 16-byte-load kernels over logits rows padded to ld (a [R, V] view of [R, ld], the vocabulary
    projection's layout; junk in the padding): same loss / gradient as the contiguous path's reference,
    and the gradient comes back with the same padded row stride, its last-chunk padding zero."""
    from kungfu_amd.ops.xent import cross_entropy

    ld = (V + 7) // 8 * 8 + 8
    g = torch.Generator(device="cuda").manual_seed(2)
    base = (torch.randn(R, ld, device="cuda", generator=g) * 4).bfloat16()
    base[:, V:] = 1e4  # must never be read as a class
    x = base[:, :V]
    lab = torch.randint(0, V, (R,), device="cuda", generator=g)
    lab[::4] = -100
    xg = x.detach().requires_grad_(True)
    loss = cross_entropy(xg, lab)
    loss.backward(torch.tensor(2.0, device="cuda"))
    xr = x.detach().float().requires_grad_(True)
    ref = F.cross_entropy(xr, lab)
    ref.backward(torch.tensor(2.0, device="cuda"))
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(xg.grad.float(), xr.grad.bfloat16().float(), rtol=1e-2, atol=1e-6)
    from kungfu_amd._lib import hip

    lse = hip().xent_forward(x, lab)[0]
    dx = hip().xent_backward(x, lab, lse, torch.ones(1, device="cuda"))
    assert dx.stride() == (ld, 1)
    full = dx.as_strided((R, ld), (ld, 1))
    assert full[:, V:(V + 7) // 8 * 8].abs().sum().item() == 0.0


def test_vocab_projection_matches_fp32():
    """ops.vocab.vocab_projection (gemm.hip ragged-N GEMM, padded logits rows) + cross_entropy vs
    F.linear + F.cross_entropy in f32 on the same bf16 operands: loss, d h, d W, d b."""
    from kungfu_amd.ops.vocab import vocab_projection
    from kungfu_amd.ops.xent import cross_entropy

    torch.manual_seed(5)
    M, V, D = 300, 30522, 768
    h = (torch.randn(4, M // 4, D, device="cuda")).bfloat16().requires_grad_(True)
    w = (torch.randn(V, D, device="cuda") * 0.02).requires_grad_(True)  # f32 master, as the tied embedding
    b = (torch.randn(V, device="cuda") * 0.1).requires_grad_(True)
    lab = torch.randint(0, V, (4, M // 4), device="cuda")
    with torch.autocast("cuda", dtype=torch.bfloat16):
        logits = vocab_projection(h, w, b)
        assert logits.shape == (4, M // 4, V) and logits.dtype == torch.bfloat16
        loss = cross_entropy(logits, lab)
    loss.backward()
    hr = h.detach().float().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().bfloat16().float().requires_grad_(True)
    lr = F.linear(hr, wr, br)
    ref = F.cross_entropy(lr.reshape(-1, V), lab.reshape(-1))
    ref.backward()
    torch.testing.assert_close(logits.float(), lr.detach(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(loss.float(), ref, rtol=2e-3, atol=2e-3)
    for got, want in ((h.grad, hr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        rel = ((got.float() - want).norm() / want.norm()).item()
        assert rel < 2e-2, rel
