"""Model zoo on the CPU: the reference's benchmark models (ResNet-50, VGG-16,
Inception-v3) build, run forward+backward, and the Inception pool-branch rewrite is exact."""
import pytest
import torch
import torch.nn.functional as F

from kungfu_amd.models import get_model
from kungfu_amd.models.inception import BasicConv2d, InceptionA, InceptionC, InceptionE


@pytest.mark.parametrize("name,params_m", [("resnet50", 25.557), ("vgg16", 138.358), ("inception_v3", 23.835)])
def test_model_builds_and_steps(name, params_m):
    torch.manual_seed(0)
    m = get_model(name)
    assert abs(sum(p.numel() for p in m.parameters()) / 1e6 - params_m) < 0.01
    y = m(torch.randn(2, 3, 96 if name != "inception_v3" else 112, 96 if name != "inception_v3" else 112))
    assert y.shape == (2, 1000)
    y.square().mean().backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


@pytest.mark.parametrize("block,args,hw", [(InceptionA, (192, 32), 9), (InceptionC, (768, 128), 5),
                                           (InceptionE, (1280,), 3)])
def test_inception_pool_branch_commutes(block, args, hw):
    """bp(x) = BN/ReLU(avg_pool(conv1x1(x))) equals the textbook BN/ReLU(conv1x1(avg_pool(x)))
    (training-mode BN, f32): the rewrite only moves the pool to the narrower tensor."""
    torch.manual_seed(1)
    b = block(*args)
    x = torch.randn(3, args[0], hw, hw, requires_grad=True)
    bp = b.bp
    assert isinstance(bp, BasicConv2d) and bp.pool_after_conv
    y_new = bp(x)
    y_old = F.relu(F.batch_norm(bp.conv(F.avg_pool2d(x, 3, 1, 1)), None, None, bp.bn.weight, bp.bn.bias,
                                True, 0.0, bp.bn.eps))
    assert torch.allclose(y_new, y_old, rtol=1e-4, atol=1e-5)
    g_new = torch.autograd.grad(y_new.sum(), [x, bp.conv.weight])
    g_old = torch.autograd.grad(y_old.sum(), [x, bp.conv.weight])
    for a, c in zip(g_new, g_old):
        assert torch.allclose(a, c, rtol=1e-3, atol=1e-4)


def test_inception_block_wiring_matches_plain_composition():
    """The Inception blocks' forwards (branch heads grouped for the fused sibling node, BN-link
    chains, the stem run layer by layer) compute exactly the plain composition of their
    modules: every branch in the reference order, concatenated."""
    import torch

    from kungfu_amd.models import get_model
    from kungfu_amd.models import inception as inc

    torch.manual_seed(3)
    m = get_model("inception_v3").eval()

    def seq(mods, x):
        for mod in mods:
            x = mod(x)
        return x

    def plain(b, x):
        if isinstance(b, inc.InceptionA):
            return torch.cat([b.b1(x), seq(b.b5, x), seq(b.b3, x), b.bp(x)], 1)
        if isinstance(b, inc.InceptionB):
            return torch.cat([b.b3(x), seq(b.bd, x), torch.nn.functional.max_pool2d(x, 3, 2)], 1)
        if isinstance(b, inc.InceptionC):
            return torch.cat([b.b1(x), seq(b.b7, x), seq(b.bd, x), b.bp(x)], 1)
        if isinstance(b, inc.InceptionD):
            return torch.cat([seq(b.b3, x), seq(b.b7, x), torch.nn.functional.max_pool2d(x, 3, 2)], 1)
        t3, td = b.b3_1(x), b.bd_2(b.bd_1(x))
        return torch.cat([b.b1(x), b.b3_2a(t3), b.b3_2b(t3), b.bd_3a(td), b.bd_3b(td), b.bp(x)], 1)

    with torch.no_grad():
        x = seq(m.stem, torch.randn(2, 3, 96, 96))
        for b in m.blocks:
            torch.testing.assert_close(b(x), plain(b, x), rtol=0, atol=0)
            x = b(x)
        img = torch.randn(2, 3, 96, 96)
        ref = m.fc(torch.flatten(torch.nn.functional.adaptive_avg_pool2d(seq(m.blocks, seq(m.stem, img)), 1), 1))
        torch.testing.assert_close(m(img), ref, rtol=0, atol=0)
