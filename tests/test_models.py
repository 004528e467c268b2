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
