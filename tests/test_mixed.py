"""bf16 shadow weights + direct gradients (kungfu_amd/parallel/mixed.py) vs stock autocast.

CPU: the default immediate sink; bf16 autocast on CPU gives the same weight
cast (round-to-nearest-even) and the same bf16 weight gradients, so the f32
gradients must match the stock path exactly.
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from kungfu_amd.parallel.flat import FlatParamSpace
from kungfu_amd.parallel import mixed


class Tiny(nn.Module):
    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2d(3, 8, 3, padding=1, bias=False)
        self.bn = nn.BatchNorm2d(8)
        self.c2 = nn.Conv2d(8, 8, 1, bias=True)
        self.fc = nn.Linear(8, 5)

    def forward(self, x):
        x = F.relu(self.bn(self.c1(x)))
        x = self.c2(x)
        return self.fc(x.mean((2, 3)))


def _grads(model, x, y):
    with torch.autocast("cpu", dtype=torch.bfloat16):
        out = model(x)
    loss = F.cross_entropy(out.float(), y)
    loss.backward()
    return loss.detach(), {n: p.grad.detach().clone() for n, p in model.named_parameters()}


def test_shadow_matches_autocast_cpu():
    torch.manual_seed(0)
    m1 = Tiny()
    m2 = Tiny()
    m2.load_state_dict(m1.state_dict())
    x = torch.randn(4, 3, 8, 8)
    y = torch.randint(0, 5, (4,))
    l1, g1 = _grads(m1, x, y)

    space = FlatParamSpace(m2.parameters())
    n = mixed.enable_bf16_shadow(m2, space)
    assert n == 5  # c1.w, c2.w, c2.b, fc.w, fc.b
    assert isinstance(space.sink, mixed.ImmediateSink)
    for _ in range(2):  # grads accumulate across backwards like .grad does
        space.zero_grad()
        l2, g2 = _grads(m2, x, y)
        assert torch.equal(l1, l2)
        for k in g1:
            torch.testing.assert_close(g2[k], g1[k], rtol=0, atol=0)
    # the master weights changed -> next forward refreshes the shadow
    with torch.no_grad():
        space.flat_param.mul_(0.5)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        o = m2(x)
    assert torch.equal(space.flat_shadow, space.flat_param.bfloat16())
    assert o.dtype == torch.bfloat16
    mixed.disable(m2)
    assert "forward" not in m2.c1.__dict__


def test_shadow_inactive_without_autocast():
    torch.manual_seed(0)
    m = Tiny()
    space = FlatParamSpace(m.parameters())
    mixed.enable_bf16_shadow(m, space)
    x = torch.randn(2, 3, 8, 8)
    out = m(x)  # no autocast: f32 weights, stock AccumulateGrad path into the flat views
    assert out.dtype == torch.float32
    out.sum().backward()
    assert m.c1.weight.grad.data_ptr() == space.grad_view(space.index(m.c1.weight)).data_ptr()
    assert m.c1.weight.grad.abs().sum() > 0
    mixed.disable(m)


def test_shadow_two_forwards_then_backwards_cpu():
    """Gradient accumulation with both graphs alive: the per-forward shadow refresh
    must not invalidate the first graph's saved bf16 weights."""
    torch.manual_seed(1)
    m1, m2 = Tiny(), Tiny()
    m2.load_state_dict(m1.state_dict())
    xs = [torch.randn(2, 3, 8, 8) for _ in range(2)]
    space = FlatParamSpace(m2.parameters())
    mixed.enable_bf16_shadow(m2, space)
    for m in (m1, m2):
        with torch.autocast("cpu", dtype=torch.bfloat16):
            outs = [m(x).float().sum() for x in xs]
        for o in outs:
            o.backward()
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        torch.testing.assert_close(b.grad, a.grad, rtol=0, atol=0, msg=n)
    mixed.disable(m2)
