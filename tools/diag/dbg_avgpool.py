import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch, torch.nn.functional as F
from kungfu_amd._lib import hip
from kungfu_amd.ops.pool import avg_pool3x3s1
H = hip()
torch.manual_seed(0)
x = torch.randn(1, 8, 5, 5, device="cuda").bfloat16().to(memory_format=torch.channels_last)
print("fwd", (H.avgpool3s1(x).float() - F.avg_pool2d(x.float(), 3, 1, 1)).abs().max().item())
dy = torch.randn(1, 8, 5, 5, device="cuda").bfloat16().to(memory_format=torch.channels_last)
xr = x.float().requires_grad_(True)
F.avg_pool2d(xr, 3, 1, 1).backward(dy.float())
print("stencil-on-dy vs torch grad", (H.avgpool3s1(dy).float() - xr.grad).abs().max().item())
xa = x.clone().requires_grad_(True)
avg_pool3x3s1(xa).backward(dy)
print("autograd vs torch grad", (xa.grad.float() - xr.grad).abs().max().item())
print(xr.grad[0, 0], xa.grad[0, 0].float(), dy[0, 0].float(), sep="\n")
