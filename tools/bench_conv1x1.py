"""Microbench: ResNet-50 1x1 convolutions (NHWC bf16) via MIOpen conv vs plain GEMM (hipBLASLt),
forward + backward (dX, dW).  Prints one line per shape."""
import time, torch, torch.nn.functional as F
torch.backends.cudnn.benchmark = False
dev = torch.device("cuda")
B = 256
shapes = [  # (H, Cin, Cout, stride)
    (56, 64, 64, 1), (56, 64, 256, 1), (56, 256, 64, 1), (56, 256, 128, 1), (28, 128, 512, 1), (28, 512, 128, 1),
    (28, 512, 256, 1), (14, 256, 1024, 1), (14, 1024, 256, 1), (14, 1024, 512, 1), (7, 512, 2048, 1), (7, 2048, 512, 1),
]
def timeit(f, n=10):
    f(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3
tot_conv = tot_gemm = 0
for H, Ci, Co, s in shapes:
    x = torch.randn(B, Ci, H, H, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
    w = torch.randn(Co, Ci, 1, 1, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
    g = torch.randn(B, Co, H, H, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    def conv():
        y = F.conv2d(x, w); y.backward(g)
    X = x.detach().permute(0, 2, 3, 1).reshape(-1, Ci); W = w.detach().reshape(Co, Ci); G = g.permute(0, 2, 3, 1).reshape(-1, Co)
    def gemm():
        y = X @ W.t(); dx = G @ W; dw = G.t() @ X
    tc, tg = timeit(conv), timeit(gemm)
    fl = 3 * 2 * B * H * H * Ci * Co
    tot_conv += tc; tot_gemm += tg
    print("H=%3d Ci=%4d Co=%4d conv %.3f ms (%.0f TF)  gemm %.3f ms (%.0f TF)" % (H, Ci, Co, tc, fl / tc / 1e9, tg, fl / tg / 1e9), flush=True)
print("total conv %.2f ms gemm %.2f ms" % (tot_conv, tot_gemm))
