"""Minimal driver for rocprofv3 --pmc passes over the row-image weight gradient
(conv_wgrad.hip wgrad_rows_rect_kernel): Inception shape SHAPE (argv[1]: 0 Conv2d_2a 111x111
32->32 3x3, 1 Conv2d_2b 109x109 32->64 3x3 pad 1, 2 Conv2d_4a 54x54 80->192 3x3, 3 Mixed_5 25x25
96->96 3x3 pad 1, 4 Mixed_6 12x12 160->160 1x7) at batch 256, variant argv[2] (6: 64-channel tiles,
8: 32-channel tiles), 5 calls."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kungfu_amd._lib import hip  # noqa: E402

SHAPES = [(111, 32, 32, 3, 3, 0, 0), (109, 32, 64, 3, 3, 1, 1), (54, 80, 192, 3, 3, 0, 0), (25, 96, 96, 3, 3, 1, 1),
          (12, 160, 160, 1, 7, 0, 3)]
hw, cin, cout, kh, kw, ph, pw = SHAPES[int(sys.argv[1])]
variant = int(sys.argv[2])
N = 256
CL = torch.channels_last
x = torch.randn(N, cin, hw, hw, device="cuda").bfloat16().contiguous(memory_format=CL)
oh, ow = hw + 2 * ph - kh + 1, hw + 2 * pw - kw + 1
dy = torch.randn(N, cout, oh, ow, device="cuda").bfloat16().contiguous(memory_format=CL)
H = hip()
for _ in range(5):
    H.conv_wgrad_rect(dy, x, kh, kw, 1, ph, pw, variant)
torch.cuda.synchronize()
print("done", sys.argv[1:])
