"""Synthetic ImageNet-shaped batches resident on the device (bench input)."""
from __future__ import annotations

import torch


class SyntheticImageNet:
    def __init__(self, batch: int, device, image_size: int = 224, classes: int = 1000, channels_last: bool = True,
                 dtype=torch.float32, seed: int = 0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        x = torch.randn(batch, 3, image_size, image_size, generator=g, dtype=dtype)
        self.x = x.to(device)
        if channels_last:
            self.x = self.x.to(memory_format=torch.channels_last)
        self.y = torch.randint(0, classes, (batch,), generator=g).to(device)

    def __iter__(self):
        while True:
            yield self.x, self.y
