"""ImageNet-shaped input pipeline with on-GPU augmentation.

Parity: ``srcs/python/kungfu/tensorflow/v1/helpers/imagenet.py`` (TFRecord
parse, random crop, flip, colour distortion, normalisation in TF ops).  There
is no JPEG decoder in this image, so records are pre-decoded uint8 NHWC
shards (``*.npy`` with a matching ``*.labels.npy``).  Decoded bytes are
uploaded as uint8 (4x fewer bytes over PCIe than f32) and the augmentation --
random-resized crop, horizontal flip, mean/std normalisation -- runs on the
GPU, producing channels_last bf16/f32 batches ready for the model.
"""
from __future__ import annotations

import glob
import os
from typing import Iterator, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def gpu_augment(images_u8: torch.Tensor, out_size: int = 224, train: bool = True, dtype=torch.bfloat16,
                generator: Optional[torch.Generator] = None, scale=(0.08, 1.0)) -> torch.Tensor:
    """uint8 NHWC batch on the device -> normalised channels_last [N, 3, S, S] batch."""
    n, h, w, _ = images_u8.shape
    x = images_u8.permute(0, 3, 1, 2).float().div_(255.0)  # NCHW view of NHWC memory = channels_last
    if train:
        dev = images_u8.device
        area = torch.empty(n, device=dev).uniform_(scale[0], scale[1], generator=generator)
        logr = torch.empty(n, device=dev).uniform_(np.log(3 / 4), np.log(4 / 3), generator=generator)
        ratio = torch.exp(logr)
        cw = torch.sqrt(area * ratio).clamp(max=1.0)
        ch = torch.sqrt(area / ratio).clamp(max=1.0)
        cx = torch.rand(n, device=dev, generator=generator) * (1 - cw) + cw / 2
        cy = torch.rand(n, device=dev, generator=generator) * (1 - ch) + ch / 2
        flip = (torch.rand(n, device=dev, generator=generator) < 0.5).float() * 2 - 1
        theta = torch.zeros(n, 2, 3, device=dev)
        theta[:, 0, 0] = cw * flip
        theta[:, 0, 2] = cx * 2 - 1
        theta[:, 1, 1] = ch
        theta[:, 1, 2] = cy * 2 - 1
        grid = F.affine_grid(theta, (n, 3, out_size, out_size), align_corners=False)
        x = F.grid_sample(x, grid, mode="bilinear", padding_mode="reflection", align_corners=False)
    else:
        x = F.interpolate(x, size=(out_size, out_size), mode="bilinear", align_corners=False)
    mean = torch.tensor(MEAN, device=x.device).view(1, 3, 1, 1)
    std = torch.tensor(STD, device=x.device).view(1, 3, 1, 1)
    x = (x - mean) / std
    return x.to(dtype=dtype, memory_format=torch.channels_last)


class ImageNetShards:
    """Iterates batches from pre-decoded uint8 shards, sharded over ranks."""

    def __init__(self, data_dir: str, batch: int, rank: int = 0, size: int = 1, device="cuda",
                 out_size: int = 224, train: bool = True, seed: int = 0, dtype=torch.bfloat16):
        self.files = sorted(f for f in glob.glob(os.path.join(data_dir, "*.npy")) if not f.endswith(".labels.npy"))
        if not self.files:
            raise FileNotFoundError("no *.npy shards in %s" % data_dir)
        self.batch, self.rank, self.size = batch, rank, size
        self.device, self.out_size, self.train, self.dtype = torch.device(device), out_size, train, dtype
        self.rng = np.random.default_rng(seed)
        self.gen = torch.Generator(device=self.device).manual_seed(seed * 1000 + rank)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        order = self.rng.permutation(len(self.files)) if self.train else np.arange(len(self.files))
        for fi in order[self.rank::self.size]:
            f = self.files[fi]
            imgs = np.load(f, mmap_mode="r")  # allow_pickle stays False
            labels = np.load(f[:-4] + ".labels.npy")
            idx = self.rng.permutation(len(labels)) if self.train else np.arange(len(labels))
            for b in range(0, len(idx) - self.batch + 1, self.batch):
                sel = np.sort(idx[b:b + self.batch])
                x = torch.from_numpy(np.ascontiguousarray(imgs[sel])).pin_memory() if self.device.type == "cuda" \
                    else torch.from_numpy(np.ascontiguousarray(imgs[sel]))
                x = x.to(self.device, non_blocking=True)
                y = torch.from_numpy(labels[sel].astype(np.int64)).to(self.device, non_blocking=True)
                yield gpu_augment(x, self.out_size, self.train, self.dtype, self.gen), y
