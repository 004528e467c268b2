"""MNIST loader (idx files) and a deterministic MNIST-shaped synthetic set.

Parity: ``srcs/python/kungfu/tensorflow/v1/helpers/{mnist,idx}.py``.  There is
no network here, so when ``KUNGFU_MNIST_DIR`` (or ``data_dir``) does not hold
the four idx files, :func:`synthetic_mnist` generates separable 28x28
10-class data with a fixed seed instead.
"""
from __future__ import annotations

import gzip
import os
import struct
from typing import Optional, Tuple

import numpy as np
import torch

_FILES = {
    "train_x": "train-images-idx3-ubyte", "train_y": "train-labels-idx1-ubyte",
    "test_x": "t10k-images-idx3-ubyte", "test_y": "t10k-labels-idx1-ubyte",
}


def read_idx(path: str) -> np.ndarray:
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        magic = struct.unpack(">I", f.read(4))[0]
        ndim = magic & 0xFF
        dtype = {0x08: np.uint8, 0x09: np.int8, 0x0B: np.int16, 0x0C: np.int32, 0x0D: np.float32,
                 0x0E: np.float64}[(magic >> 8) & 0xFF]
        shape = struct.unpack(">" + "I" * ndim, f.read(4 * ndim))
        return np.frombuffer(f.read(), dtype=np.dtype(dtype).newbyteorder(">")).reshape(shape)


def load_mnist(data_dir: Optional[str] = None, normalize: bool = True):
    data_dir = data_dir or os.environ.get("KUNGFU_MNIST_DIR", "")
    paths = {}
    for k, f in _FILES.items():
        for cand in (f, f + ".gz"):
            p = os.path.join(data_dir, cand)
            if data_dir and os.path.exists(p):
                paths[k] = p
    if len(paths) != 4:
        return None
    out = {}
    for k, p in paths.items():
        a = read_idx(p)
        t = torch.from_numpy(a.astype(np.float32 if k.endswith("x") else np.int64))
        if k.endswith("x") and normalize:
            t = t / 255.0
        out[k] = t
    return out


def synthetic_mnist(n_train: int = 6000, n_test: int = 1000, seed: int = 0) -> dict:
    g = torch.Generator().manual_seed(seed)
    centers = torch.rand(10, 28 * 28, generator=g)

    def make(n):
        y = torch.randint(0, 10, (n,), generator=g)
        x = (centers[y] * 0.15 + torch.rand(n, 28 * 28, generator=g) * 0.85 - 0.5).clamp(min=0).reshape(n, 28, 28)
        return x, y

    tx, ty = make(n_train)
    vx, vy = make(n_test)
    return {"train_x": tx, "train_y": ty, "test_x": vx, "test_y": vy}
