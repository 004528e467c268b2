"""Dataset helpers: CIFAR binary records, ImageNet shards + augmentation, elastic shard ranges."""
import os

import numpy as np
import torch

from kungfu_amd.datasets import Cifar10Loader, ImageNetShards, gpu_augment, shard_range
from kungfu_amd.datasets.cifar import write_cifar10_binary


def test_cifar10_binary_roundtrip(tmp_path):
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (12, 32, 32, 3), dtype=np.uint8)
    lab = rng.integers(0, 10, 12)
    for i in range(1, 6):
        write_cifar10_binary(str(d / ("data_batch_%d.bin" % i)), imgs, lab)
    write_cifar10_binary(str(d / "test_batch.bin"), imgs, lab)
    ds = Cifar10Loader(str(tmp_path), normalize=False, one_hot=False).load_datasets()
    assert ds.train.images.shape == (60, 32, 32, 3) and ds.train.images.dtype == np.uint8
    assert np.array_equal(ds.test.images, imgs) and np.array_equal(ds.test.labels, lab)
    oh = Cifar10Loader(str(tmp_path), normalize=True, one_hot=True).load_test()
    assert oh.labels.shape == (12, 10) and np.allclose(oh.labels.argmax(1), lab)
    assert oh.images.dtype == np.float32 and oh.images.max() <= 1.0


def test_gpu_augment_shapes_and_eval_normalisation():
    x = torch.full((2, 40, 40, 3), 255, dtype=torch.uint8)
    y = gpu_augment(x, 32, train=False, dtype=torch.float32)
    assert y.shape == (2, 3, 32, 32) and y.is_contiguous(memory_format=torch.channels_last)
    expect = (1 - torch.tensor([0.485, 0.456, 0.406])) / torch.tensor([0.229, 0.224, 0.225])
    assert torch.allclose(y[0, :, 5, 5], expect, atol=1e-5)
    z = gpu_augment(x, 24, train=True, dtype=torch.bfloat16, generator=torch.Generator().manual_seed(1))
    assert z.shape == (2, 3, 24, 24) and z.dtype == torch.bfloat16


def test_imagenet_shards_rank_sharding(tmp_path):
    rng = np.random.default_rng(1)
    for s in range(4):
        np.save(tmp_path / ("s%d.npy" % s), rng.integers(0, 256, (10, 20, 20, 3), dtype=np.uint8))
        np.save(tmp_path / ("s%d.labels.npy" % s), np.full(10, s))
    seen = []
    for r in range(2):
        it = ImageNetShards(str(tmp_path), batch=5, rank=r, size=2, device="cpu", out_size=16, train=False)
        labels = set()
        for xb, yb in it:
            assert xb.shape == (5, 3, 16, 16)
            labels |= set(yb.tolist())
        seen.append(labels)
    assert seen[0].isdisjoint(seen[1]) and seen[0] | seen[1] == {0, 1, 2, 3}


def test_shard_range_covers_batch():
    for n in (1, 3, 4, 7):
        parts = [shard_range(100, r, n) for r in range(n)]
        assert parts[0][0] == 0 and parts[-1][1] == 100
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
