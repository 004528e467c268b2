"""CIFAR-10 / CIFAR-100 loaders (binary distribution, no pickle).

Parity: ``srcs/python/kungfu/tensorflow/v1/helpers/cifar.py`` (Cifar10Loader /
Cifar100Loader: NHWC uint8 images, optional [0,1] normalisation and one-hot
labels).  The reference reads the *python* (pickled) batches; this reads the
equivalent *binary* batches (``cifar-10-batches-bin/data_batch_{1..5}.bin``,
``test_batch.bin``: records of 1 label byte + 3072 CHW image bytes;
``cifar-100-binary/{train,test}.bin``: coarse + fine label bytes), which need
no unpickling.  Results are numpy arrays, images NHWC.
"""
from __future__ import annotations

import os
from collections import namedtuple
from typing import Optional

import numpy as np

DataSet = namedtuple("DataSet", "images labels")
DataSets = namedtuple("DataSets", "train test")
_default_dir = os.path.join(os.path.expanduser("~"), "var/data/cifar")


def _onehot(k: int, a: np.ndarray) -> np.ndarray:
    out = np.zeros((a.shape[0], k), np.float32)
    out[np.arange(a.shape[0]), a] = 1
    return out


def _read_records(path: str, label_bytes: int, label_index: int):
    rec = label_bytes + 3072
    raw = np.fromfile(path, dtype=np.uint8)
    if raw.size % rec:
        raise ValueError("%s: size %d is not a multiple of %d" % (path, raw.size, rec))
    raw = raw.reshape(-1, rec)
    labels = raw[:, label_index].astype(np.int64)
    images = raw[:, label_bytes:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    return np.ascontiguousarray(images), labels


class _Loader:
    classes = 10
    label_bytes = 1
    label_index = 0

    def __init__(self, data_dir: str = _default_dir, normalize: bool = False, one_hot: bool = False):
        self.data_dir, self.normalize, self.one_hot = data_dir, normalize, one_hot

    def _finish(self, images, labels) -> DataSet:
        if self.normalize:
            images = (images / 255.0).astype(np.float32)
        if self.one_hot:
            labels = _onehot(self.classes, labels)
        return DataSet(images, labels)

    def _load(self, files) -> DataSet:
        parts = [_read_records(os.path.join(self.data_dir, f), self.label_bytes, self.label_index) for f in files]
        return self._finish(np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))

    def load_datasets(self) -> DataSets:
        return DataSets(self.load_train(), self.load_test())


class Cifar10Loader(_Loader):
    def load_train(self) -> DataSet:
        return self._load(["cifar-10-batches-bin/data_batch_%d.bin" % i for i in range(1, 6)])

    def load_test(self) -> DataSet:
        return self._load(["cifar-10-batches-bin/test_batch.bin"])


class Cifar100Loader(_Loader):
    classes = 100
    label_bytes = 2
    label_index = 1  # fine label

    def load_train(self) -> DataSet:
        return self._load(["cifar-100-binary/train.bin"])

    def load_test(self) -> DataSet:
        return self._load(["cifar-100-binary/test.bin"])


def write_cifar10_binary(path: str, images: np.ndarray, labels: np.ndarray) -> None:
    """Writes NHWC uint8 images + labels in the CIFAR-10 binary record format (tests, tools)."""
    recs = np.concatenate([labels.astype(np.uint8)[:, None],
                           images.transpose(0, 3, 1, 2).reshape(images.shape[0], -1).astype(np.uint8)], axis=1)
    recs.tofile(path)
