"""Vision datasets (reference: python/paddle/vision/datasets/).

There is no network access here, so ``MNIST``/``Cifar10``/``FashionMNIST`` read local files when
``image_path``/``data_file`` are given and otherwise fall back to a deterministic synthetic
dataset of the same shapes/dtypes (labels correlated with image content, so models can learn).
"""
from __future__ import annotations

import gzip
import os

import numpy as np

from ...io import Dataset


def _read_idx(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    nd = magic & 0xFF
    dims = [int.from_bytes(data[4 + 4 * i: 8 + 4 * i], "big") for i in range(nd)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd).reshape(dims)


class _Synthetic(Dataset):
    def __init__(self, n, shape, num_classes, seed, transform=None, backend="cv2", dtype=np.uint8):
        rs = np.random.RandomState(seed)
        self.labels = rs.randint(0, num_classes, size=(n,)).astype(np.int64)
        protos = rs.randint(0, 255, size=(num_classes,) + shape).astype(np.float32)
        noise = rs.randint(0, 64, size=(n,) + shape).astype(np.float32)
        self.images = np.clip(protos[self.labels] * 0.75 + noise, 0, 255).astype(dtype)
        self.transform = transform
        self.backend = backend

    def __getitem__(self, idx):
        img, lab = self.images[idx], self.labels[idx]
        if self.transform is not None:
            img = self.transform(img)
        else:
            img = img.astype(np.float32)
        return img, np.array([lab], dtype=np.int64)

    def __len__(self):
        return len(self.labels)


class MNIST(Dataset):
    NAME = "mnist"

    def __init__(self, image_path=None, label_path=None, mode="train", transform=None, download=True, backend=None,
                 num_samples=None):
        self.mode, self.transform, self.backend = mode, transform, backend or "cv2"
        if image_path and label_path and os.path.exists(image_path):
            self.images = _read_idx(image_path)
            self.labels = _read_idx(label_path).astype(np.int64)
            self._syn = None
        else:
            n = num_samples or (60000 if mode == "train" else 10000)
            self._syn = _Synthetic(n, (28, 28), 10, 0 if mode == "train" else 1, transform)
            self.images, self.labels = self._syn.images, self._syn.labels

    def __getitem__(self, idx):
        img = self.images[idx]
        lab = np.array([self.labels[idx]], dtype=np.int64)
        if self.transform is not None:
            img = self.transform(img)
        else:
            img = img.astype(np.float32)
        return img, lab

    def __len__(self):
        return len(self.labels)


class FashionMNIST(MNIST):
    NAME = "fashion-mnist"


class Cifar10(Dataset):
    def __init__(self, data_file=None, mode="train", transform=None, download=True, backend=None, num_samples=None):
        n = num_samples or (50000 if mode == "train" else 10000)
        self._syn = _Synthetic(n, (32, 32, 3), 10, 2 if mode == "train" else 3, transform)
        self.transform = transform

    def __getitem__(self, idx):
        return self._syn[idx]

    def __len__(self):
        return len(self._syn)


class Cifar100(Cifar10):
    def __init__(self, data_file=None, mode="train", transform=None, download=True, backend=None, num_samples=None):
        n = num_samples or (50000 if mode == "train" else 10000)
        self._syn = _Synthetic(n, (32, 32, 3), 100, 4 if mode == "train" else 5, transform)


class FakeData(Dataset):
    def __init__(self, num_samples=1000, image_shape=(3, 224, 224), num_classes=1000, transform=None):
        self.n, self.shape, self.nc, self.transform = num_samples, tuple(image_shape), num_classes, transform

    def __getitem__(self, idx):
        rs = np.random.RandomState(idx)
        img = rs.rand(*self.shape).astype(np.float32)
        if self.transform is not None:
            img = self.transform(img)
        return img, np.array([rs.randint(0, self.nc)], dtype=np.int64)

    def __len__(self):
        return self.n


class DatasetFolder(Dataset):
    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.root = root
        classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
        self.classes = classes
        self.class_to_idx = {c: i for i, c in enumerate(classes)}
        self.samples = []
        for c in classes:
            for fn in sorted(os.listdir(os.path.join(root, c))):
                p = os.path.join(root, c, fn)
                if extensions is None or fn.lower().endswith(tuple(extensions)):
                    self.samples.append((p, self.class_to_idx[c]))
        self.loader = loader or (lambda p: np.load(p) if p.endswith(".npy") else open(p, "rb").read())
        self.transform = transform

    def __getitem__(self, idx):
        p, t = self.samples[idx]
        s = self.loader(p)
        if self.transform is not None:
            s = self.transform(s)
        return s, t

    def __len__(self):
        return len(self.samples)


ImageFolder = DatasetFolder
