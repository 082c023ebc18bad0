"""paddle.dataset.cifar: readers of (3072 float32 image in [0, 1], int label) (reference dataset/cifar.py)."""
import numpy as np

from . import common

__all__ = ["train10", "test10", "train100", "test100"]


def _reader(cls_name, fname, mode):
    def r():
        from ..vision import datasets as V

        ds = getattr(V, cls_name)(data_file=common._local("cifar", fname), mode=mode, download=False, backend="cv2")
        for i in range(len(ds)):
            x, y = ds[i]
            yield np.asarray(x, np.float32).transpose(2, 0, 1).reshape(-1) / 255.0, int(np.asarray(y).reshape(-1)[0])

    return r


def train10(cycle=False):
    return _reader("Cifar10", "cifar-10-python.tar.gz", "train")


def test10(cycle=False):
    return _reader("Cifar10", "cifar-10-python.tar.gz", "test")


def train100():
    return _reader("Cifar100", "cifar-100-python.tar.gz", "train")


def test100():
    return _reader("Cifar100", "cifar-100-python.tar.gz", "test")
