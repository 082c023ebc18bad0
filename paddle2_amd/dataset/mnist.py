"""paddle.dataset.mnist: readers of (784 float32 image in [-1, 1], int label) (reference dataset/mnist.py)."""
import numpy as np

from . import common

__all__ = ["train", "test"]


def _reader(mode):
    def r():
        from ..vision.datasets import MNIST

        img = common._local("mnist", f"{'train' if mode == 'train' else 't10k'}-images-idx3-ubyte.gz")
        lab = common._local("mnist", f"{'train' if mode == 'train' else 't10k'}-labels-idx1-ubyte.gz")
        ds = MNIST(image_path=img, label_path=lab, mode=mode, download=False, backend="cv2")
        for i in range(len(ds)):
            x, y = ds[i]
            yield (np.asarray(x, np.float32).reshape(-1) / 255.0 * 2.0 - 1.0), int(np.asarray(y).reshape(-1)[0])

    return r


def train():
    return _reader("train")


def test():
    return _reader("test")
