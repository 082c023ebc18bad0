"""paddle.vision.transforms (numpy/HWC based subset; reference: python/paddle/vision/transforms/)."""
from __future__ import annotations

import numbers

import numpy as np

from ..framework.tensor import Tensor


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


class BaseTransform:
    def __init__(self, keys=None):
        self.keys = keys

    def __call__(self, x):
        return self._apply_image(x)


class ToTensor(BaseTransform):
    def __init__(self, data_format="CHW", keys=None):
        self.fmt = data_format

    def _apply_image(self, img):
        a = np.asarray(img)
        if a.ndim == 2:
            a = a[:, :, None]
        a = a.astype(np.float32)
        if a.max() > 1.0:
            a = a / 255.0
        if self.fmt == "CHW":
            a = a.transpose(2, 0, 1)
        return a


class Normalize(BaseTransform):
    def __init__(self, mean=0.0, std=1.0, data_format="CHW", to_rgb=False, keys=None):
        self.mean = np.asarray([mean] if isinstance(mean, numbers.Number) else mean, dtype=np.float32)
        self.std = np.asarray([std] if isinstance(std, numbers.Number) else std, dtype=np.float32)
        self.fmt = data_format

    def _apply_image(self, img):
        a = np.asarray(img, dtype=np.float32)
        if a.ndim == 2:
            return (a - self.mean[0]) / self.std[0]
        if self.fmt == "CHW":
            return (a - self.mean[:, None, None]) / self.std[:, None, None]
        return (a - self.mean) / self.std


class Transpose(BaseTransform):
    def __init__(self, order=(2, 0, 1), keys=None):
        self.order = order

    def _apply_image(self, img):
        a = np.asarray(img)
        if a.ndim == 2:
            a = a[:, :, None]
        return a.transpose(self.order)


class Resize(BaseTransform):
    def __init__(self, size, interpolation="bilinear", keys=None):
        self.size = (size, size) if isinstance(size, int) else tuple(size)

    def _apply_image(self, img):
        import torch

        a = np.asarray(img, dtype=np.float32)
        chw = a.ndim == 3 and a.shape[0] in (1, 3) and a.shape[-1] not in (1, 3)
        t = torch.from_numpy(a if chw else (a[None] if a.ndim == 2 else a.transpose(2, 0, 1)))
        r = torch.nn.functional.interpolate(t[None], size=self.size, mode="bilinear", align_corners=False)[0].numpy()
        if chw:
            return r
        return r[0] if a.ndim == 2 else r.transpose(1, 2, 0)


class CenterCrop(BaseTransform):
    def __init__(self, size, keys=None):
        self.size = (size, size) if isinstance(size, int) else tuple(size)

    def _apply_image(self, img):
        a = np.asarray(img)
        h, w = a.shape[:2]
        th, tw = self.size
        i, j = (h - th) // 2, (w - tw) // 2
        return a[i:i + th, j:j + tw]


class RandomCrop(BaseTransform):
    def __init__(self, size, padding=None, pad_if_needed=False, fill=0, padding_mode="constant", keys=None):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.padding = padding

    def _apply_image(self, img):
        a = np.asarray(img)
        if self.padding:
            p = self.padding
            a = np.pad(a, ((p, p), (p, p)) + ((0, 0),) * (a.ndim - 2))
        h, w = a.shape[:2]
        th, tw = self.size
        i = np.random.randint(0, h - th + 1)
        j = np.random.randint(0, w - tw + 1)
        return a[i:i + th, j:j + tw]


class RandomHorizontalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        self.prob = prob

    def _apply_image(self, img):
        a = np.asarray(img)
        return a[:, ::-1].copy() if np.random.rand() < self.prob else a


class RandomVerticalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        self.prob = prob

    def _apply_image(self, img):
        a = np.asarray(img)
        return a[::-1].copy() if np.random.rand() < self.prob else a


RandomResizedCrop = RandomCrop


def to_tensor(pic, data_format="CHW"):
    return Tensor(ToTensor(data_format)(pic))


def normalize(img, mean, std, data_format="CHW", to_rgb=False):
    return Normalize(mean, std, data_format)(img)
