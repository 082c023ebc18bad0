"""paddle.vision.transforms classes (reference: python/paddle/vision/transforms/transforms.py — BaseTransform
:179 with ``keys`` dispatch, Resize :418, RandomResizedCrop :489, CenterCrop :715, flips :760 / :823, Normalize
:886, Transpose :960, colour transforms :1016-1211, RandomCrop :1309, Pad :1443, RandomAffine :1555,
RandomRotation :1738, RandomPerspective :1846, Grayscale :1989, RandomErasing :2041).

Images are PIL images, numpy HWC arrays or paddle CHW Tensors; every transform returns the input's kind
(functional.py).  ``keys`` names what each element of a tuple input is ("image", "coords", "boxes", "mask");
only "image" / "mask" elements are transformed geometrically and only images photometrically.
"""
from __future__ import annotations

import math
import numbers
import random

import numpy as np

from ...framework.tensor import Tensor
from . import functional as F


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data

    def __repr__(self):
        return "Compose(" + ", ".join(type(t).__name__ for t in self.transforms) + ")"


class BaseTransform:
    """Subclasses implement ``_apply_image`` (and optionally ``_apply_mask`` / ``_apply_coords`` /
    ``_apply_boxes``); ``_get_params`` draws the random parameters once per call, shared by every key."""

    def __init__(self, keys=None):
        if keys is None:
            keys = ("image",)
        elif not isinstance(keys, (list, tuple)):
            raise ValueError(f"keys should be a sequence, got {keys!r}")
        self.keys = tuple(keys)
        self.params = None

    def _get_params(self, inputs):
        return None

    def __call__(self, inputs):
        single = not isinstance(inputs, tuple)
        items = (inputs,) if single else inputs
        self.params = self._get_params(items)
        out = []
        for key, item in zip(self.keys, items):
            fn = getattr(self, f"_apply_{key}", None)
            out.append(fn(item) if fn is not None else item)
        out.extend(items[len(self.keys):])
        return out[0] if single else tuple(out)

    def _apply_image(self, img):
        raise NotImplementedError

    def _apply_mask(self, mask):
        return mask


class ToTensor(BaseTransform):
    def __init__(self, data_format="CHW", keys=None):
        super().__init__(keys)
        self.data_format = data_format

    def _apply_image(self, img):
        return F.to_tensor(img, self.data_format)


class Normalize(BaseTransform):
    def __init__(self, mean=0.0, std=1.0, data_format="CHW", to_rgb=False, keys=None):
        super().__init__(keys)
        self.mean = [mean] * 3 if isinstance(mean, numbers.Number) else list(mean)
        self.std = [std] * 3 if isinstance(std, numbers.Number) else list(std)
        self.data_format, self.to_rgb = data_format, to_rgb

    def _apply_image(self, img):
        a = img if isinstance(img, Tensor) else np.asarray(img, np.float32)
        ch = (a.shape[0] if self.data_format == "CHW" else a.shape[-1]) if len(a.shape) == 3 else 1
        return F.normalize(a, self.mean[:ch], self.std[:ch], self.data_format, self.to_rgb)


class Transpose(BaseTransform):
    def __init__(self, order=(2, 0, 1), keys=None):
        super().__init__(keys)
        self.order = order

    def _apply_image(self, img):
        if isinstance(img, Tensor):
            return Tensor._wrap(img._t.permute(*self.order))
        a = np.asarray(img)
        if a.ndim == 2:
            a = a[:, :, None]
        return a.transpose(self.order)


class Resize(BaseTransform):
    def __init__(self, size, interpolation="bilinear", keys=None):
        super().__init__(keys)
        self.size, self.interpolation = size, interpolation

    def _apply_image(self, img):
        return F.resize(img, self.size, self.interpolation)

    def _apply_mask(self, mask):
        return F.resize(mask, self.size, "nearest")


class RandomResizedCrop(BaseTransform):
    """Crop a random area (``scale`` of the image) with a random aspect ratio, then resize to ``size``."""

    def __init__(self, size, scale=(0.08, 1.0), ratio=(3.0 / 4, 4.0 / 3), interpolation="bilinear", keys=None):
        super().__init__(keys)
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.scale, self.ratio, self.interpolation = scale, ratio, interpolation

    def _get_params(self, inputs):
        h, w = F._hw(inputs[0])
        area = h * w
        log_r = (math.log(self.ratio[0]), math.log(self.ratio[1]))
        for _ in range(10):
            target = area * random.uniform(*self.scale)
            ar = math.exp(random.uniform(*log_r))
            cw, ch = int(round(math.sqrt(target * ar))), int(round(math.sqrt(target / ar)))
            if 0 < cw <= w and 0 < ch <= h:
                return random.randint(0, h - ch), random.randint(0, w - cw), ch, cw
        in_ratio = w / h
        if in_ratio < min(self.ratio):
            cw, ch = w, int(round(w / min(self.ratio)))
        elif in_ratio > max(self.ratio):
            ch, cw = h, int(round(h * max(self.ratio)))
        else:
            cw, ch = w, h
        return (h - ch) // 2, (w - cw) // 2, ch, cw

    def _apply_image(self, img):
        i, j, h, w = self.params
        return F.resize(F.crop(img, i, j, h, w), self.size, self.interpolation)

    def _apply_mask(self, mask):
        i, j, h, w = self.params
        return F.resize(F.crop(mask, i, j, h, w), self.size, "nearest")


class CenterCrop(BaseTransform):
    def __init__(self, size, keys=None):
        super().__init__(keys)
        self.size = size

    def _apply_image(self, img):
        return F.center_crop(img, self.size)

    _apply_mask = _apply_image


class RandomCrop(BaseTransform):
    def __init__(self, size, padding=None, pad_if_needed=False, fill=0, padding_mode="constant", keys=None):
        super().__init__(keys)
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.padding, self.pad_if_needed, self.fill, self.padding_mode = padding, pad_if_needed, fill, padding_mode

    def _prep(self, img):
        if self.padding is not None:
            img = F.pad(img, self.padding, self.fill, self.padding_mode)
        h, w = F._hw(img)
        th, tw = self.size
        if self.pad_if_needed and w < tw:
            img = F.pad(img, (tw - w, 0), self.fill, self.padding_mode)
        if self.pad_if_needed and h < th:
            img = F.pad(img, (0, th - h), self.fill, self.padding_mode)
        return img

    def _get_params(self, inputs):
        h, w = F._hw(self._prep(inputs[0]))
        th, tw = self.size
        if h < th or w < tw:
            raise ValueError(f"crop size {self.size} is larger than the (padded) image {(h, w)}")
        return random.randint(0, h - th), random.randint(0, w - tw)

    def _apply_image(self, img):
        i, j = self.params
        return F.crop(self._prep(img), i, j, *self.size)

    _apply_mask = _apply_image


class RandomHorizontalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _get_params(self, inputs):
        return random.random() < self.prob

    def _apply_image(self, img):
        return F.hflip(img) if self.params else img

    _apply_mask = _apply_image


class RandomVerticalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _get_params(self, inputs):
        return random.random() < self.prob

    def _apply_image(self, img):
        return F.vflip(img) if self.params else img

    _apply_mask = _apply_image


def _factor_range(value, name, center=1.0, bound=(0, float("inf"))):
    if isinstance(value, numbers.Number):
        if value < 0:
            raise ValueError(f"{name} must be non-negative")
        value = (center - value, center + value)
    lo, hi = max(bound[0], value[0]), min(bound[1], value[1])
    return None if lo == hi == center else (lo, hi)


class BrightnessTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = _factor_range(value, "brightness")

    def _apply_image(self, img):
        return img if self.value is None else F.adjust_brightness(img, random.uniform(*self.value))


class ContrastTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = _factor_range(value, "contrast")

    def _apply_image(self, img):
        return img if self.value is None else F.adjust_contrast(img, random.uniform(*self.value))


class SaturationTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = _factor_range(value, "saturation")

    def _apply_image(self, img):
        return img if self.value is None else F.adjust_saturation(img, random.uniform(*self.value))


class HueTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = _factor_range(value, "hue", center=0.0, bound=(-0.5, 0.5))

    def _apply_image(self, img):
        return img if self.value is None else F.adjust_hue(img, random.uniform(*self.value))


class ColorJitter(BaseTransform):
    """Brightness, contrast, saturation and hue jitter applied in a random order."""

    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0, keys=None):
        super().__init__(keys)
        self.brightness, self.contrast, self.saturation, self.hue = brightness, contrast, saturation, hue

    def _apply_image(self, img):
        ts = [BrightnessTransform(self.brightness), ContrastTransform(self.contrast),
              SaturationTransform(self.saturation), HueTransform(self.hue)]
        random.shuffle(ts)
        for t in ts:
            img = t._apply_image(img)
        return img


class Pad(BaseTransform):
    def __init__(self, padding, fill=0, padding_mode="constant", keys=None):
        super().__init__(keys)
        if padding_mode not in ("constant", "edge", "reflect", "symmetric"):
            raise ValueError("padding_mode should be constant, edge, reflect or symmetric")
        self.padding, self.fill, self.padding_mode = padding, fill, padding_mode

    def _apply_image(self, img):
        return F.pad(img, self.padding, self.fill, self.padding_mode)

    _apply_mask = _apply_image


def _angle_range(x, name):
    if isinstance(x, numbers.Number):
        if x < 0:
            raise ValueError(f"{name}: a single number must be non-negative")
        return (-float(x), float(x))
    if len(x) != 2:
        raise ValueError(f"{name} should be a number or a sequence of two numbers")
    return (float(x[0]), float(x[1]))


class RandomAffine(BaseTransform):
    def __init__(self, degrees, translate=None, scale=None, shear=None, interpolation="nearest", fill=0,
                 center=None, keys=None):
        super().__init__(keys)
        self.degrees = _angle_range(degrees, "degrees")
        if translate is not None and not all(0.0 <= t <= 1.0 for t in translate):
            raise ValueError("translate values should be between 0 and 1")
        if scale is not None and not all(s > 0 for s in scale):
            raise ValueError("scale values should be positive")
        self.translate, self.scale = translate, scale
        if shear is not None:
            shear = _angle_range(shear, "shear") if isinstance(shear, numbers.Number) or len(shear) == 2 \
                else tuple(float(s) for s in shear)
        self.shear, self.interpolation, self.fill, self.center = shear, interpolation, fill, center

    def _get_params(self, inputs):
        h, w = F._hw(inputs[0])
        angle = random.uniform(*self.degrees)
        if self.translate is not None:
            mx, my = self.translate[0] * w, self.translate[1] * h
            tr = (int(round(random.uniform(-mx, mx))), int(round(random.uniform(-my, my))))
        else:
            tr = (0, 0)
        sc = random.uniform(*self.scale) if self.scale is not None else 1.0
        sh = (0.0, 0.0)
        if self.shear is not None:
            sh = (random.uniform(self.shear[0], self.shear[1]),
                  random.uniform(self.shear[2], self.shear[3]) if len(self.shear) == 4 else 0.0)
        return angle, tr, sc, sh

    def _apply_image(self, img):
        a, tr, sc, sh = self.params
        return F.affine(img, a, tr, sc, sh, self.interpolation, self.fill, self.center)

    def _apply_mask(self, mask):
        a, tr, sc, sh = self.params
        return F.affine(mask, a, tr, sc, sh, "nearest", 0, self.center)


class RandomRotation(BaseTransform):
    def __init__(self, degrees, interpolation="nearest", expand=False, center=None, fill=0, keys=None):
        super().__init__(keys)
        self.degrees = _angle_range(degrees, "degrees")
        self.interpolation, self.expand, self.center, self.fill = interpolation, expand, center, fill

    def _get_params(self, inputs):
        return random.uniform(*self.degrees)

    def _apply_image(self, img):
        return F.rotate(img, self.params, self.interpolation, self.expand, self.center, self.fill)

    def _apply_mask(self, mask):
        return F.rotate(mask, self.params, "nearest", self.expand, self.center, 0)


class RandomPerspective(BaseTransform):
    def __init__(self, prob=0.5, distortion_scale=0.5, interpolation="nearest", fill=0, keys=None):
        super().__init__(keys)
        if not 0 <= distortion_scale <= 1:
            raise ValueError("distortion_scale must be in [0, 1]")
        self.prob, self.distortion_scale, self.interpolation, self.fill = prob, distortion_scale, interpolation, fill

    def _get_params(self, inputs):
        if random.random() >= self.prob:
            return None
        h, w = F._hw(inputs[0])
        dw, dh = int(self.distortion_scale * w / 2), int(self.distortion_scale * h / 2)
        tl = [random.randint(0, dw), random.randint(0, dh)]
        tr = [w - 1 - random.randint(0, dw), random.randint(0, dh)]
        br = [w - 1 - random.randint(0, dw), h - 1 - random.randint(0, dh)]
        bl = [random.randint(0, dw), h - 1 - random.randint(0, dh)]
        start = [[0, 0], [w - 1, 0], [w - 1, h - 1], [0, h - 1]]
        return start, [tl, tr, br, bl]

    def _apply_image(self, img):
        if self.params is None:
            return img
        return F.perspective(img, self.params[0], self.params[1], self.interpolation, self.fill)


class Grayscale(BaseTransform):
    def __init__(self, num_output_channels=1, keys=None):
        super().__init__(keys)
        self.num_output_channels = num_output_channels

    def _apply_image(self, img):
        return F.to_grayscale(img, self.num_output_channels)


class RandomErasing(BaseTransform):
    """Erase a random box of ``scale`` of the area and ``ratio`` aspect with ``value`` (a number, a per-channel
    sequence, or "random" for normal noise)."""

    def __init__(self, prob=0.5, scale=(0.02, 0.33), ratio=(0.3, 3.3), value=0, inplace=False, keys=None):
        super().__init__(keys)
        if not (0 <= prob <= 1 and scale[0] <= scale[1] and ratio[0] <= ratio[1]):
            raise ValueError("invalid RandomErasing arguments")
        self.prob, self.scale, self.ratio, self.value, self.inplace = prob, scale, ratio, value, inplace

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        h, w = F._hw(img)
        ch = 1 if len(img.shape if hasattr(img, "shape") else np.asarray(img).shape) == 2 else (
            img.shape[0] if isinstance(img, Tensor) else np.asarray(img).shape[-1])
        log_r = (math.log(self.ratio[0]), math.log(self.ratio[1]))
        for _ in range(10):
            area = h * w * random.uniform(*self.scale)
            ar = math.exp(random.uniform(*log_r))
            eh, ew = int(round(math.sqrt(area * ar))), int(round(math.sqrt(area / ar)))
            if eh < h and ew < w:
                i, j = random.randint(0, h - eh), random.randint(0, w - ew)
                if isinstance(self.value, str) and self.value == "random":
                    v = np.random.normal(size=(ch, eh, ew)).astype(np.float32)
                elif isinstance(self.value, numbers.Number):
                    v = [float(self.value)] * ch
                else:
                    v = list(self.value)
                return F.erase(img, i, j, eh, ew, v, self.inplace)
        return img
