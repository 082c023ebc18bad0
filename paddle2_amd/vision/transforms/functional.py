"""paddle.vision.transforms.functional (reference: python/paddle/vision/transforms/functional.py with its PIL /
cv2 / tensor backends functional_pil.py, functional_cv2.py, functional_tensor.py).

One implementation instead of three backends: every op converts its input to a float32 CHW torch tensor,
works there (interpolate / grid_sample for the geometry, closed-form blends for the colour ops) and converts
back to the input's kind — a PIL image stays a PIL image, a numpy HWC array (the cv2 backend's layout)
stays an HWC array of its dtype, a paddle Tensor stays a CHW (or ``data_format``) Tensor.  uint8 results
are rounded and clipped to [0, 255], float results are clipped to [0, 1] for the colour ops only.
"""
from __future__ import annotations

import math
import numbers

import numpy as np
import torch
import torch.nn.functional as F

from ...framework.tensor import Tensor

_INTERP = {"nearest": "nearest", "bilinear": "bilinear", "bicubic": "bicubic", "linear": "bilinear",
           "area": "area", "lanczos": "bicubic", "box": "area", "hamming": "bilinear"}


# ------------------------------------------------------------------------------------------ conversion
def _is_pil(img):
    try:
        from PIL import Image

        return isinstance(img, Image.Image)
    except ImportError:
        return False


class _Img:
    """An image as float32 CHW torch + how to give it back (kind, dtype, data_format)."""

    def __init__(self, img, data_format="CHW"):
        self.kind, self.fmt = "np", data_format
        if _is_pil(img):
            self.kind, self.mode = "pil", img.mode
            a = np.array(img)
            self.dtype = a.dtype
            self.t = torch.from_numpy(np.ascontiguousarray(a if a.ndim == 3 else a[:, :, None])).permute(2, 0, 1)
        elif isinstance(img, (Tensor, torch.Tensor)):
            self.kind = "tensor"
            t = img._t if isinstance(img, Tensor) else img
            self.dtype, self.squeeze = t.dtype, t.dim() == 2
            t = t[None] if t.dim() == 2 else t
            self.t = t.permute(2, 0, 1) if data_format == "HWC" else t
        else:
            a = np.asarray(img)
            self.dtype, self.squeeze = a.dtype, a.ndim == 2
            self.t = torch.from_numpy(np.ascontiguousarray(a if a.ndim == 3 else a[:, :, None])).permute(2, 0, 1)
        self.t = self.t.float()

    @property
    def is_int(self):
        return self.dtype in (np.uint8, torch.uint8) or (isinstance(self.dtype, np.dtype) and self.dtype.kind in "ui")

    def out(self, t):
        if self.is_int:
            t = t.round().clamp(0, 255)
        if self.kind == "tensor":
            t = t.to(self.dtype if isinstance(self.dtype, torch.dtype) else torch.float32)
            if self.fmt == "HWC":
                t = t.permute(1, 2, 0)
            if self.squeeze and t.shape[0] == 1 and self.fmt != "HWC":
                t = t[0]
            return Tensor._wrap(t.contiguous())
        a = t.permute(1, 2, 0).contiguous().numpy().astype(self.dtype)
        if self.kind == "pil":
            from PIL import Image

            return Image.fromarray(a[:, :, 0] if a.shape[2] == 1 else a, mode=self.mode if a.shape[2] in
                                   (1, 3, 4) else None)
        return a[:, :, 0] if self.squeeze and a.shape[2] == 1 else a

    def maxval(self):
        return 255.0 if self.is_int else 1.0


def _hw(img, data_format="CHW"):
    if _is_pil(img):
        return img.size[1], img.size[0]
    if isinstance(img, (Tensor, torch.Tensor)):
        s = list(img.shape)
        return (s[-2], s[-1]) if data_format == "CHW" else (s[0], s[1])
    a = np.asarray(img)
    return a.shape[0], a.shape[1]


# ------------------------------------------------------------------------------------------ basic
def to_tensor(pic, data_format="CHW"):
    """uint8 images scale to [0, 1]; layout CHW (or HWC)."""
    im = _Img(pic)
    t = im.t / 255.0 if im.is_int else im.t
    if data_format == "HWC":
        t = t.permute(1, 2, 0)
    return Tensor._wrap(t.contiguous())


def normalize(img, mean, std, data_format="CHW", to_rgb=False):
    t = img._t.float() if isinstance(img, Tensor) else torch.as_tensor(np.asarray(img, np.float32))
    chw = data_format == "CHW"
    if to_rgb:
        t = t.flip(0 if chw else -1)
    mean = torch.as_tensor(np.asarray([mean] if isinstance(mean, numbers.Number) else mean, np.float32))
    std = torch.as_tensor(np.asarray([std] if isinstance(std, numbers.Number) else std, np.float32))
    shp = (-1, 1, 1) if chw else (1, 1, -1)
    if t.dim() == 2:
        shp = (1, 1) if mean.numel() == 1 else shp
    out = (t - mean.reshape(shp)) / std.reshape(shp)
    return Tensor._wrap(out) if isinstance(img, Tensor) else out.numpy()


def resize(img, size, interpolation="bilinear"):
    """``size`` int: the shorter edge becomes ``size`` (aspect kept); (h, w): exact."""
    h, w = _hw(img)
    if isinstance(size, int):
        if h <= w:
            oh, ow = size, int(size * w / h)
        else:
            oh, ow = int(size * h / w), size
    else:
        oh, ow = int(size[0]), int(size[1])
    im = _Img(img)
    mode = _INTERP.get(interpolation, "bilinear")
    kw = {"align_corners": False} if mode in ("bilinear", "bicubic") else {}
    if mode == "bilinear" and (oh < h or ow < w):
        kw["antialias"] = True
    return im.out(F.interpolate(im.t[None], size=(oh, ow), mode=mode, **kw)[0])


def crop(img, top, left, height, width):
    im = _Img(img)
    t = im.t
    H, W = t.shape[1:]
    pt, pl = max(0, -top), max(0, -left)
    pb, pr = max(0, top + height - H), max(0, left + width - W)
    if pt or pl or pb or pr:
        t = F.pad(t, (pl, pr, pt, pb))
    return im.out(t[:, top + pt:top + pt + height, left + pl:left + pl + width])


def center_crop(img, output_size):
    th, tw = (output_size, output_size) if isinstance(output_size, int) else output_size
    h, w = _hw(img)
    return crop(img, int(round((h - th) / 2.0)), int(round((w - tw) / 2.0)), th, tw)


def hflip(img):
    im = _Img(img)
    return im.out(im.t.flip(-1))


def vflip(img):
    im = _Img(img)
    return im.out(im.t.flip(-2))


def pad(img, padding, fill=0, padding_mode="constant"):
    """padding: int | (left/right, top/bottom) | (left, top, right, bottom); modes constant / edge / reflect /
    symmetric."""
    if isinstance(padding, int):
        l = t = r = b = padding
    elif len(padding) == 2:
        l, t = padding
        r, b = padding
    else:
        l, t, r, b = padding
    im = _Img(img)
    x = im.t
    if padding_mode == "constant":
        if isinstance(fill, (list, tuple)):
            out = torch.empty(x.shape[0], x.shape[1] + t + b, x.shape[2] + l + r)
            for c in range(x.shape[0]):
                out[c] = fill[c % len(fill)]
            out[:, t:t + x.shape[1], l:l + x.shape[2]] = x
            return im.out(out)
        return im.out(F.pad(x, (l, r, t, b), value=float(fill)))
    if padding_mode == "edge":
        return im.out(F.pad(x[None], (l, r, t, b), mode="replicate")[0])
    if padding_mode == "reflect":
        return im.out(F.pad(x[None], (l, r, t, b), mode="reflect")[0])
    if padding_mode == "symmetric":
        a = np.pad(x.numpy(), ((0, 0), (t, b), (l, r)), mode="symmetric")
        return im.out(torch.from_numpy(a))
    raise ValueError(f"padding_mode must be constant / edge / reflect / symmetric, got {padding_mode!r}")


def erase(img, i, j, h, w, v, inplace=False):
    """Fill the box [i:i+h, j:j+w] with v (scalar or per-channel / per-pixel values)."""
    if isinstance(img, Tensor) and inplace:
        vv = v._t if isinstance(v, Tensor) else torch.as_tensor(v, dtype=img._t.dtype)
        img._t[..., i:i + h, j:j + w] = vv
        return img
    im = _Img(img)
    x = im.t.clone()
    vv = torch.as_tensor(np.asarray(v._t.cpu() if isinstance(v, Tensor) else v, np.float32))
    if vv.dim() == 1:
        vv = vv.reshape(-1, 1, 1)
    x[:, i:i + h, j:j + w] = vv
    return im.out(x)


# ------------------------------------------------------------------------------------------ colour
def _gray(t):
    if t.shape[0] == 1:
        return t
    return (0.299 * t[0] + 0.587 * t[1] + 0.114 * t[2])[None]


def _blend(a, b, ratio, hi):
    return (ratio * a + (1.0 - ratio) * b).clamp(0, hi)


def adjust_brightness(img, brightness_factor):
    im = _Img(img)
    return im.out(_blend(im.t, torch.zeros_like(im.t), brightness_factor, im.maxval()))


def adjust_contrast(img, contrast_factor):
    im = _Img(img)
    mean = _gray(im.t[:3] if im.t.shape[0] >= 3 else im.t).mean()
    if im.is_int:
        mean = mean.round()   # PIL computes the mean of the uint8 grayscale image
    return im.out(_blend(im.t, mean.expand_as(im.t), contrast_factor, im.maxval()))


def adjust_saturation(img, saturation_factor):
    im = _Img(img)
    return im.out(_blend(im.t, _gray(im.t).expand_as(im.t), saturation_factor, im.maxval()))


def _rgb_to_hsv(rgb):
    r, g, b = rgb
    mx, _ = rgb.max(0)
    mn, _ = rgb.min(0)
    d = mx - mn
    s = torch.where(mx > 0, d / mx.clamp_min(1e-12), torch.zeros_like(mx))
    dd = d.clamp_min(1e-12)
    h = torch.where(mx == r, ((g - b) / dd) % 6, torch.where(mx == g, (b - r) / dd + 2, (r - g) / dd + 4)) / 6.0
    h = torch.where(d > 0, h, torch.zeros_like(h))
    return torch.stack([h % 1.0, s, mx])


def _hsv_to_rgb(hsv):
    h, s, v = hsv
    i = torch.floor(h * 6.0)
    f = h * 6.0 - i
    p, q, t = v * (1 - s), v * (1 - s * f), v * (1 - s * (1 - f))
    i = i.long() % 6
    r = torch.stack([v, q, p, p, t, v])
    g = torch.stack([t, v, v, q, p, p])
    b = torch.stack([p, p, t, v, v, q])
    idx = i[None]
    return torch.stack([r.gather(0, idx)[0], g.gather(0, idx)[0], b.gather(0, idx)[0]])


def adjust_hue(img, hue_factor):
    """Shift the hue channel by hue_factor in [-0.5, 0.5] (a full turn = 1)."""
    if not -0.5 <= hue_factor <= 0.5:
        raise ValueError(f"hue_factor {hue_factor} is not in [-0.5, 0.5]")
    im = _Img(img)
    if im.t.shape[0] == 1:
        return im.out(im.t)
    hi = im.maxval()
    hsv = _rgb_to_hsv(im.t[:3] / hi)
    hsv[0] = (hsv[0] + hue_factor) % 1.0
    rgb = _hsv_to_rgb(hsv) * hi
    return im.out(torch.cat([rgb, im.t[3:]]) if im.t.shape[0] > 3 else rgb)


def to_grayscale(img, num_output_channels=1):
    im = _Img(img)
    g = _gray(im.t)
    if num_output_channels == 3:
        g = g.expand(3, -1, -1)
    out = im.out(g.contiguous())
    if im.kind == "pil":
        from PIL import Image

        return Image.fromarray(np.asarray(out)) if num_output_channels == 1 else out
    return out


# ------------------------------------------------------------------------------------------ geometry
def _inverse_affine(center, angle, translate, scale, shear):
    """Output pixel -> input pixel matrix of the affine map rotate(angle, clockwise) * scale * shear about
    ``center`` followed by ``translate``."""
    cx, cy = center
    tx, ty = translate
    rot = math.radians(angle)
    sx, sy = (math.radians(s) for s in shear)
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [d / scale, -b / scale, 0.0, -c / scale, a / scale, 0.0]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty)
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty)
    m[2] += cx
    m[5] += cy
    return m


def _warp(im, coords_fn, out_hw, interpolation, fill):
    """Sample im.t at input pixel coordinates coords_fn(x_out, y_out) (pixel centres at integer + 0.5 not used:
    pixel (0, 0) is at coordinate 0); outside pixels take ``fill``."""
    H, W = im.t.shape[1:]
    oh, ow = out_hw
    ys, xs = torch.meshgrid(torch.arange(oh, dtype=torch.float64), torch.arange(ow, dtype=torch.float64),
                            indexing="ij")
    sx, sy = coords_fn(xs, ys)
    gx = (2 * sx + 1) / W - 1
    gy = (2 * sy + 1) / H - 1
    grid = torch.stack([gx, gy], -1).float()[None]
    mode = "nearest" if interpolation == "nearest" else "bilinear"
    ones = torch.ones(1, 1, H, W)
    src = torch.cat([im.t[None], ones], 1)
    out = F.grid_sample(src, grid, mode=mode, padding_mode="zeros", align_corners=False)[0]
    val, mask = out[:-1], out[-1:]
    fv = torch.as_tensor(np.asarray(fill if isinstance(fill, (list, tuple)) else [fill] * val.shape[0],
                                    np.float32)).reshape(-1, 1, 1)
    return val + fv[:val.shape[0]] * (1 - mask)   # outside samples are 0 in val and weigh in through the mask


def affine(img, angle, translate, scale, shear, interpolation="nearest", fill=0, center=None):
    """Rotate by ``angle`` degrees clockwise about ``center`` (default: the image centre), scale, shear
    (x, y degrees) and translate (dx, dy pixels); the output keeps the input size."""
    if isinstance(shear, numbers.Number):
        shear = (shear, 0.0)
    h, w = _hw(img)
    c = ((w - 1) * 0.5, (h - 1) * 0.5) if center is None else center
    m = _inverse_affine(c, angle, translate, scale, shear)
    im = _Img(img)

    def coords(x, y):
        return m[0] * x + m[1] * y + m[2], m[3] * x + m[4] * y + m[5]

    return im.out(_warp(im, coords, (h, w), interpolation, fill))


def rotate(img, angle, interpolation="nearest", expand=False, center=None, fill=0):
    """Rotate counter-clockwise by ``angle`` degrees; ``expand`` grows the canvas to hold the whole image."""
    h, w = _hw(img)
    c = ((w - 1) * 0.5, (h - 1) * 0.5) if center is None else center
    m = _inverse_affine(c, -angle, (0.0, 0.0), 1.0, (0.0, 0.0))
    oh, ow = h, w
    if expand:
        corners = np.array([[0, 0], [w - 1, 0], [w - 1, h - 1], [0, h - 1]], np.float64)
        # forward map = inverse of m (2x2 part), about the same centre
        A = np.array([[m[0], m[1]], [m[3], m[4]]])
        Ai = np.linalg.inv(A)
        pts = (corners - np.array(c)) @ Ai.T + np.array(c)
        ow = int(math.ceil(pts[:, 0].max() - pts[:, 0].min() + 1 - 1e-6))
        oh = int(math.ceil(pts[:, 1].max() - pts[:, 1].min() + 1 - 1e-6))
        shift_x, shift_y = pts[:, 0].min(), pts[:, 1].min()
    else:
        shift_x = shift_y = 0.0
    im = _Img(img)

    def coords(x, y):
        x, y = x + shift_x, y + shift_y
        return m[0] * x + m[1] * y + m[2], m[3] * x + m[4] * y + m[5]

    return im.out(_warp(im, coords, (oh, ow), interpolation, fill))


def _perspective_coeffs(startpoints, endpoints):
    """(a..h) of the map output (endpoints) -> input (startpoints): x_in = (a x + b y + c) / (g x + h y + 1)."""
    A = np.zeros((8, 8))
    for i, ((xo, yo), (xi, yi)) in enumerate(zip(endpoints, startpoints)):
        A[2 * i] = [xo, yo, 1, 0, 0, 0, -xi * xo, -xi * yo]
        A[2 * i + 1] = [0, 0, 0, xo, yo, 1, -yi * xo, -yi * yo]
    rhs = np.asarray(startpoints, np.float64).reshape(8)
    return np.linalg.lstsq(A, rhs, rcond=None)[0]


def perspective(img, startpoints, endpoints, interpolation="nearest", fill=0):
    """Warp so the quadrilateral ``startpoints`` (tl, tr, br, bl) lands on ``endpoints``."""
    a, b, c, d, e, f, g, h_ = _perspective_coeffs(startpoints, endpoints)
    H, W = _hw(img)
    im = _Img(img)

    def coords(x, y):
        den = g * x + h_ * y + 1.0
        return (a * x + b * y + c) / den, (d * x + e * y + f) / den

    return im.out(_warp(im, coords, (H, W), interpolation, fill))


__all__ = ["to_tensor", "normalize", "resize", "crop", "center_crop", "hflip", "vflip", "pad", "erase",
           "adjust_brightness", "adjust_contrast", "adjust_saturation", "adjust_hue", "to_grayscale", "affine",
           "rotate", "perspective"]
