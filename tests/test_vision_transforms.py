"""paddle.vision.transforms: functional ops on numpy HWC / PIL / Tensor CHW inputs vs numpy oracles, and the
random transform classes (reference tests: test/legacy_test/test_transforms.py, test_transforms_static.py)."""
import numpy as np
import pytest
from PIL import Image

import paddle2_amd as paddle
from paddle2_amd.vision import transforms as T
from paddle2_amd.vision.transforms import functional as F


def _img(h=6, w=8, c=3, seed=0):
    return np.random.RandomState(seed).randint(0, 256, (h, w, c)).astype(np.uint8)


def test_types_roundtrip_and_resize():
    a = _img(6, 8)
    r = F.resize(a, 3)                       # shorter edge -> 3, aspect kept
    assert isinstance(r, np.ndarray) and r.shape == (3, 4, 3) and r.dtype == np.uint8
    p = F.resize(Image.fromarray(a), (4, 5))
    assert isinstance(p, Image.Image) and p.size == (5, 4)
    t = F.resize(paddle.to_tensor(a.transpose(2, 0, 1).astype("float32")), (12, 16))
    assert list(t.shape) == [3, 12, 16]
    assert np.array_equal(F.resize(a, (6, 8), "nearest"), a)


def test_flips_crop_pad():
    a = _img()
    assert np.array_equal(F.hflip(a), a[:, ::-1]) and np.array_equal(F.vflip(a), a[::-1])
    assert np.array_equal(F.crop(a, 1, 2, 3, 4), a[1:4, 2:6])
    assert np.array_equal(F.center_crop(a, 4), a[1:5, 2:6])
    for mode, npm in [("constant", "constant"), ("edge", "edge"), ("reflect", "reflect"), ("symmetric", "symmetric")]:
        ref = np.pad(a, ((2, 1), (3, 4), (0, 0)), mode=npm)
        assert np.array_equal(F.pad(a, (3, 2, 4, 1), padding_mode=mode), ref), mode
    e = F.erase(a, 1, 1, 2, 2, [0, 0, 0])
    assert (e[1:3, 1:3] == 0).all() and np.array_equal(e[0], a[0])


def test_geometry():
    a = _img(7, 7)
    assert np.array_equal(F.rotate(a, 90), np.rot90(a))                 # counter-clockwise
    assert np.array_equal(F.rotate(a, 0), a)
    sh = F.affine(a, 0, (2, 1), 1.0, 0.0)
    ref = np.zeros_like(a)
    ref[1:, 2:] = a[:-1, :-2]
    assert np.array_equal(sh, ref)
    assert np.array_equal(F.affine(a, -90, (0, 0), 1.0, 0.0), np.rot90(a))   # affine angle is clockwise
    pts = [[0, 0], [6, 0], [6, 6], [0, 6]]
    assert np.array_equal(F.perspective(a, pts, pts), a)
    big = F.rotate(_img(4, 8), 90, expand=True)
    assert big.shape[:2] == (8, 4)


def test_colour_ops():
    a = _img().astype(np.float32) / 255.0
    np.testing.assert_allclose(F.adjust_brightness(a, 1.0), a, atol=1e-6)
    np.testing.assert_allclose(F.adjust_brightness(a, 0.5), a * 0.5, atol=1e-6)
    np.testing.assert_allclose(F.adjust_contrast(a, 1.0), a, atol=1e-6)
    gray = F.to_grayscale(a, 3)
    np.testing.assert_allclose(F.adjust_saturation(a, 0.0), gray, atol=1e-6)
    assert np.allclose(gray[..., 0], gray[..., 1])
    np.testing.assert_allclose(F.adjust_hue(a, 0.0), a, atol=1e-5)
    back = F.adjust_hue(F.adjust_hue(a, 0.3), -0.3)
    np.testing.assert_allclose(back, a, atol=1e-4)
    red = np.zeros((1, 1, 3), np.float32)
    red[..., 0] = 1.0
    np.testing.assert_allclose(F.adjust_hue(red, 1 / 3)[0, 0], [0, 1, 0], atol=1e-5)   # red -> green
    with pytest.raises(ValueError):
        F.adjust_hue(a, 0.7)


def test_tensor_input_and_to_tensor_normalize():
    a = _img()
    t = F.to_tensor(a)
    assert list(t.shape) == [3, 6, 8] and float(t.numpy().max()) <= 1.0
    np.testing.assert_allclose(F.hflip(t).numpy(), t.numpy()[:, :, ::-1])
    n = F.normalize(t, [0.5] * 3, [0.5] * 3)
    np.testing.assert_allclose(n.numpy(), (t.numpy() - 0.5) / 0.5, atol=1e-6)


def test_random_transforms():
    import random

    random.seed(0)
    np.random.seed(0)
    a = _img(32, 40)
    assert T.RandomResizedCrop(16)(a).shape == (16, 16, 3)
    assert T.ColorJitter(0.4, 0.4, 0.4, 0.1)(a).shape == a.shape
    assert T.RandomErasing(prob=1.0)(a).shape == a.shape
    assert np.array_equal(T.RandomAffine(0)(a), a)
    assert T.RandomRotation(30)(a).shape == a.shape
    assert T.RandomPerspective(prob=1.0)(a).shape == a.shape
    assert T.Grayscale()(a).shape == (32, 40, 1)   # the cv2 backend keeps a channel axis
    assert T.Pad(2)(a).shape == (36, 44, 3)
    assert T.RandomCrop(20, padding=2)(a).shape == (20, 20, 3)
    assert np.array_equal(T.BrightnessTransform(0.0)(a), a)
    img, mask = T.RandomHorizontalFlip(1.0, keys=("image", "mask"))((a, a[..., 0]))
    assert np.array_equal(img, a[:, ::-1]) and np.array_equal(mask, a[:, ::-1, 0])
    pipe = T.Compose([T.Resize(16), T.CenterCrop(16), T.ToTensor(), T.Normalize([0.5] * 3, [0.5] * 3)])
    out = pipe(Image.fromarray(a))
    assert list(out.shape) == [3, 16, 16]
