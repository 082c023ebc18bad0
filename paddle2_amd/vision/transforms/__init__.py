"""paddle.vision.transforms (reference: python/paddle/vision/transforms/__init__.py)."""
from .functional import (adjust_brightness, adjust_contrast, adjust_hue, adjust_saturation, affine,  # noqa: F401
                         center_crop, crop, erase, hflip, normalize, pad, perspective, resize, rotate, to_grayscale,
                         to_tensor, vflip)
from .transforms import (BaseTransform, BrightnessTransform, CenterCrop, ColorJitter, Compose,  # noqa: F401
                         ContrastTransform, Grayscale, HueTransform, Normalize, Pad, RandomAffine, RandomCrop,
                         RandomErasing, RandomHorizontalFlip, RandomPerspective, RandomResizedCrop, RandomRotation,
                         RandomVerticalFlip, Resize, SaturationTransform, ToTensor, Transpose)
from . import functional  # noqa: F401

__all__ = ["BaseTransform", "Compose", "Resize", "RandomResizedCrop", "CenterCrop", "RandomHorizontalFlip",
           "RandomVerticalFlip", "Transpose", "Normalize", "BrightnessTransform", "SaturationTransform",
           "ContrastTransform", "HueTransform", "ColorJitter", "RandomCrop", "Pad", "RandomAffine", "RandomRotation",
           "RandomPerspective", "Grayscale", "ToTensor", "RandomErasing", "to_tensor", "hflip", "vflip", "resize",
           "pad", "affine", "rotate", "perspective", "to_grayscale", "crop", "center_crop", "adjust_brightness",
           "adjust_contrast", "adjust_hue", "normalize", "erase"]
