"""paddle.vision (reference: python/paddle/vision/)."""
from . import datasets, models, ops, transforms  # noqa: F401
from .models import *  # noqa: F401,F403


def set_image_backend(backend):
    pass


def get_image_backend():
    return "cv2"
