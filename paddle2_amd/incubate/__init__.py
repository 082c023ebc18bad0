"""paddle.incubate (reference: python/paddle/incubate/)."""
from . import nn  # noqa: F401


def __getattr__(name):
    import importlib

    if name in ("distributed", "autograd", "optimizer", "asp", "tensor", "fp8", "autotune"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
