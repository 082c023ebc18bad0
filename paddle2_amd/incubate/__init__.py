"""paddle.incubate (reference: python/paddle/incubate/)."""
from . import nn  # noqa: F401


def softmax_mask_fuse(x, mask, name=None):
    """softmax(x + mask) over the last axis of [B, H, Sq, Sk] scores, mask [B, 1, Sq, Sk] shared by heads
    (reference: python/paddle/incubate/operators/softmax_mask_fuse.py; fused HIP kernel on the GPU)."""
    from ..framework.tensor import Tensor
    from ..ops import torch_ops as T

    return Tensor._wrap(T.softmax_mask(x._t, mask._t, causal=False))


def softmax_mask_fuse_upper_triangle(x, name=None):
    """Causal softmax of square [B, H, S, S] scores; entries above the diagonal are exactly 0 (reference:
    python/paddle/incubate/operators/softmax_mask_fuse_upper_triangle.py)."""
    from ..framework.tensor import Tensor
    from ..ops import torch_ops as T

    return Tensor._wrap(T.softmax_mask(x._t, None, causal=True))


def __getattr__(name):
    import importlib

    if name in ("distributed", "autograd", "optimizer", "asp", "tensor", "fp8", "autotune", "jit", "layers",
                "operators", "multiprocessing", "checkpoint", "framework"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
