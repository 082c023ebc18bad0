"""paddle.utils.dlpack."""
import torch

from ..framework.tensor import Tensor


def to_dlpack(x):
    return torch.utils.dlpack.to_dlpack(x._t)


def from_dlpack(dlpack):
    return Tensor._wrap(torch.utils.dlpack.from_dlpack(dlpack))
