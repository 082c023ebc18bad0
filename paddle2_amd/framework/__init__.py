"""Core runtime objects: dtype, place, Tensor, Parameter, RNG, flags, serialization."""
from . import dtype, flags, grad_mode, io, param, place, random, tensor  # noqa: F401
from .random import seed  # noqa: F401
from .io import load, save  # noqa: F401
from .grad_mode import no_grad  # noqa: F401
from .param import ParamAttr  # noqa: F401
from .flags import get_flags, set_flags  # noqa: F401
from . import tensor_types  # noqa: F401,E402
from .tensor_types import SelectedRows, StringTensor, TensorArray  # noqa: F401,E402


def in_dynamic_mode():
    from ..static import in_dynamic_mode as _d

    return _d()


def get_default_dtype():
    return dtype.get_default_dtype()


def set_default_dtype(d):
    return dtype.set_default_dtype(d)
