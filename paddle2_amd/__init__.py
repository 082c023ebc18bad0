"""paddle2_amd — an MI355X-native deep-learning framework with PaddlePaddle's ``paddle.*`` API.

Compute path: PyTorch-ROCm tensors + hand-written HIP/CDNA4 kernels (``paddle2_amd._C``, built for
gfx950) + RCCL collectives over xGMI (``torch.distributed`` backend "nccl" == RCCL on ROCm).

``import paddle2_amd as paddle`` gives the familiar surface: Tensor ops, nn, optimizer, amp, io,
autograd, distributed/fleet, vision, hapi (Model.fit), static/jit, profiler, device.
"""
from __future__ import annotations

import torch as _torch  # noqa: F401  (brings up the HIP runtime before our extension loads)

from .device import allocator as _allocator

_allocator._maybe_enable_from_env()  # FLAGS_use_native_allocator: must precede the first device allocation

from .framework import dtype as _dtype_mod
from .framework.dtype import (bfloat16, bool_ as bool, complex64, complex128, float8_e4m3fn, float8_e5m2,  # noqa: F401,A001
                              float16, float32, float64, get_default_dtype, int8, int16, int32, int64,
                              set_default_dtype, uint8, finfo, iinfo)
from .framework.flags import get_flags, set_flags  # noqa: F401
from .framework.grad_mode import enable_grad, is_grad_enabled, no_grad, set_grad_enabled  # noqa: F401
from .framework.io import async_save, clear_async_save_task_queue, load, save  # noqa: F401
from .framework.param import ParamAttr, create_parameter  # noqa: F401
from .framework.place import (CPUPlace, CUDAPinnedPlace, CUDAPlace, CustomPlace, IPUPlace, XPUPlace,  # noqa: F401
                              get_device, is_compiled_with_cinn, is_compiled_with_cuda,
                              is_compiled_with_custom_device, is_compiled_with_distribute, is_compiled_with_rocm,
                              is_compiled_with_xpu, set_device)
from .framework.random import get_cuda_rng_state, get_rng_state, seed, set_cuda_rng_state, set_rng_state  # noqa: F401
from .framework.tensor import Tensor, to_tensor  # noqa: F401
from .tensor import *  # noqa: F401,F403
from .tensor import creation, linalg as _linalg_ops, logic, manipulation, math as _math_ops, random as _random_ops  # noqa: F401
from . import tensor  # noqa: F401

from . import amp, autograd, device, io, nn, ops, optimizer  # noqa: F401,E402
from .autograd import PyLayer, grad  # noqa: F401,E402
from . import distributed  # noqa: F401,E402
from .distributed.parallel import DataParallel  # noqa: F401,E402
from . import metric, vision, hapi, static, jit, profiler, incubate, utils, sparse, linalg, fft, signal  # noqa: F401,E402
from . import distribution, regularizer, callbacks, version  # noqa: F401,E402
from . import _C_ops  # noqa: F401,E402
from . import pir, decomposition  # noqa: F401,E402
from .hapi import Model, summary, flops  # noqa: F401,E402
from .static import enable_static, disable_static, in_dynamic_mode  # noqa: F401,E402
from .framework import dtype  # noqa: F401,E402

__version__ = "3.0.0+mi355x"

dtype = _torch.dtype
float = float32  # noqa: A001
double = float64
half = float16
long = int64


def is_tensor(x):
    return isinstance(x, Tensor)


def in_dygraph_mode():
    return in_dynamic_mode()


def disable_signal_handler():
    pass


def get_cudnn_version():
    return None


def set_printoptions(precision=None, threshold=None, edgeitems=None, sci_mode=None, linewidth=None):
    _torch.set_printoptions(precision=precision, threshold=threshold, edgeitems=edgeitems, sci_mode=sci_mode,
                            linewidth=linewidth)


def numel(x, name=None):
    return manipulation.numel(x)


def shape(input):
    return manipulation.shape(input)


def rank(input):
    return manipulation.rank(input)


def tolist(x):
    return x.tolist()


def where(condition, x=None, y=None, name=None):
    from .tensor.search import where as _w

    return _w(condition, x, y)


def concat(x, axis=0, name=None):
    return manipulation.concat(x, axis)


def stack(x, axis=0, name=None):
    return manipulation.stack(x, axis)


def batch(reader, batch_size, drop_last=False):
    def gen():
        b = []
        for s in reader():
            b.append(s)
            if len(b) == batch_size:
                yield b
                b = []
        if b and not drop_last:
            yield b

    return gen


def check_shape(shape):
    return shape


def get_default_dtype_name():
    return get_default_dtype()


def __getattr__(name):
    # heavier sub-packages load on first use
    import importlib

    if name in ("inference", "serving", "text", "audio", "geometric", "quantization", "onnx", "hub"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(f"module 'paddle2_amd' has no attribute '{name}'")
