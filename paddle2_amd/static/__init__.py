"""paddle.static: Program capture, Executor, backward/optimizer in static mode, inference-model
save/load (reference: python/paddle/static/, python/paddle/base/framework.py, executor.py,
static/io.py save_inference_model/load_inference_model)."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor
from . import graph as _g
from .executor import BuildStrategy, CompiledProgram, ExecutionStrategy, Executor, Scope, global_scope  # noqa: F401
from .graph import Program, SymTensor, default_main_program, default_startup_program, graph_op  # noqa: F401
from .graph import program_guard  # noqa: F401
from .io import (deserialize_persistables, deserialize_program, load, load_inference_model, load_program_state,  # noqa
                 save, save_inference_model, serialize_persistables, serialize_program, set_program_state)
from .input import InputSpec  # noqa: F401

Variable = Tensor  # a static Variable is a Tensor whose storage is a SymTensor


def enable_static():
    _g._state.static = True


def disable_static(place=None):
    _g._state.static = False


def in_dynamic_mode():
    return not _g._state.static


_static_mode_enabled = lambda: _g._state.static  # noqa: E731


def data(name, shape, dtype=None, lod_level=0):
    """Feed placeholder.  Unknown dims (-1 / None) get size 1 for build-time shape inference; ops
    that only use -1 / 0 reshapes stay valid for any runtime size."""
    from ..framework.dtype import convert_dtype, get_default_dtype

    dt = convert_dtype(dtype) if dtype is not None else convert_dtype(get_default_dtype())
    shp = [1 if (d is None or d < 0) else int(d) for d in shape]
    prog = default_main_program()
    v = prog.new_var(torch.empty(shp, dtype=dt, device="meta"), name=name)
    prog.feeds[name] = v
    t = Tensor._wrap(v)
    t.name = name
    t.stop_gradient = True
    return t


def _sym(x):
    t = x._t if isinstance(x, Tensor) else x
    return t if isinstance(t, SymTensor) else None


def append_backward(loss, parameter_list=None, no_grad_set=None, callbacks=None, checkpoints=None):
    """Record the backward pass; returns [(param, grad_variable)] like the reference."""
    s = _sym(loss)
    assert s is not None, "append_backward expects a static Variable"
    prog = s._program
    prog.append_special("backward", loss=s._vid)
    params = parameter_list if parameter_list is not None else prog.all_parameters()
    out = []
    for p in params:
        if p.stop_gradient:
            continue
        gv = prog.new_var(torch.empty_like(p._t, device="meta"), name=f"{p.name}@GRAD")
        prog.append_special("param_grad", param=p, out=gv._vid)
        out.append((p, Tensor._wrap(gv)))
    return out


def gradients(targets, inputs, target_gradients=None, no_grad_set=None):
    tl = targets if isinstance(targets, (list, tuple)) else [targets]
    il = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    prog = _sym(tl[0])._program
    outs = []
    ins = []
    for x in il:
        s = _sym(x)
        ins.append(s._vid if s is not None else x._t)
        outs.append(prog.new_var(torch.empty_like(s if s is not None else x._t, device="meta")))
    prog.append_special("grad", targets=[_sym(t)._vid for t in tl], inputs=ins, outs=[o._vid for o in outs])
    return [Tensor._wrap(o) for o in outs]


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from ..framework.param import create_parameter as _cp

    return _cp(shape, dtype, name=name, attr=attr, is_bias=is_bias, default_initializer=default_initializer)


def create_global_var(shape, value, dtype, persistable=False, force_cpu=False, name=None):
    from ..tensor.creation import full

    return full(shape, value, dtype)


def cpu_places(device_count=None):
    from ..framework.place import CPUPlace

    return [CPUPlace()] * (device_count or 1)


def cuda_places(device_ids=None):
    from ..framework.place import CUDAPlace

    ids = device_ids if device_ids is not None else list(range(max(1, torch.cuda.device_count())))
    return [CUDAPlace(i) for i in ids]


class _NullCtx:
    def __init__(self, *a, **k):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


name_scope = _NullCtx


class device_guard:
    """paddle.static.device_guard (reference base/framework.py device_guard): ops recorded inside carry
    ``op_device`` ("gpu:<pipeline stage>", "gpu:all"; "cpu" / bare "gpu" are accepted and recorded as
    given) — HybridParallelInferenceHelper splits a program into pipeline stages by it."""

    def __init__(self, device=None):
        if device is not None and not (device in ("cpu", "gpu") or device.startswith("gpu:")):
            raise ValueError(f"device_guard: expected 'cpu', 'gpu', 'gpu:<n>' or 'gpu:all', got {device!r}")
        self.device = device

    def __enter__(self):
        self._prev = _g._state.op_device
        _g._state.op_device = self.device
        return self

    def __exit__(self, *a):
        _g._state.op_device = self._prev
        return False


scope_guard = _NullCtx
ipu_shard_guard = _NullCtx


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    return func(x)


from . import nn  # noqa: E402,F401
from .extras import (ExponentialMovingAverage, IpuCompiledProgram, IpuStrategy, Print,  # noqa: E402,F401
                     WeightNormParamAttr, accuracy, auc, ctr_metric_bundle, load_from_file, normalize_program,
                     save_to_file, set_ipu_shard, xpu_places)
