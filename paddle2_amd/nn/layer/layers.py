"""``paddle.nn.Layer`` (reference: python/paddle/nn/layer/layers.py, 2,699 LoC).

Parameters/sub-layers/buffers are tracked in ordered dicts; ``state_dict`` keys are the
structured names Paddle uses (``linear.weight``), which is what ``.pdparams`` files contain.
"""
from __future__ import annotations

import collections
import itertools
import re
from typing import Callable

import numpy as np
import torch

from ...framework import dtype as _dt
from ...framework import nan_inf as _nan_inf
from ...framework.param import Parameter, ParamAttr, create_parameter
from ...framework.tensor import Tensor

_layer_uid = collections.defaultdict(itertools.count)


def _camel_to_snake(name):
    s = re.sub("(.)([A-Z][a-z]+)", r"\1_\2", name)
    return re.sub("([a-z0-9])([A-Z])", r"\1_\2", s).lower()


class HookRemoveHelper:
    def __init__(self, hooks: dict, hid: int):
        self._hooks = hooks
        self._hid = hid

    def remove(self):
        self._hooks.pop(self._hid, None)


class Layer:
    """Base building block of all models."""

    training = True

    def __init__(self, name_scope=None, dtype="float32"):
        object.__setattr__(self, "_parameters", collections.OrderedDict())
        object.__setattr__(self, "_sub_layers", collections.OrderedDict())
        object.__setattr__(self, "_buffers", collections.OrderedDict())
        object.__setattr__(self, "_non_persistable_buffer_names_set", set())
        object.__setattr__(self, "_forward_pre_hooks", collections.OrderedDict())
        object.__setattr__(self, "_forward_post_hooks", collections.OrderedDict())
        object.__setattr__(self, "_hook_id", itertools.count())
        object.__setattr__(self, "training", True)
        object.__setattr__(self, "_dtype", dtype)
        if name_scope is None:
            name_scope = _camel_to_snake(self.__class__.__name__)
        object.__setattr__(self, "_full_name", f"{name_scope}_{next(_layer_uid[name_scope])}")
        object.__setattr__(self, "_helper", None)
        object.__setattr__(self, "_casted_by_pure_fp16", False)
        object.__setattr__(self, "_state_dict_hooks", collections.OrderedDict())

    # ------------------------------------------------------------ attributes
    def __setattr__(self, name, value):
        params = self.__dict__.get("_parameters")
        if isinstance(value, Parameter):
            if params is None:
                raise RuntimeError("super().__init__() must be called before assigning parameters")
            self._sub_layers.pop(name, None)
            self._buffers.pop(name, None)
            self.__dict__.pop(name, None)
            params[name] = value
            if value.name is None:
                value.name = f"{self._full_name}.{name}"
            return
        if isinstance(value, Layer):
            if params is None:
                raise RuntimeError("super().__init__() must be called before assigning sub-layers")
            params.pop(name, None)
            self._buffers.pop(name, None)
            self.__dict__.pop(name, None)
            self._sub_layers[name] = value
            return
        if params is not None:
            if name in params:
                if value is None:
                    params[name] = None
                    return
                raise TypeError(f"cannot assign {type(value)} to parameter {name}")
            if name in self._sub_layers:
                if value is None:
                    self._sub_layers[name] = None
                    return
            if name in self._buffers:
                if value is None or isinstance(value, Tensor):
                    self._buffers[name] = value
                    return
        object.__setattr__(self, name, value)

    def __getattr__(self, name):
        d = self.__dict__
        if "_parameters" in d:
            p = d["_parameters"]
            if name in p:
                return p[name]
            s = d["_sub_layers"]
            if name in s:
                return s[name]
            b = d["_buffers"]
            if name in b:
                return b[name]
        raise AttributeError(f"'{type(self).__name__}' object has no attribute '{name}'")

    def __delattr__(self, name):
        for store in ("_parameters", "_sub_layers", "_buffers"):
            if name in self.__dict__.get(store, {}):
                del self.__dict__[store][name]
                return
        object.__delattr__(self, name)

    def __dir__(self):
        return list(super().__dir__()) + list(self._parameters) + list(self._sub_layers) + list(self._buffers)

    # ------------------------------------------------------------ creation
    def create_parameter(self, shape, attr=None, dtype=None, is_bias=False, default_initializer=None):
        dtype = dtype or self._dtype or "float32"
        return create_parameter(shape, dtype=dtype, attr=attr, is_bias=is_bias,
                                default_initializer=default_initializer)

    def create_variable(self, name=None, persistable=None, dtype=None):
        from ...tensor.creation import create_tensor

        return create_tensor(dtype or self._dtype, name=name, persistable=bool(persistable))

    create_tensor = create_variable

    def add_parameter(self, name, parameter):
        if parameter is None:
            self._parameters[name] = None
            return None
        if not isinstance(parameter, Parameter):
            raise TypeError("add_parameter expects a Parameter")
        self._parameters[name] = parameter
        return parameter

    def add_sublayer(self, name, sublayer):
        self._sub_layers[str(name)] = sublayer
        return sublayer

    def register_buffer(self, name, tensor, persistable=True):
        if tensor is not None and not isinstance(tensor, Tensor):
            raise TypeError("buffer must be a Tensor")
        self._buffers[name] = tensor
        if persistable:
            self._non_persistable_buffer_names_set.discard(name)
        else:
            self._non_persistable_buffer_names_set.add(name)
        if tensor is not None:
            tensor.persistable = persistable

    # ------------------------------------------------------------ traversal
    def named_parameters(self, prefix="", include_sublayers=True, remove_duplicate=True):
        seen = set()
        layers = self.named_sublayers(prefix=prefix, include_self=True) if include_sublayers else [(prefix, self)]
        for lp, layer in layers:
            for k, p in layer._parameters.items():
                if p is None or (remove_duplicate and id(p) in seen):
                    continue
                seen.add(id(p))
                yield (lp + ("." if lp else "") + k), p

    def parameters(self, include_sublayers=True):
        return [p for _, p in self.named_parameters(include_sublayers=include_sublayers)]

    def named_buffers(self, prefix="", include_sublayers=True):
        seen = set()
        layers = self.named_sublayers(prefix=prefix, include_self=True) if include_sublayers else [(prefix, self)]
        for lp, layer in layers:
            for k, b in layer._buffers.items():
                if b is None or id(b) in seen:
                    continue
                seen.add(id(b))
                yield (lp + ("." if lp else "") + k), b

    def buffers(self, include_sublayers=True):
        return [b for _, b in self.named_buffers(include_sublayers=include_sublayers)]

    def named_children(self):
        seen = set()
        for k, l in self._sub_layers.items():
            if l is not None and id(l) not in seen:
                seen.add(id(l))
                yield k, l

    def children(self):
        return [l for _, l in self.named_children()]

    def named_sublayers(self, prefix="", include_self=False, layers_set=None):
        if layers_set is None:
            layers_set = set()
        if include_self and id(self) not in layers_set:
            layers_set.add(id(self))
            yield prefix, self
        for k, l in self._sub_layers.items():
            if l is None:
                continue
            p = prefix + ("." if prefix else "") + k
            if id(l) in layers_set:
                continue
            layers_set.add(id(l))
            yield p, l
            yield from l.named_sublayers(prefix=p, include_self=False, layers_set=layers_set)

    def sublayers(self, include_self=False):
        return [l for _, l in self.named_sublayers(include_self=include_self)]

    def apply(self, fn: Callable):
        for l in self.children():
            l.apply(fn)
        fn(self)
        return self

    def full_name(self):
        return self._full_name

    # ------------------------------------------------------------ modes
    def train(self, mode=True):
        for l in self.sublayers(include_self=True):
            object.__setattr__(l, "training", bool(mode))
        return self

    def eval(self):
        return self.train(False)

    # ------------------------------------------------------------ hooks / call
    def register_forward_pre_hook(self, hook):
        hid = next(self._hook_id)
        self._forward_pre_hooks[hid] = hook
        return HookRemoveHelper(self._forward_pre_hooks, hid)

    def register_forward_post_hook(self, hook):
        hid = next(self._hook_id)
        self._forward_post_hooks[hid] = hook
        return HookRemoveHelper(self._forward_post_hooks, hid)

    def register_state_dict_hook(self, hook):
        hid = next(self._hook_id)
        self._state_dict_hooks[hid] = hook
        return HookRemoveHelper(self._state_dict_hooks, hid)

    def forward(self, *args, **kwargs):
        raise NotImplementedError

    def __call__(self, *args, **kwargs):
        if self._forward_pre_hooks:
            for hook in list(self._forward_pre_hooks.values()):
                r = hook(self, args)
                if r is not None:
                    args = r if isinstance(r, tuple) else (r,)
        out = self.forward(*args, **kwargs)
        if _nan_inf.enabled:
            _nan_inf.check_layer(self, out)
        if self._forward_post_hooks:
            for hook in list(self._forward_post_hooks.values()):
                r = hook(self, args, out)
                if r is not None:
                    out = r
        return out

    # ------------------------------------------------------------ state
    def _state_dict_impl(self, destination, include_sublayers, structured_name_prefix, include_non_persistable_buffer=False):
        for k, p in self._parameters.items():
            if p is not None:
                destination[structured_name_prefix + k] = p
        for k, b in self._buffers.items():
            if b is None:
                continue
            if not include_non_persistable_buffer and k in self._non_persistable_buffer_names_set:
                continue
            destination[structured_name_prefix + k] = b
        if include_sublayers:
            for k, l in self._sub_layers.items():
                if l is not None:
                    l._state_dict_impl(destination, include_sublayers, structured_name_prefix + k + ".",
                                       include_non_persistable_buffer)
        return destination

    def state_dict(self, destination=None, include_sublayers=True, structured_name_prefix="", use_hook=True,
                   keep_vars=True):
        dest = collections.OrderedDict() if destination is None else destination
        self._state_dict_impl(dest, include_sublayers, structured_name_prefix)
        if use_hook:
            for hook in self._state_dict_hooks.values():
                r = hook(dest)
                if r is not None:
                    dest = r
        return dest

    def to_static_state_dict(self, destination=None, include_sublayers=True, structured_name_prefix="", use_hook=True):
        dest = collections.OrderedDict() if destination is None else destination
        return self._state_dict_impl(dest, include_sublayers, structured_name_prefix, True)

    def set_state_dict(self, state_dict, use_structured_name=True):
        own = self.state_dict(use_hook=False)
        missing, unexpected = [], []
        by_name = {}
        if not use_structured_name:
            by_name = {v.name: k for k, v in own.items()}
        matched = set()
        for k, v in state_dict.items():
            key = k if use_structured_name else by_name.get(k)
            if key is None or key not in own:
                unexpected.append(k)
                continue
            matched.add(key)
            tgt = own[key]
            if isinstance(v, Tensor):
                src = v._t
            elif isinstance(v, np.ndarray):
                src = torch.from_numpy(np.ascontiguousarray(v))
                if v.dtype == np.uint16 and tgt.dtype == torch.bfloat16:
                    src = src.view(torch.bfloat16)
            elif isinstance(v, torch.Tensor):
                src = v
            else:
                src = torch.as_tensor(np.asarray(v))
            if src.dtype == torch.uint16 and tgt._t.dtype == torch.bfloat16:
                src = src.view(torch.bfloat16)
            if list(src.shape) != list(tgt._t.shape):
                raise ValueError(f"{key}: shape mismatch loading {list(src.shape)} into {tgt.shape}")
            with torch.no_grad():
                tgt._t.copy_(src.to(device=tgt._t.device, dtype=tgt._t.dtype))
        for k in own:
            if k not in matched:
                missing.append(k)
        return missing, unexpected

    set_dict = set_state_dict
    load_dict = set_state_dict

    # ------------------------------------------------------------ dtype/device
    def _apply_to_tensors(self, fn, include_buffers=True):
        for p in self.parameters():
            with torch.no_grad():
                new = fn(p._t)
            if new is not p._t:
                rg = p._t.requires_grad
                p._t = new.detach().requires_grad_(rg)
        if include_buffers:
            for b in self.buffers():
                b._t = fn(b._t)
        return self

    def to(self, device=None, dtype=None, blocking=None):
        from ...framework.place import _parse_device

        dev = _parse_device(device) if device is not None else None
        dt = _dt.convert_dtype(dtype) if dtype is not None else None

        def fn(t):
            if dev is not None:
                t = t.to(dev)
            if dt is not None and t.is_floating_point():
                t = t.to(dt)
            return t

        return self._apply_to_tensors(fn)

    def astype(self, dtype=None):
        return self.to(dtype=dtype)

    def float(self, excluded_layers=None):
        return self.to(dtype="float32")

    def float16(self, excluded_layers=None):
        return self.to(dtype="float16")

    half = float16

    def bfloat16(self, excluded_layers=None):
        return self.to(dtype="bfloat16")

    def cuda(self):
        return self.to("gpu")

    def cpu(self):
        return self.to("cpu")

    def clear_gradients(self, set_to_zero=True):
        for p in self.parameters():
            if p.trainable:
                p.clear_gradient(set_to_zero)

    clear_grad = clear_gradients

    # ------------------------------------------------------------ repr
    def extra_repr(self):
        return ""

    def __repr__(self):
        lines = []
        for k, l in self._sub_layers.items():
            r = repr(l).replace("\n", "\n  ")
            lines.append(f"({k}): {r}")
        main = f"{type(self).__name__}({self.extra_repr()}"
        if lines:
            main += "\n  " + "\n  ".join(lines) + "\n"
        return main + ")"

    def _dygraph_call_func(self, *args, **kwargs):
        return self(*args, **kwargs)

    def __getstate__(self):
        return self.__dict__

    def __setstate__(self, state):
        self.__dict__.update(state)


def _as_param_attr(attr):
    return ParamAttr._to_attr(attr)
