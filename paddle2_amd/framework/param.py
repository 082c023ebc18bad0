"""Trainable parameters (reference: python/paddle/base/framework.py ``EagerParamBase``)."""
from __future__ import annotations

import itertools

import torch

from .tensor import Tensor

_param_counter = itertools.count()


def _unique_param_name(prefix="param"):
    return f"{prefix}_{next(_param_counter)}"


class ParamAttr:
    """paddle.ParamAttr (python/paddle/base/param_attr.py)."""

    def __init__(self, name=None, initializer=None, learning_rate=1.0, regularizer=None,
                 trainable=True, do_model_average=True, need_clip=True):
        self.name = name
        self.initializer = initializer
        self.learning_rate = learning_rate
        self.regularizer = regularizer
        self.trainable = trainable
        self.do_model_average = do_model_average
        self.need_clip = need_clip

    @staticmethod
    def _to_attr(arg):
        if arg is None:
            return ParamAttr()
        if isinstance(arg, ParamAttr):
            return arg
        if isinstance(arg, str):
            return ParamAttr(name=arg)
        if isinstance(arg, bool):
            return ParamAttr() if arg else False
        # an initializer instance
        return ParamAttr(initializer=arg)


class Parameter(Tensor):
    """EagerParamBase equivalent: a leaf tensor with ``stop_gradient=False`` and optimizer attrs."""

    _is_param = True
    persistable = True

    def __init__(self, t: torch.Tensor, name=None, trainable=True, optimize_attr=None,
                 regularizer=None, need_clip=True, do_model_average=None, is_distributed=False):
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(t)
        self._t = t.detach().requires_grad_(bool(trainable) and (t.is_floating_point() or t.is_complex()))
        self._t._pd_param = self  # lets a static Program find the parameters it references
        self.name = name or _unique_param_name()
        self.optimize_attr = optimize_attr or {"learning_rate": 1.0}
        self.regularizer = regularizer
        self.need_clip = need_clip
        self.do_model_average = do_model_average
        self.is_distributed = is_distributed
        self._trainable = bool(trainable)

    @property
    def trainable(self):
        return self._trainable

    @trainable.setter
    def trainable(self, v):
        self._trainable = bool(v)
        self.stop_gradient = not v

    def __repr__(self):
        return "Parameter containing:\n" + super().__repr__()

    def __deepcopy__(self, memo):
        p = Parameter(self._t.detach().clone(), name=self.name, trainable=self._trainable,
                      optimize_attr=dict(self.optimize_attr), regularizer=self.regularizer,
                      need_clip=self.need_clip, do_model_average=self.do_model_average,
                      is_distributed=self.is_distributed)
        for k, v in self.__dict__.items():
            if k not in p.__dict__:
                p.__dict__[k] = v
        memo[id(self)] = p
        return p


EagerParamBase = Parameter


def create_parameter(shape, dtype="float32", name=None, attr=None, is_bias=False, default_initializer=None):
    """paddle.create_parameter (python/paddle/tensor/creation.py)."""
    from . import dtype as _dt
    from .place import current_torch_device
    from ..nn import initializer as I

    attr = ParamAttr._to_attr(attr)
    if attr is False:
        return None
    t = torch.empty([int(s) for s in shape], dtype=_dt.convert_dtype(dtype), device=current_torch_device())
    init = attr.initializer or default_initializer
    if init is None:
        init = I.Constant(0.0) if is_bias else I.XavierUniform()
    p = Parameter(t, name=attr.name or name, trainable=attr.trainable,
                  optimize_attr={"learning_rate": attr.learning_rate}, regularizer=attr.regularizer,
                  need_clip=attr.need_clip, do_model_average=attr.do_model_average)
    init(p)
    return p
