"""paddle.nn.utils (reference: python/paddle/nn/utils/)."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor
from .clip import clip_grad_norm_, clip_grad_value_  # noqa: F401


def parameters_to_vector(parameters, name=None):
    return Tensor._wrap(torch.cat([p._t.detach().reshape(-1) for p in parameters]))


def vector_to_parameters(vec, parameters, name=None):
    off = 0
    for p in parameters:
        n = p._t.numel()
        with torch.no_grad():
            p._t.copy_(vec._t[off:off + n].reshape(p._t.shape))
        off += n


def weight_norm(layer, name="weight", dim=0):
    from ..framework.param import Parameter

    w = getattr(layer, name)
    t = w._t.detach()
    dims = [d for d in range(t.dim()) if d != dim]
    g = Parameter(torch.linalg.vector_norm(t, dim=dims, keepdim=True))
    v = Parameter(t.clone())
    del layer._parameters[name]
    layer.add_parameter(name + "_g", g)
    layer.add_parameter(name + "_v", v)

    def hook(l, inputs):
        vv = getattr(l, name + "_v")._t
        gg = getattr(l, name + "_g")._t
        object.__setattr__(l, name, Tensor._wrap(vv * (gg / torch.linalg.vector_norm(vv, dim=dims, keepdim=True))))

    layer.register_forward_pre_hook(hook)
    hook(layer, None)
    return layer


def remove_weight_norm(layer, name="weight"):
    from ..framework.param import Parameter

    w = getattr(layer, name)
    del layer._parameters[name + "_g"]
    del layer._parameters[name + "_v"]
    layer._forward_pre_hooks.clear()
    layer.__dict__.pop(name, None)
    layer.add_parameter(name, Parameter(w._t.detach()))
    return layer


def spectral_norm(layer, name="weight", n_power_iterations=1, eps=1e-12, dim=None):
    return layer
