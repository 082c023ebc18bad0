"""Normalisation (reference: python/paddle/nn/functional/norm.py).

``layer_norm``/``rms_norm`` route to the hand-written HIP kernels in :mod:`paddle2_amd.ops`
when the input lives on the MI355X.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ...framework.tensor import Tensor
from ...amp import amp_op as _amp_op  # noqa: E402

_wrap = Tensor._wrap


@_amp_op("batch_norm")
def batch_norm(x, running_mean, running_var, weight=None, bias=None, training=False, momentum=0.9,
               epsilon=1e-05, data_format="NCHW", use_global_stats=None, name=None, act=None, residual=None):
    """Paddle batch_norm; ``act`` ('relu') and ``residual`` (added before the activation) are
    fused into the HIP kernel for channels-last activations on the MI355X (the
    fused_bn_add_activation op of the reference)."""
    from ...ops.torch_ops import batch_norm_act

    t = x._t
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    use_batch = training if use_global_stats is None else (not use_global_stats)
    z = residual._t if isinstance(residual, Tensor) else residual
    w = None if weight is None else weight._t
    b = None if bias is None else bias._t
    if t.dim() >= 2:
        tl = t if cl else t.movedim(1, -1)  # channels-last view (contiguous for channels_last memory)
        zl = None if z is None else (z if cl else z.movedim(1, -1))
        out = batch_norm_act(tl, running_mean._t, running_var._t, w, b, use_batch, momentum, epsilon, act, zl)
        return _wrap(out if cl else out.movedim(-1, 1))
    out = F.batch_norm(t, running_mean._t, running_var._t, w, b, use_batch, 1.0 - momentum, epsilon)
    if z is not None:
        out = out + z
    if act == "relu":
        out = torch.relu(out)
    return _wrap(out)


@_amp_op("layer_norm")
def layer_norm(x, normalized_shape, weight=None, bias=None, epsilon=1e-05, name=None):
    if isinstance(normalized_shape, int):
        normalized_shape = [normalized_shape]
    from ...ops import layer_norm as _ln

    return _ln(x, list(normalized_shape), weight, bias, epsilon)


def rms_norm(x, normalized_shape, weight=None, epsilon=1e-6, name=None):
    from ...ops import rms_norm as _rms

    return _rms(x, weight, epsilon)


def instance_norm(x, running_mean=None, running_var=None, weight=None, bias=None, use_input_stats=True,
                  momentum=0.9, eps=1e-05, data_format="NCHW", name=None):
    t = x._t
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    if cl:
        t = t.movedim(-1, 1)
    out = F.instance_norm(t, None if running_mean is None else running_mean._t,
                          None if running_var is None else running_var._t,
                          None if weight is None else weight._t, None if bias is None else bias._t,
                          use_input_stats, 1.0 - momentum, eps)
    if cl:
        out = out.movedim(1, -1)
    return _wrap(out)


def group_norm(x, num_groups, epsilon=1e-05, weight=None, bias=None, data_format="NCHW", name=None):
    t = x._t
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    if cl:
        t = t.movedim(-1, 1)
    out = F.group_norm(t, num_groups, None if weight is None else weight._t,
                       None if bias is None else bias._t, epsilon)
    if cl:
        out = out.movedim(1, -1)
    return _wrap(out)


def local_response_norm(x, size, alpha=0.0001, beta=0.75, k=1.0, data_format="NCHW", name=None):
    t = x._t
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    if cl:
        t = t.movedim(-1, 1)
    out = F.local_response_norm(t, size, alpha, beta, k)
    if cl:
        out = out.movedim(1, -1)
    return _wrap(out)
