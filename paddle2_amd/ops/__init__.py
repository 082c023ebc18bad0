"""paddle2_amd.ops — the op table's hot path (SURVEY §7.1 "Op table").

Tensor-level wrappers around :mod:`.torch_ops` (HIP kernels on the MI355X).  The reference
registers these as Phi GPU kernels (rms_norm, fused_rotary_position_embedding, swiglu,
flash_attn, c_embedding, cross_entropy_with_softmax, adamw_); here each maps to one
hand-written CDNA4 kernel pair (forward/backward).
"""
from __future__ import annotations

from ..framework.tensor import Tensor
from . import _native, torch_ops
from ._native import available as native_available

_wrap = Tensor._wrap


def _u(x):
    return None if x is None else (x._t if isinstance(x, Tensor) else x)


def rms_norm(x, weight, epsilon=1e-6, residual=None):
    r = torch_ops.rms_norm(_u(x), _u(weight), epsilon, _u(residual))
    if residual is not None:
        return _wrap(r[0]), _wrap(r[1])
    return _wrap(r)


def layer_norm(x, normalized_shape, weight=None, bias=None, epsilon=1e-5):
    t = x._t
    n = 1
    for s in normalized_shape:
        n *= int(s)
    if len(normalized_shape) == 1:
        r = torch_ops.layer_norm(t, _u(weight), _u(bias), epsilon)
        return _wrap(r)
    # multi-dim normalized_shape: flatten trailing dims
    lead = list(t.shape[: t.dim() - len(normalized_shape)])
    w = None if weight is None else weight._t.reshape(-1)
    b = None if bias is None else bias._t.reshape(-1)
    r = torch_ops.layer_norm(t.reshape(lead + [n]), w, b, epsilon)
    return _wrap(r.reshape(t.shape))


def swiglu(x, y=None):
    return _wrap(torch_ops.swiglu(_u(x), _u(y)))


def embedding(ids, weight, padding_idx=None, start=0):
    return _wrap(torch_ops.embedding(_u(ids), _u(weight), padding_idx, start))


def softmax_cross_entropy(logits, labels, ignore_index=-100):
    return torch_ops.softmax_cross_entropy(_u(logits), _u(labels), ignore_index)


def flash_attention(q, k, v, causal=False, scale=None):
    o, lse = torch_ops.flash_attention(_u(q), _u(k), _u(v), causal, scale)
    return _wrap(o), _wrap(lse)


def rope(x, cos, sin, position_ids=None, style=0, time_major=False):
    return _wrap(torch_ops.rope(_u(x), _u(cos), _u(sin), _u(position_ids), style, time_major))


__all__ = ["rms_norm", "layer_norm", "swiglu", "embedding", "softmax_cross_entropy", "flash_attention", "rope",
           "native_available", "torch_ops", "_native"]
