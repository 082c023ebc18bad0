"""paddle.incubate.nn.memory_efficient_attention (reference python/paddle/incubate/nn/memory_efficient_attention.py,
op memory_efficient_attention): q/k/v [B, S, H, D].  No bias / LowerTriangularMask run the native flash kernel
(causal for the mask); BlockDiagonal(Causal)Mask over packed sequences runs the varlen flash kernel from the
masks' cumulative offsets; a tensor bias (or mask + tensor bias) runs the fp32-accumulating math path."""
from __future__ import annotations

import math

import torch

from ...framework.tensor import Tensor
from .attn_bias import BlockDiagonalMask, LowerTriangularMask, LowerTriangularMaskWithTensorBias


def _raw(x):
    return x._t if isinstance(x, Tensor) else x


def memory_efficient_attention(query, key, value, attn_bias=None, p=0.0, scale=None, training=True):
    from ...ops import torch_ops as T

    q, k, v = _raw(query), _raw(key), _raw(value)
    D = q.shape[-1]
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(D)
    drop = float(p) if training else 0.0
    if drop == 0.0 and (attn_bias is None or type(attn_bias) is LowerTriangularMask):
        out, _ = T.flash_attention(q, k, v, attn_bias is not None, scale)
        return Tensor._wrap(out)
    if drop == 0.0 and isinstance(attn_bias, BlockDiagonalMask):
        qi, ki = attn_bias.q_seqinfo, attn_bias.k_seqinfo
        cu_q = torch.tensor(qi.seqstart, dtype=torch.int32, device=q.device)
        cu_k = torch.tensor(ki.seqstart, dtype=torch.int32, device=q.device)
        out = T.flash_attention_varlen(q.reshape(-1, q.shape[-2], D), k.reshape(-1, k.shape[-2], D),
                                       v.reshape(-1, v.shape[-2], D), cu_q, cu_k, qi.max_seqlen, ki.max_seqlen,
                                       attn_bias._causal, scale)[0]
        return Tensor._wrap(out.reshape(q.shape))
    # math path: explicit bias (tensor, mask+bias) or dropout
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))          # [B, H, S, D]
    if kf.shape[1] != qf.shape[1]:
        g = qf.shape[1] // kf.shape[1]
        kf, vf = kf.repeat_interleave(g, 1), vf.repeat_interleave(g, 1)
    s = (qf @ kf.transpose(-1, -2)) * scale
    if isinstance(attn_bias, (LowerTriangularMask, BlockDiagonalMask)) or isinstance(
            attn_bias, LowerTriangularMaskWithTensorBias):
        s = s + attn_bias.materialize(s.shape, torch.float32, s.device)
    elif attn_bias is not None:
        s = s + _raw(attn_bias).float()
    pr = torch.softmax(s, -1)
    if drop > 0.0:
        pr = torch.nn.functional.dropout(pr, drop, True)
    return Tensor._wrap((pr @ vf).transpose(1, 2).to(q.dtype))


def memory_efficient_attention_op(query, key, value, bias=None, cu_seqlens_q=None, cu_seqlens_k=None,
                                  causal_diagonal=None, seqlen_k=None, max_seqlen_q=-1, max_seqlen_k=-1, causal=False,
                                  dropout_p=0.0, scale=-1.0, is_test=True):
    """The ops.yaml signature (output, logsumexp, seed_and_offset)."""
    ab = LowerTriangularMask() if causal and bias is None else bias
    if causal and bias is not None:
        ab = LowerTriangularMaskWithTensorBias(bias)
    out = memory_efficient_attention(query, key, value, ab, dropout_p, None if scale is None or scale < 0 else scale,
                                     not is_test)
    return out, None, None
