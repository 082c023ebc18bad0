"""Attention functional API (reference: python/paddle/nn/functional/flash_attention.py).

All entry points take Paddle's [batch, seq, heads, head_dim] layout and run the hand-written
CDNA4 flash-attention kernel (paddle2_amd.ops.torch_ops.flash_attention) on the MI355X.
"""
from __future__ import annotations

import math

import torch

from ...framework.tensor import Tensor

_wrap = Tensor._wrap


def flash_attention(query, key, value, dropout=0.0, causal=False, return_softmax=False, *, fixed_seed_offset=None,
                    rng_name="", training=True, name=None):
    """Returns (out, softmax) like paddle: softmax is None unless return_softmax."""
    from ...ops.torch_ops import flash_attention as _fa

    q, k, v = query._t, key._t, value._t
    if dropout > 0.0 and training:
        out = _sdpa_dropout(q, k, v, dropout, causal)
        return _wrap(out), None
    out, lse = _fa(q, k, v, causal)
    sm = None
    if return_softmax:
        s = torch.einsum("bqhd,bkhd->bhqk", q.float(), _rep(k, q.shape[2]).float()) / math.sqrt(q.shape[-1])
        sm = _wrap(torch.exp(s - lse[..., None]).to(q.dtype))
    return _wrap(out), sm


def _rep(k, hq):
    hk = k.shape[2]
    return k if hk == hq else k.repeat_interleave(hq // hk, 2)


def _sdpa_dropout(q, k, v, p, causal):
    qt, kt, vt = q.transpose(1, 2), _rep(k, q.shape[2]).transpose(1, 2), _rep(v, q.shape[2]).transpose(1, 2)
    o = torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, dropout_p=p, is_causal=causal)
    return o.transpose(1, 2)


def flash_attn_qkvpacked(qkv, dropout=0.0, causal=False, return_softmax=False, *, fixed_seed_offset=None,
                         rng_name="", training=True, name=None):
    """qkv: [b, s, num_group + 2, num_heads_k, d] (paddle packed GQA layout)."""
    t = qkv._t
    ng = t.shape[2] - 2
    b, s, _, hk, d = t.shape
    q = t[:, :, :ng].reshape(b, s, ng * hk, d)
    k = t[:, :, ng]
    v = t[:, :, ng + 1]
    return flash_attention(_wrap(q), _wrap(k), _wrap(v), dropout, causal, return_softmax, training=training)


def flash_attn_unpadded(query, key, value, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, scale,
                        dropout=0.0, causal=False, return_softmax=False, fixed_seed_offset=None, rng_name="",
                        training=True, name=None):
    """Varlen attention over packed [total_tokens, heads, d] with cumulative sequence offsets (one launch of the
    kVarlen MFMA kernel for all sequences; reference flash_attention.py:652)."""
    from ...ops.torch_ops import flash_attention_varlen

    out, _ = flash_attention_varlen(query._t, key._t, value._t, cu_seqlens_q._t, cu_seqlens_k._t, int(max_seqlen_q),
                                    int(max_seqlen_k), causal, scale)
    return _wrap(out), None


def flash_attn_varlen_qkvpacked(qkv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, scale, dropout=0.0,
                                causal=False, return_softmax=False, fixed_seed_offset=None, rng_name="",
                                varlen_padded=True, training=True, name=None):
    t = qkv._t
    ng = t.shape[1] - 2
    tot, _, hk, d = t.shape
    q = t[:, :ng].reshape(tot, ng * hk, d)
    return flash_attn_unpadded(_wrap(q), _wrap(t[:, ng]), _wrap(t[:, ng + 1]), cu_seqlens_q, cu_seqlens_k,
                               max_seqlen_q, max_seqlen_k, scale, dropout, causal, return_softmax, training=training)


def scaled_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, training=True,
                                 name=None):
    if attn_mask is None and (dropout_p == 0.0 or not training):
        out, _ = flash_attention(query, key, value, 0.0, is_causal, training=training)
        return out
    q, k, v = query._t, key._t, value._t
    qt, kt, vt = q.transpose(1, 2), _rep(k, q.shape[2]).transpose(1, 2), _rep(v, q.shape[2]).transpose(1, 2)
    m = None if attn_mask is None else attn_mask._t
    o = torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, attn_mask=m,
                                                         dropout_p=dropout_p if training else 0.0, is_causal=is_causal)
    return _wrap(o.transpose(1, 2))


def flashmask_attention(query, key, value, startend_row_indices=None, *, dropout=0.0, causal=False, window_size=None,
                        return_softmax_lse=False, return_seed_offset=False, fixed_seed_offset=None, rng_name="",
                        training=True, name=None):
    """FlashMask (reference flash_attention.py:1098): per-key-column row-range masks [b, h, s_k, {1,2,4}]
    (LTS / LTE / UTS / UTE).  Runs the kMask MFMA kernel, which skips fully masked (query block x key tile)
    products and only evaluates element masks on partially masked tiles; window_size is lowered to row ranges
    as in the reference."""
    from ...ops.torch_ops import flash_attention_mask

    q, k, v = query._t, key._t, value._t
    sq = q.shape[1]
    if window_size is not None:
        if startend_row_indices is not None:
            raise ValueError("can't use window_size with startend_row_indices")
        if isinstance(window_size, int):
            window_size = (window_size, window_size)
        lts = torch.arange(window_size[0] + 1, sq + window_size[0] + 1, dtype=torch.int32, device=q.device)
        if causal:
            idx = lts.clamp(max=sq).view(1, 1, sq, 1)
        else:
            ute = torch.arange(-window_size[1], sq - window_size[1], dtype=torch.int32, device=q.device)
            idx = torch.stack([lts, ute], -1).clamp(0, sq).view(1, 1, sq, 2)
        startend_row_indices = _wrap(idx.expand(q.shape[0], 1, sq, idx.shape[-1]).contiguous())
    if startend_row_indices is None:
        out, _ = flash_attention(query, key, value, dropout, causal, training=training)
        return (out, None) if return_softmax_lse else out
    if dropout > 0.0 and training:
        raise NotImplementedError("flashmask_attention: dropout is not supported")
    out, lse = flash_attention_mask(q, k, v, startend_row_indices._t, causal)
    return (_wrap(out), _wrap(lse)) if return_softmax_lse else _wrap(out)


def sdp_kernel(enable_math=False, enable_flash=True, enable_mem_efficient=True):
    import contextlib

    return contextlib.nullcontext()
