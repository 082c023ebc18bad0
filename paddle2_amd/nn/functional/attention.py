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
    """Varlen attention over packed [total_tokens, heads, d] with cumulative sequence offsets."""
    from ...ops.torch_ops import flash_attention as _fa

    q, k, v = query._t, key._t, value._t
    cq = cu_seqlens_q._t.tolist()
    ck = cu_seqlens_k._t.tolist()
    outs = []
    for i in range(len(cq) - 1):
        qs = q[cq[i]:cq[i + 1]].unsqueeze(0)
        ks = k[ck[i]:ck[i + 1]].unsqueeze(0)
        vs = v[ck[i]:ck[i + 1]].unsqueeze(0)
        o, _ = _fa(qs, ks, vs, causal, scale)
        outs.append(o.squeeze(0))
    return _wrap(torch.cat(outs, 0)), None


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
    """FlashMask: per-column row-range masks ([b, h, s_k, {1,2,4}] start/end row indices).

    Builds the dense mask from the compact row ranges (reference flash_attn_kernel.cu:445-494);
    the sparse-skipping MFMA kernel is future work.
    """
    q, k, v = query._t, key._t, value._t
    b, sq, hq, d = q.shape
    sk = k.shape[1]
    if startend_row_indices is None:
        out, _ = flash_attention(query, key, value, dropout, causal, training=training)
        return out
    idx = startend_row_indices._t.long()  # [b, h', sk, n]
    rows = torch.arange(sq, device=q.device)[:, None]  # [sq, 1]
    n = idx.shape[-1]
    if n == 1:
        start = idx[..., 0][:, :, None, :]
        masked = rows[None, None] >= start
    elif n == 2:
        if causal:
            s0, s1 = idx[..., 0][:, :, None, :], idx[..., 1][:, :, None, :]
            masked = (rows[None, None] >= s0) & (rows[None, None] < s1)
        else:
            s0, e0 = idx[..., 0][:, :, None, :], idx[..., 1][:, :, None, :]
            masked = (rows[None, None] >= s0) | (rows[None, None] < e0)
    else:
        a, bb, c, dd = [idx[..., i][:, :, None, :] for i in range(4)]
        r = rows[None, None]
        masked = ((r >= a) & (r < bb)) | ((r >= c) & (r < dd))
    if causal:
        masked = masked | (torch.arange(sk, device=q.device)[None, :] > rows)[None, None]
    bias = torch.zeros(masked.shape, dtype=torch.float32, device=q.device).masked_fill(masked, float("-inf"))
    qt, kt, vt = q.transpose(1, 2), _rep(k, hq).transpose(1, 2), _rep(v, hq).transpose(1, 2)
    s = torch.matmul(qt.float(), kt.float().transpose(-1, -2)) / math.sqrt(d) + bias
    p = torch.softmax(s, -1).nan_to_num(0.0)
    o = torch.matmul(p, vt.float()).to(q.dtype).transpose(1, 2)
    return _wrap(o)


def sdp_kernel(enable_math=False, enable_flash=True, enable_mem_efficient=True):
    import contextlib

    return contextlib.nullcontext()
