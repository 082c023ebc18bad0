"""paddle.incubate.nn.functional fused ops (reference: python/paddle/incubate/nn/functional/).

Each maps onto a hand-written CDNA4 kernel in :mod:`paddle2_amd.ops` where the hot path needs one
(rms_norm, layer_norm, rotary embedding, swiglu, flash attention); the GEMM parts use hipBLASLt.
"""
from __future__ import annotations

import math

import torch

from ....framework.tensor import Tensor
from ....ops import torch_ops as T
from ....distributed.collective import ring_all_reduce

_wrap = Tensor._wrap


def _u(x):
    return None if x is None else x._t


def fused_rms_norm(x, norm_weight, norm_bias, epsilon, begin_norm_axis, bias=None, residual=None, quant_scale=-1,
                   quant_round_type=0, quant_max_bound=0, quant_min_bound=0):
    """Returns (out, residual_out) like ``_C_ops.rms_norm`` in dygraph (fused_rms_norm.py:106)."""
    t = x._t
    if bias is not None:
        t = t + bias._t
    lead = list(t.shape[:begin_norm_axis])
    n = int(torch.tensor(t.shape[begin_norm_axis:]).prod())
    t2 = t.reshape(lead + [n])
    res = None if residual is None else residual._t.reshape(lead + [n])
    w = norm_weight._t.reshape(-1)
    if res is not None:
        y, h = T.rms_norm(t2, w, epsilon, res)
        h = h.reshape(t.shape)
    else:
        y, h = T.rms_norm(t2, w, epsilon), None
    if norm_bias is not None:
        y = y + norm_bias._t.reshape(-1)
    y = y.reshape(t.shape)
    if quant_scale > 0:
        q = torch.clamp(torch.round(y.float() * quant_scale * quant_max_bound), quant_min_bound, quant_max_bound)
        y = q.to(torch.int8)
    return _wrap(y), (None if h is None else _wrap(h))


def fused_layer_norm(x, norm_weight, norm_bias, epsilon, residual_alpha=1.0, begin_norm_axis=1, bias=None,
                     residual=None, quant_scale=-1, quant_round_type=0, quant_max_bound=0, quant_min_bound=0):
    t = x._t
    if bias is not None:
        t = t + bias._t
    if residual is not None:
        t = t + residual_alpha * residual._t
    lead = list(t.shape[:begin_norm_axis])
    n = int(torch.tensor(t.shape[begin_norm_axis:]).prod())
    y = T.layer_norm(t.reshape(lead + [n]), _u(norm_weight), _u(norm_bias), epsilon).reshape(t.shape)
    return _wrap(y), (_wrap(t) if residual is not None else None)


def _rope_one(x, sin, cos, position_ids, use_neox_rotary_style, time_major, rotary_emb_base):
    if x is None:
        return None
    t = x._t
    D = t.shape[-1]
    style = 1 if use_neox_rotary_style else 0
    if sin is None or cos is None:
        S = t.shape[0] if time_major else t.shape[1]
        c, s = T.rope_tables(S, D, rotary_emb_base, interleaved=bool(use_neox_rotary_style), device=t.device)
    else:
        c, s = cos._t.reshape(-1, D), sin._t.reshape(-1, D)
    pos = None if position_ids is None else position_ids._t
    return _wrap(T.rope(t, c, s, pos, style, time_major))


def fused_rotary_position_embedding(q, k=None, v=None, sin=None, cos=None, position_ids=None,
                                    use_neox_rotary_style=True, time_major=False, rotary_emb_base=10000.0):
    """Rotary embedding on q/k/v ([b, s, h, d] or time-major). Returns a 3-tuple like the reference."""
    args = (sin, cos, position_ids, use_neox_rotary_style, time_major, rotary_emb_base)
    return _rope_one(q, *args), _rope_one(k, *args), _rope_one(v, *args)


def swiglu(x, y=None, name=None):
    return _wrap(T.swiglu(x._t, None if y is None else y._t))


def fused_matmul_bias(x, y, bias=None, transpose_x=False, transpose_y=False, name=None):
    a = x._t.transpose(-1, -2) if transpose_x else x._t
    b = y._t.transpose(-1, -2) if transpose_y else y._t
    if bias is not None and a.dim() == 2:
        return _wrap(torch.addmm(bias._t, a, b))
    out = torch.matmul(a, b)
    return _wrap(out if bias is None else out + bias._t)


def fused_linear(x, weight, bias=None, transpose_weight=False, name=None):
    return fused_matmul_bias(x, weight, bias, False, transpose_weight)


def fused_linear_activation(x, y, bias, trans_x=False, trans_y=False, activation=None):
    out = fused_matmul_bias(x, y, bias, trans_x, trans_y)._t
    if activation == "gelu":
        out = torch.nn.functional.gelu(out)
    elif activation == "relu":
        out = torch.relu(out)
    return _wrap(out)


def fused_dropout_add(x, y, p=0.5, training=True, mode="upscale_in_train", name=None):
    t = x._t
    if training and p > 0:
        t = torch.nn.functional.dropout(t, p, True) if mode == "upscale_in_train" else t * torch.bernoulli(
            torch.full_like(t, 1 - p))
    elif mode == "downscale_in_infer" and not training:
        t = t * (1 - p)
    return _wrap(t + y._t)


def fused_bias_act(x, bias=None, dequant_scales=None, shift=None, smooth=None, act_method="gelu",
                   compute_dtype="default", quant_scale=-1, quant_round_type=0, quant_max_bound=0,
                   quant_min_bound=0):
    t = x._t if bias is None else x._t + bias._t
    if act_method == "swiglu":
        return _wrap(T.swiglu(t))  # SwiGLU HIP kernel on the GPU (csrc/kernels/elementwise.hip)
    if act_method == "geglu":
        a, b = t.chunk(2, -1)
        act = torch.nn.functional.gelu(a.float())
        return _wrap((act * b.float()).to(t.dtype))
    fn = {"gelu": torch.nn.functional.gelu, "relu": torch.relu, "silu": torch.nn.functional.silu,
          "swish": torch.nn.functional.silu, "identity": lambda v: v}[act_method]
    return _wrap(fn(t))


def fused_feedforward(x, linear1_weight, linear2_weight, linear1_bias=None, linear2_bias=None, ln1_scale=None,
                      ln1_bias=None, ln2_scale=None, ln2_bias=None, dropout1_rate=0.5, dropout2_rate=0.5,
                      activation="relu", ln1_epsilon=1e-5, ln2_epsilon=1e-5, pre_layer_norm=False, training=True,
                      mode="upscale_in_train", ring_id=-1, add_residual=True, name=None):
    """Transformer FFN block (reference fused_feedforward_kernel.cu): [LN] -> x W1 -> bias+act (fused kernel) ->
    dropout -> W2 -> bias -> dropout + residual (fused kernel) -> [LN]; GEMMs through the Linear GEMM path."""
    from ....ops import fused as FU

    t = x._t
    res = t
    if pre_layer_norm:
        t = T.layer_norm(t, _u(ln1_scale), _u(ln1_bias), ln1_epsilon)
    h = T.linear(t, linear1_weight._t)
    h = FU.bias_act(h, _u(linear1_bias), activation)
    if training and dropout1_rate:
        h = torch.nn.functional.dropout(h, dropout1_rate)
    if ring_id is not None and int(ring_id) >= 0:
        o = T.linear(h, linear2_weight._t)
        ring_all_reduce(o, ring_id)   # tensor parallel: linear1 column / linear2 row shards -> partial sums
        if linear2_bias is not None:
            o = o + linear2_bias._t
    else:
        o = T.linear(h, linear2_weight._t, _u(linear2_bias))
    if training and dropout2_rate and mode == "upscale_in_train" and add_residual:
        o = FU.dropout_add(o, res, dropout2_rate)
    else:
        if training and dropout2_rate:
            o = torch.nn.functional.dropout(o, dropout2_rate)
        if add_residual:
            o = o + res
    if not pre_layer_norm:
        o = T.layer_norm(o, _u(ln2_scale), _u(ln2_bias), ln2_epsilon)
    return _wrap(o)


def fused_multi_head_attention(x, qkv_weight, linear_weight, pre_layer_norm=False, pre_ln_scale=None,
                               pre_ln_bias=None, ln_scale=None, ln_bias=None, pre_ln_epsilon=1e-05, qkv_bias=None,
                               linear_bias=None, cache_kv=None, attn_mask=None, dropout_rate=0.5,
                               attn_dropout_rate=0.5, ln_epsilon=1e-05, training=True, mode="upscale_in_train",
                               ring_id=-1, add_residual=True, num_heads=-1, transpose_qkv_wb=False, name=None):
    t = x._t
    b, s, e = t.shape
    res = t
    if pre_layer_norm:
        t = T.layer_norm(t, _u(pre_ln_scale), _u(pre_ln_bias), pre_ln_epsilon)
    w = qkv_weight._t  # [3, nh, hd, e]
    nh, hd = w.shape[1], w.shape[2]
    qkv = torch.einsum("bse,tnde->bstnd", t, w)
    if qkv_bias is not None:
        qkv = qkv + qkv_bias._t
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    if attn_mask is None and q.dtype == torch.bfloat16:
        o, _ = T.flash_attention(q.contiguous(), k.contiguous(), v.contiguous(), False)
    else:
        sc = torch.einsum("bqnd,bknd->bnqk", q.float(), k.float()) / math.sqrt(hd)
        if attn_mask is not None:
            sc = sc + attn_mask._t.float()
        o = torch.einsum("bnqk,bknd->bqnd", torch.softmax(sc, -1), v.float()).to(t.dtype)
    o = torch.matmul(o.reshape(b, s, nh * hd), linear_weight._t)
    ring_all_reduce(o, ring_id)   # tensor parallel: this rank's heads only -> out-projection partial sum
    if linear_bias is not None:
        o = o + linear_bias._t
    if add_residual:
        o = o + res
    if not pre_layer_norm:
        o = T.layer_norm(o, _u(ln_scale), _u(ln_bias), ln_epsilon)
    return _wrap(o)


def variable_length_memory_efficient_attention(query, key, value, seq_lens, kv_seq_lens, mask=None, scale=None,
                                               causal=False, pre_cache_length=0):
    """[b, h, s, d] padded layout with per-sequence query / key lengths (reference: CUTLASS
    variable_length_memory_efficient_attention; causal = bottom-right aligned on the actual lengths).

    MI355X path: ONE FlashMask launch for the whole batch — key columns past ``kv_seq_lens[b]`` are masked for
    every row and the causal band is expressed per key column as the row interval [0, j - (kv_len - q_len)),
    so there is no per-sequence loop and no host read of the lengths; rows past ``seq_lens[b]`` are zeroed.
    An additive ``mask`` [b, 1 or h, s_q, s_k] takes the batched fp32 path."""
    q, k, v = query._t, key._t, value._t
    b, h, sq, d = q.shape
    sk = k.shape[2]
    scale = scale or 1.0 / math.sqrt(d)
    sl = seq_lens._t.reshape(-1).to(q.device).long()
    kl = kv_seq_lens._t.reshape(-1).to(q.device).long()
    j = torch.arange(sk, device=q.device)[None, :]
    key_ok = j < kl[:, None]                                           # [b, sk]
    row_ok = torch.arange(sq, device=q.device)[None, :] < sl[:, None]  # [b, sq]
    if mask is None:
        lts = torch.where(key_ok, torch.full_like(j, 1 << 30), torch.zeros_like(j))
        ute = (j - (kl - sl)[:, None]).clamp_min(0) if causal else torch.zeros_like(lts)
        idx = torch.stack([lts, ute], -1)[:, None].to(torch.int32)       # [b, 1, sk, 2] (LTS, UTE)
        o, _ = T.flash_attention_mask(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), idx, False, scale)
        o = o.transpose(1, 2)
    else:
        sc = torch.einsum("bhqd,bhkd->bhqk", q.float(), k.float()) * scale + mask._t.float()
        bad = ~key_ok[:, None, None, :]
        if causal:
            i = torch.arange(sq, device=q.device)[None, :, None]
            bad = bad | (j[:, None, :] > i + (kl - sl)[:, None, None])[:, None]
        sc = sc.masked_fill(bad, float("-inf"))
        o = torch.nan_to_num(torch.softmax(sc, -1), nan=0.0)
        o = torch.einsum("bhqk,bhkd->bhqd", o, v.float()).to(q.dtype)
    return _wrap(o * row_ok[:, None, :, None].to(o.dtype))


def masked_multihead_attention(*args, **kwargs):
    """Single-token decode attention over a [2, b, nh, max_s, hd] KV cache (reference
    masked_multihead_attention_kernel.cu): writes k/v at ``sequence_lengths`` and runs the flash-decoding HIP
    kernel (serving.masked_multihead_attention). Returns (out [b, nh*hd], cache_kv)."""
    from ....serving import masked_multihead_attention as _mmha

    return _mmha(*args, **kwargs)


def block_multihead_attention(*args, **kwargs):
    from ....serving import block_multihead_attention as _bma

    return _bma(*args, **kwargs)


def fused_multi_transformer(*args, **kwargs):
    from ....serving import fused_multi_transformer as _fmt

    return _fmt(*args, **kwargs)


def fused_moe(x, gate_weight, ffn1_weight, ffn2_weight, ffn1_bias=None, ffn1_scale=None, ffn2_bias=None,
              ffn2_scale=None, quant_method="None", moe_topk=2, norm_topk_prob=True):
    """Top-k gated MoE FFN with the reference public signature
    (python/paddle/incubate/nn/functional/fused_moe.py:20; kernel fusion/cutlass/fused_moe_kernel.cu).

    ``gate_weight`` [H, E] (the router Linear's weight); ``ffn1_weight`` [E, H, 2F] packs [gate | up];
    ``ffn2_weight`` [E, F, H].  ``quant_method`` "weight_only_int8" / "weight_only_int4": the expert
    weights are ``nn.quant.weight_quantize`` outputs (int8 [N, K] / packed int4 [N/2, K] per expert, viewed
    with the float weight's shape as in the reference test) with per-channel ``ffn*_scale`` [E, N]; each
    expert's weights are dequantized once per call.

    MI355X path (ops/moe.py): routing, the expert sort and the per-expert offsets stay on the device; each
    projection is ONE grouped launch of the native MFMA GEMM (the first with the SwiGLU epilogue when there is
    no ffn1 bias) and the weighted outputs are scatter-added back — no host read of the expert counts."""
    from ....ops import moe as MOE

    if quant_method not in ("None", "weight_only_int8", "weight_only_int4"):
        raise NotImplementedError(f"fused_moe: quant_method {quant_method!r}")
    quant = quant_method != "None"
    if quant and (ffn1_scale is None or ffn2_scale is None):
        raise ValueError(f"fused_moe: quant_method {quant_method!r} needs ffn1_scale and ffn2_scale")
    t = x._t
    shp = t.shape
    t2 = t.reshape(-1, shp[-1])
    w1, w2 = ffn1_weight._t, ffn2_weight._t
    E = w1.shape[0]
    Hd = t2.shape[1]
    if quant:
        from ....nn.quant import _dequant

        wd = "int4" if quant_method == "weight_only_int4" else "int8"

        def deq(wt, scale, K):
            N_ = scale._t.shape[-1]
            rows = N_ // 2 if wd == "int4" else N_
            return torch.stack([_dequant(wt[e].reshape(rows, K), scale._t[e], wd, -1, t.dtype).t()
                                for e in range(E)]).contiguous()  # [E, K, N], one dequant per call

        w1 = deq(w1, ffn1_scale, Hd)
        w2 = deq(w2, ffn2_scale, w1.shape[2] // 2)
    b1 = None if ffn1_bias is None else ffn1_bias._t.reshape(E, -1)
    b2 = None if ffn2_bias is None else ffn2_bias._t.reshape(E, -1)
    out = MOE.moe_ffn(t2, gate_weight._t, w1.to(t.dtype).contiguous(), w2.to(t.dtype).contiguous(), moe_topk,
                      norm_topk_prob, b1, b2)
    N2 = out.shape[-1]
    return _wrap(out.reshape(*shp[:-1], N2))
