"""Inference / serving runtime: KV caches, decode attention, fused multi-transformer, generation.

Reference: incubate/nn/functional/masked_multihead_attention.py (MMHA, cache [2, b, nh, max_s, hd]),
block_multihead_attention.py (paged cache [blocks, nh, block_size, hd] + block tables),
fused_transformer.py:1053/:1263 ``fused_multi_transformer`` (+ the ``FusedMultiTransformer``
layer), and the PaddleNLP-style generation loop on top.

MI355X design:
  * prefill = the MFMA flash-attention forward kernel (causal, GQA, per-sequence strided views);
  * decode = csrc/kernels/decode_attn.hip (flash-decoding: one workgroup per (seq, kv head,
    split), GQA heads served from one K/V read, fp32 split merge), same kernel for the
    contiguous MMHA cache and the paged block cache via stride/block-table addressing;
  * new K/V rows land in the cache with one gather-free write kernel (block-table addressed);
  * the per-token decode step of a fixed batch is a static-shape graph: ``LlamaGenerator`` can
    capture it once in a HIP graph and replay it (launch-bound loops -> one graph launch).
"""
from __future__ import annotations

import math
import os

import torch

from ..framework.tensor import Tensor
from ..ops import _native as N
from ..ops import torch_ops as T
from ..distributed.collective import ring_all_reduce

_wrap = Tensor._wrap


def _u(x):
    return x._t if isinstance(x, Tensor) else x


# ============================================================================ core attention ops
# 0 auto (MFMA kernel for D = 128 and 2..16 q heads per kv head, vector kernel for MHA), 1 vector kernel,
# 2 MFMA kernel (raises if unusable)
_DECODE_IMPL = {"auto": 0, "vec": 1, "mfma": 2}[os.environ.get("PADDLE2_AMD_DECODE_KERNEL", "auto")]
# KV-split sizing: at least WG_TARGET workgroups over the cache's capacity, at least SPLIT_TOKENS keys per split
_DECODE_WG_TARGET = int(os.environ.get("PADDLE2_AMD_DECODE_WG_TARGET", "2048"))
_DECODE_SPLIT_TOKENS = int(os.environ.get("PADDLE2_AMD_DECODE_SPLIT_TOKENS", "64"))


def decode_attention(q, k_cache, v_cache, seq_lens, block_table=None, block_size=None, layout="paged",
                     scale=None, splits=None, out=None):
    """One query token per sequence.

    q: [B, Hq, D] (any strides with unit inner stride); seq_lens: [B] int32 (#valid keys incl. the
    new token).  layout "paged": caches [num_blocks, block_size, Hk, D] + block_table [B, max_blocks];
    layout "bhsd": caches [B, Hk, max_s, D] (MMHA); layout "paddle_block": [num_blocks, Hk, block_size, D].
    Returns out [B, Hq, D]."""
    B, Hq, D = q.shape
    if layout == "paged":
        _, bs, Hk, _ = k_cache.shape
        s_blk, s_tok, s_head = k_cache.stride(0), k_cache.stride(1), k_cache.stride(2)
    elif layout == "paddle_block":
        _, Hk, bs, _ = k_cache.shape
        s_blk, s_tok, s_head = k_cache.stride(0), k_cache.stride(2), k_cache.stride(1)
    else:  # bhsd
        _, Hk, bs, _ = k_cache.shape
        s_blk, s_tok, s_head = k_cache.stride(0), k_cache.stride(2), k_cache.stride(1)
        block_table = None
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if out is None:
        out = torch.empty(B, Hq, D, dtype=q.dtype, device=q.device)
    G = Hq // Hk
    native = (q.device.type == "cuda" and N.use_native(q) and q.dtype == torch.bfloat16 and D in (64, 128)
              and (G in (1, 2, 4, 8) or (D == 128 and G == 16 and _DECODE_IMPL != 1)))
    if native:
        max_len = int(k_cache.shape[0] * bs) if block_table is not None else int(bs)
        if splits is None:
            # enough workgroups to fill the chip: B * Hk * splits >= ~2 per CU
            splits = max(1, min(64, (_DECODE_WG_TARGET + B * Hk - 1) // (B * Hk)))
            if block_table is not None:
                splits = max(1, min(splits, (block_table.shape[1] * bs) // _DECODE_SPLIT_TOKENS or 1))
        lens = seq_lens.to(torch.int32).contiguous()
        max_len = int(block_table.shape[1] * bs) if block_table is not None else int(bs)
        part_o = torch.empty(B * Hq * splits * D, dtype=torch.float32, device=q.device) if splits > 1 else None
        part_ml = torch.empty(B * Hq * splits * 2, dtype=torch.float32, device=q.device) if splits > 1 else None
        bt = block_table.to(torch.int32).contiguous() if block_table is not None else None
        N.native().decode_attn(q.data_ptr(), q.stride(0), q.stride(1), k_cache.data_ptr(), v_cache.data_ptr(),
                               s_blk, s_tok, s_head, N.ptr(bt), 0 if bt is None else bt.shape[1], bs,
                               lens.data_ptr(), max_len, N.ptr(part_o), N.ptr(part_ml), out.data_ptr(),
                               out.stride(0), out.stride(1), B, Hq, Hk, D, splits, float(scale), _DECODE_IMPL,
                               N.stream())
        return out
    # reference path (CPU / other dtypes)
    G = Hq // Hk
    for b in range(B):
        L = int(seq_lens[b])
        if layout == "bhsd":
            ks = k_cache[b, :, :L].float()
            vs = v_cache[b, :, :L].float()
        else:
            idx = torch.arange(L, device=q.device)
            blocks = block_table[b, idx // bs].long()
            if layout == "paged":
                ks = k_cache[blocks, idx % bs].permute(1, 0, 2).float()
                vs = v_cache[blocks, idx % bs].permute(1, 0, 2).float()
            else:
                ks = k_cache[blocks, :, idx % bs].permute(1, 0, 2).float()
                vs = v_cache[blocks, :, idx % bs].permute(1, 0, 2).float()
        qq = q[b].float().reshape(Hk, G, D)
        sc = torch.einsum("hgd,hsd->hgs", qq, ks) * scale
        p = torch.softmax(sc, -1)
        out[b] = torch.einsum("hgs,hsd->hgd", p, vs).reshape(Hq, D).to(out.dtype)
    return out


def write_kv(k, v, k_cache, v_cache, tok_batch, tok_pos, block_table=None, layout="paged"):
    """Store rows k/v [n_tok, Hk, D] at (sequence tok_batch[i], position tok_pos[i]) of the cache."""
    n, Hk, D = k.shape
    if layout == "paged":
        bs = k_cache.shape[1]
        s_blk, s_tok, s_head = k_cache.stride(0), k_cache.stride(1), k_cache.stride(2)
    else:  # bhsd or paddle_block: [X, Hk, S, D]
        bs = k_cache.shape[2]
        s_blk, s_tok, s_head = k_cache.stride(0), k_cache.stride(2), k_cache.stride(1)
        if layout == "bhsd":
            block_table = None
    if (k.device.type == "cuda" and N.use_native(k) and k.dtype == torch.bfloat16 and D % 8 == 0
            and k.stride(2) == 1 and k.stride(1) == D and v.stride(1) == D):
        tb = tok_batch.to(torch.int32).contiguous()
        tp = tok_pos.to(torch.int32).contiguous()
        bt = block_table.to(torch.int32).contiguous() if block_table is not None else None
        N.native().cache_write(k.data_ptr(), v.data_ptr(), k.stride(0), v.stride(0), k_cache.data_ptr(),
                               v_cache.data_ptr(), s_blk, s_tok, s_head, N.ptr(bt), 0 if bt is None else bt.shape[1],
                               bs, tb.data_ptr(), tp.data_ptr(), n, Hk, D, N.stream())
        return
    tb, tp = tok_batch.long(), tok_pos.long()
    if block_table is not None:
        blk = block_table.long()[tb, tp // bs]
        off = tp % bs
    else:
        blk, off = tb, tp
    if layout == "paged":
        k_cache[blk, off] = k.to(k_cache.dtype)
        v_cache[blk, off] = v.to(v_cache.dtype)
    else:
        k_cache[blk, :, off] = k.to(k_cache.dtype)
        v_cache[blk, :, off] = v.to(v_cache.dtype)


# ============================================================================ paged KV cache
class PagedKVCache:
    """Per-layer K/V block pools [num_blocks, block_size, Hk, D] with a free list and block tables."""

    def __init__(self, num_layers, num_blocks, block_size, num_kv_heads, head_dim, max_batch, max_seq_len,
                 dtype=torch.bfloat16, device=None):
        dev = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                         else torch.device("cpu"))
        self.block_size = block_size
        self.k = [torch.zeros(num_blocks, block_size, num_kv_heads, head_dim, dtype=dtype, device=dev)
                  for _ in range(num_layers)]
        self.v = [torch.zeros_like(t) for t in self.k]
        self.max_blocks_per_seq = (max_seq_len + block_size - 1) // block_size
        self.block_table = torch.zeros(max_batch, self.max_blocks_per_seq, dtype=torch.int32, device=dev)
        self.seq_lens = torch.zeros(max_batch, dtype=torch.int32, device=dev)
        self._free = list(range(num_blocks - 1, -1, -1))
        self._owned = {}

    def allocate(self, slot, num_tokens):
        """Make sure sequence ``slot`` has blocks for ``num_tokens`` tokens."""
        have = self._owned.setdefault(slot, [])
        need = (num_tokens + self.block_size - 1) // self.block_size
        while len(have) < need:
            if not self._free:
                raise RuntimeError("PagedKVCache out of blocks")
            b = self._free.pop()
            self.block_table[slot, len(have)] = b
            have.append(b)

    def free(self, slot):
        for b in self._owned.pop(slot, []):
            self._free.append(b)
        self.seq_lens[slot] = 0

    @property
    def num_free_blocks(self):
        return len(self._free)


# ============================================================================ Paddle APIs
@torch.no_grad()
def masked_multihead_attention(x, cache_kv=None, bias=None, src_mask=None, cum_offsets=None, sequence_lengths=None,
                               rotary_tensor=None, beam_cache_offset=None, qkv_out_scale=None, out_shift=None,
                               out_smooth=None, seq_len=1, rotary_emb_dims=0, use_neox_rotary_style=False,
                               compute_dtype="default", out_scale=-1, quant_round_type=1, quant_max_bound=127.0,
                               quant_min_bound=-127.0):
    """Decode step over the contiguous [2, b, nh, max_s, hd] cache: writes the new k/v at position
    ``sequence_lengths[b]`` and attends over positions [0, sequence_lengths[b]]."""
    t = _u(x)
    if bias is not None:
        t = t + _u(bias).reshape(1, -1)
    ck = _u(cache_kv)
    _, b, nh, max_s, hd = ck.shape
    qkv = t.reshape(b, 3, nh, hd)
    lens = (_u(sequence_lengths).reshape(-1).to(torch.int32) if sequence_lengths is not None
            else torch.zeros(b, dtype=torch.int32, device=t.device))
    write_kv(qkv[:, 1].contiguous(), qkv[:, 2].contiguous(), ck[0], ck[1], torch.arange(b, device=t.device), lens,
             layout="bhsd")
    q = qkv[:, 0]
    if src_mask is not None or t.dtype != torch.bfloat16 or t.device.type != "cuda":
        keys, vals = ck[0].float(), ck[1].float()
        sc = torch.einsum("bnd,bnsd->bns", q.float(), keys) / math.sqrt(hd)
        valid = torch.arange(max_s, device=t.device)[None, :] <= lens[:, None]
        sc = sc.masked_fill(~valid[:, None, :], float("-inf"))
        if src_mask is not None:
            sc = sc + _u(src_mask).reshape(b, 1, -1)[..., :max_s].float()
        p = torch.softmax(sc, -1)
        o = torch.einsum("bns,bnsd->bnd", p, vals).to(t.dtype)
    else:
        o = decode_attention(q, ck[0], ck[1], lens + 1, layout="bhsd")
    return _wrap(o.reshape(b, nh * hd)), cache_kv


@torch.no_grad()
def block_multihead_attention(qkv, key_cache, value_cache, seq_lens_encoder, seq_lens_decoder, seq_lens_this_time,
                              padding_offsets, cum_offsets, cu_seqlens_q, cu_seqlens_k, block_tables,
                              pre_key_cache=None, pre_value_cache=None, cache_k_quant_scales=None,
                              cache_v_quant_scales=None, cache_k_dequant_scales=None, cache_v_dequant_scales=None,
                              qkv_out_scale=None, qkv_bias=None, out_shift=None, out_smooth=None,
                              max_enc_len_this_time=None, max_dec_len_this_time=None, rope_emb=None, mask=None,
                              tgt_mask=None, max_seq_len=-1, block_size=64, use_neox_style=False,
                              use_dynamic_cachekv_quant=False, quant_round_type=1, quant_max_bound=127.0,
                              quant_min_bound=-127.0, out_scale=-1, compute_dtype="default", rope_theta=10000.0):
    """Ragged batch over a paged cache [blocks, nh, block_size, hd]: sequences with
    seq_lens_encoder > 0 run causal prefill (flash kernel) and fill the cache; the others append
    one token and run decode attention.  Returns (out [token_num, nh*hd], qkv, key_cache, value_cache)."""
    t = _u(qkv)
    if qkv_bias is not None:
        t = t + _u(qkv_bias).reshape(1, -1)
    kc, vc = _u(key_cache), _u(value_cache)
    _, Hk, bs, D = kc.shape
    tok = t.shape[0]
    Hq = t.shape[1] // D - 2 * Hk
    enc = _u(seq_lens_encoder).reshape(-1).tolist()
    dec = _u(seq_lens_decoder).reshape(-1).tolist()
    now = _u(seq_lens_this_time).reshape(-1).tolist()
    cu = _u(cu_seqlens_q).reshape(-1).tolist()
    bt = _u(block_tables)
    qkv3 = t.reshape(tok, Hq + 2 * Hk, D)
    out = torch.empty(tok, Hq, D, dtype=t.dtype, device=t.device)
    cos = sin = None
    if rope_emb is not None:
        re = _u(rope_emb)  # [2, b, max_s, 1, D/2]
    dec_rows, dec_b = [], []
    for b in range(len(now)):
        if now[b] == 0:
            continue
        s0 = cu[b]
        n = now[b]
        start = dec[b] if enc[b] == 0 else 0
        pos = torch.arange(start, start + n, device=t.device)
        q = qkv3[s0:s0 + n, :Hq]
        k = qkv3[s0:s0 + n, Hq:Hq + Hk]
        v = qkv3[s0:s0 + n, Hq + Hk:]
        if rope_emb is not None:
            c = re[0, b, pos, 0].float()
            sn = re[1, b, pos, 0].float()
            cos = torch.cat([c, c], -1) if not use_neox_style else torch.repeat_interleave(c, 2, -1)
            sin = torch.cat([sn, sn], -1) if not use_neox_style else torch.repeat_interleave(sn, 2, -1)
            st = 1 if use_neox_style else 0
            q = T.rope(q[None], cos, sin, None, style=st)[0]
            k = T.rope(k[None], cos, sin, None, style=st)[0]
        write_kv(k.contiguous(), v.contiguous(), kc, vc, torch.full((n,), b, device=t.device), pos, bt,
                 layout="paddle_block")
        if enc[b] > 0:
            o, _ = T.flash_attention(q[None], k[None], v[None], causal=True)
            out[s0:s0 + n] = o[0]
        else:
            dec_rows.append(s0)
            dec_b.append((b, q))
    if dec_rows:
        idx = torch.tensor([b for b, _ in dec_b], device=t.device)
        qd = torch.stack([q[0] for _, q in dec_b])
        lens = torch.tensor([dec[b] + 1 for b, _ in dec_b], dtype=torch.int32, device=t.device)
        od = decode_attention(qd, kc, vc, lens, bt[idx], layout="paddle_block")
        for i, r in enumerate(dec_rows):
            out[r] = od[i]
    return _wrap(out.reshape(tok, Hq * D)), qkv, key_cache, value_cache


def _static_mm(x, w):
    """x @ W for a static inference weight W [K, N]: on the GPU through a contiguous W^T, the layout hipBLASLt
    streams fastest at decode shapes (profiles/r3_decode_gemm_layouts.jsonl).  The transposed copy is attached to
    W itself (attribute ``_pd_wt``), so it lives exactly as long as W does — nothing global holds W — and it is
    re-transposed in place when W's version changes (``clear_static_weight_cache`` drops it)."""
    if not w.is_cuda or w.dim() != 2:
        return torch.matmul(x, w)
    ent = getattr(w, "_pd_wt", None)
    if ent is None or ent[1].shape != (w.shape[1], w.shape[0]):
        ent = [w._version, T.transpose2d(w)]
        w._pd_wt = ent
    elif ent[0] != w._version:
        ent[1].copy_(w.t())
        ent[0] = w._version
    return torch.matmul(x, ent[1].t())


def clear_static_weight_cache(*weights):
    """Drop the transposed copies that ``_static_mm`` attached to ``weights`` (paddle or torch tensors)."""
    for w in weights:
        t = getattr(w, "_t", w)
        if hasattr(t, "_pd_wt"):
            del t._pd_wt


@torch.no_grad()
def fused_multi_transformer(x, ln_scales, ln_biases, qkv_weights, qkv_biases, linear_weights, linear_biases,
                            ffn_ln_scales, ffn_ln_biases, ffn1_weights, ffn1_biases, ffn2_weights, ffn2_biases,
                            pre_layer_norm=True, epsilon=1e-5, residual_alpha=1.0, cache_kvs=None, beam_offset=None,
                            pre_caches=None, seq_lens=None, rotary_embs=None, time_step=None, attn_mask=None,
                            dropout_rate=0.0, rotary_emb_dims=0, activation="gelu", training=False,
                            mode="upscale_in_train", trans_qkvw=True, ring_id=-1, norm_type="layernorm",
                            use_neox_rotary_style=False, gqa_group_size=-1, name=None):
    """Stack of pre-LN decoder layers for inference (reference fused_transformer.py:1053).

    Tensor parallel (``ring_id`` >= 0): every rank holds its head slice of qkv / out-projection and its column
    slice of ffn1 / row slice of ffn2; the two partial sums per layer are all-reduced over communicator
    ``ring_id`` (reference fused_multi_transformer_kernel.cu:474) before the replicated bias — decode-sized
    messages take the xGMI one-shot path when that is enabled (distributed/ipc_allreduce.py).

    x [b, s, d]; qkv_weights[i]: [3, nh, hd, d] (trans_qkvw) or [d, 3*nh*hd]; cache_kvs[i]:
    [2, b, nh, max_s, hd].  time_step None -> context phase (causal flash attention over the
    prompt, cache filled at [0, s)); else decode phase at position ``time_step`` (s == 1)."""
    h = _u(x)
    b, s, d = h.shape
    L = len(qkv_weights)
    rms = norm_type == "rmsnorm"
    outs_cache = cache_kvs
    step = None if time_step is None else int(_u(time_step).reshape(-1)[0]) if isinstance(
        time_step, (Tensor, torch.Tensor)) else int(time_step)
    for i in range(L):
        w_ln = _u(ln_scales[i])
        b_ln = None if ln_biases is None or ln_biases[i] is None else _u(ln_biases[i])
        resid = h
        x1 = T.rms_norm(h, w_ln, epsilon) if rms else T.layer_norm(h, w_ln, b_ln, epsilon)
        wq = _u(qkv_weights[i])
        if trans_qkvw:
            three_nh, hd = wq.shape[0] * wq.shape[1], wq.shape[2]
            qkv = torch.matmul(x1, wq.reshape(-1, d).t())
            nh = wq.shape[1]
        else:
            qkv = _static_mm(x1, wq)
            hd = _u(cache_kvs[i]).shape[-1] if cache_kvs is not None else d // (qkv.shape[-1] // (3 * (d // 64)))
            nh = qkv.shape[-1] // (3 * hd)
        if qkv_biases is not None and qkv_biases[i] is not None:
            qkv = qkv + _u(qkv_biases[i]).reshape(-1)
        qkv = qkv.reshape(b, s, 3, nh, hd)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        if rotary_embs is not None and rotary_emb_dims > 0:
            re = _u(rotary_embs)  # [2, b, 1, max_s, hd]
            pos0 = 0 if step is None else step
            cos = re[0, 0, 0, pos0:pos0 + s].float()
            sin = re[1, 0, 0, pos0:pos0 + s].float()
            st = 1 if use_neox_rotary_style else 0
            q = T.rope(q.contiguous(), cos, sin, None, style=st)
            k = T.rope(k.contiguous(), cos, sin, None, style=st)
        ck = _u(cache_kvs[i]) if cache_kvs is not None else None
        if step is None:
            if ck is not None:
                for bb in range(b):
                    write_kv(k[bb].contiguous(), v[bb].contiguous(), ck[0], ck[1],
                             torch.full((s,), bb, device=h.device), torch.arange(s, device=h.device), layout="bhsd")
            if attn_mask is not None:
                sc = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) / math.sqrt(hd) + _u(attn_mask).float()
                o = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(sc, -1), v.float()).to(h.dtype)
            else:
                o, _ = T.flash_attention(q, k, v, causal=True)
        else:
            write_kv(k[:, 0].contiguous(), v[:, 0].contiguous(), ck[0], ck[1], torch.arange(b, device=h.device),
                     torch.full((b,), step, dtype=torch.int32, device=h.device), layout="bhsd")
            lens = torch.full((b,), step + 1, dtype=torch.int32, device=h.device)
            o = decode_attention(q[:, 0], ck[0], ck[1], lens, layout="bhsd")[:, None]
        o = o.reshape(b, s, nh * hd)
        a = _static_mm(o, _u(linear_weights[i]))
        ring_all_reduce(a, ring_id)   # tensor parallel: heads are sharded, the out-projection partial sums add
        if linear_biases is not None and linear_biases[i] is not None:
            a = a + _u(linear_biases[i])
        w2 = _u(ffn_ln_scales[i])
        b2 = None if ffn_ln_biases is None or ffn_ln_biases[i] is None else _u(ffn_ln_biases[i])
        if rms:
            x2, h = T.rms_norm(a, w2, epsilon, resid)
        else:
            x2, h = T.layer_norm(a, w2, b2, epsilon, resid)
        f = _static_mm(x2, _u(ffn1_weights[i]))
        if ffn1_biases is not None and ffn1_biases[i] is not None:
            f = f + _u(ffn1_biases[i])
        if activation in ("swiglu",):
            f = T.swiglu(f)
        elif activation == "relu":
            f = torch.relu(f)
        else:
            f = torch.nn.functional.gelu(f, approximate="tanh" if activation == "gelu_tanh" else "none")
        f = _static_mm(f, _u(ffn2_weights[i]))
        ring_all_reduce(f, ring_id)   # FFN hidden sharded: partial sums add before the (replicated) bias
        if ffn2_biases is not None and ffn2_biases[i] is not None:
            f = f + _u(ffn2_biases[i])
        h = h + f
    if cache_kvs is not None:
        return _wrap(h), outs_cache
    return _wrap(h)


class FusedMultiTransformerImpl:
    """Parameter holder behind incubate.nn.FusedMultiTransformer."""

    def __init__(self, layer, embed_dim, num_heads, dim_feedforward, activation, num_layers, epsilon, norm_type,
                 gqa_group_size):
        from ..nn import initializer as I

        hd = embed_dim // num_heads
        self.layer, self.activation, self.eps, self.norm_type = layer, activation, epsilon, norm_type
        self.num_layers = num_layers
        P = layer.create_parameter
        mk = lambda shape, init=None, bias=False: P(shape, is_bias=bias,  # noqa: E731
                                                   default_initializer=init or I.XavierUniform())
        layer.ln_scales = [mk([embed_dim], I.Constant(1.0)) for _ in range(num_layers)]
        layer.ln_biases = [mk([embed_dim], I.Constant(0.0), True) for _ in range(num_layers)]
        layer.qkv_weights = [mk([3, num_heads, hd, embed_dim]) for _ in range(num_layers)]
        layer.qkv_biases = [mk([3 * num_heads * hd], I.Constant(0.0), True) for _ in range(num_layers)]
        layer.linear_weights = [mk([num_heads * hd, embed_dim]) for _ in range(num_layers)]
        layer.linear_biases = [mk([embed_dim], I.Constant(0.0), True) for _ in range(num_layers)]
        layer.ffn_ln_scales = [mk([embed_dim], I.Constant(1.0)) for _ in range(num_layers)]
        layer.ffn_ln_biases = [mk([embed_dim], I.Constant(0.0), True) for _ in range(num_layers)]
        f_in = dim_feedforward * (2 if activation == "swiglu" else 1)
        layer.ffn1_weights = [mk([embed_dim, f_in]) for _ in range(num_layers)]
        layer.ffn1_biases = [mk([f_in], I.Constant(0.0), True) for _ in range(num_layers)]
        layer.ffn2_weights = [mk([dim_feedforward, embed_dim]) for _ in range(num_layers)]
        layer.ffn2_biases = [mk([embed_dim], I.Constant(0.0), True) for _ in range(num_layers)]
        for name in ("ln_scales", "ln_biases", "qkv_weights", "qkv_biases", "linear_weights", "linear_biases",
                     "ffn_ln_scales", "ffn_ln_biases", "ffn1_weights", "ffn1_biases", "ffn2_weights", "ffn2_biases"):
            for j, p in enumerate(getattr(layer, name)):
                layer.add_parameter(f"{name}_{j}", p)

    def forward(self, src, attn_mask=None, caches=None, seq_lens=None, time_step=None):
        L = self.layer
        return fused_multi_transformer(src, L.ln_scales, L.ln_biases, L.qkv_weights, L.qkv_biases, L.linear_weights,
                                       L.linear_biases, L.ffn_ln_scales, L.ffn_ln_biases, L.ffn1_weights,
                                       L.ffn1_biases, L.ffn2_weights, L.ffn2_biases, epsilon=self.eps,
                                       cache_kvs=caches, time_step=time_step, attn_mask=attn_mask,
                                       activation=self.activation, norm_type=self.norm_type)


from .generation import LlamaGenerator, sample_logits  # noqa: E402,F401
