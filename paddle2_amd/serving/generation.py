"""Autoregressive generation for Llama models on a paged KV cache, with the per-token decode step
captured in a HIP graph.

Prefill runs each prompt through the training kernels (fused-residual RMSNorm, hipBLASLt GEMMs,
RoPE, causal MFMA flash attention) and stores K/V rows in the paged cache; every decode step
processes one token per sequence with the flash-decoding kernel.  The decode step has static
shapes (fixed batch, device-side positions / sequence lengths / block tables, no host syncs),
so it is captured once with ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) and replayed: one
graph launch instead of ~10 kernel launches per layer per token.

Weights are static during generation, so every projection keeps a one-time transposed [N, K] copy
(``weight_layout="nk"``, the default on the GPU): hipBLASLt streams that layout ~1.5x faster at decode
shapes (M = batch; qkv 2.8 -> 4.0 TB/s, down_proj 1.1 -> 2.7 TB/s, profiles/r3_decode_gemm_layouts.jsonl)
for 13.5 GB of extra HBM on a 288 GB part.
"""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor
from ..ops import torch_ops as T
from . import PagedKVCache, decode_attention, write_kv


def sample_logits(logits, temperature=1.0, top_k=0, top_p=1.0, generator=None):
    """logits [B, V] -> token ids [B] (greedy when temperature == 0)."""
    if temperature == 0:
        return logits.argmax(-1)
    x = logits.float() / max(temperature, 1e-6)
    if top_k and top_k > 0:
        kth = torch.topk(x, top_k, dim=-1).values[:, -1:]
        x = x.masked_fill(x < kth, float("-inf"))
    if top_p < 1.0:
        sx, si = torch.sort(x, descending=True, dim=-1)
        cp = torch.softmax(sx, -1).cumsum(-1)
        drop = cp - torch.softmax(sx, -1) > top_p
        sx = sx.masked_fill(drop, float("-inf"))
        x = torch.full_like(x, float("-inf")).scatter(-1, si, sx)
    return torch.multinomial(torch.softmax(x, -1), 1, generator=generator).squeeze(-1)


class LlamaGenerator:
    def __init__(self, model, max_batch=8, max_seq_len=4096, block_size=64, num_blocks=None, use_graph=True,
                 weight_layout=None):
        self.model = model
        cfg = model.config
        self.cfg = cfg
        self.nh, self.nkv, self.d = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        dev = model.llama.embed_tokens.weight._t.device
        self.dev = dev
        dt = model.llama.embed_tokens.weight._t.dtype
        if num_blocks is None:
            num_blocks = max_batch * ((max_seq_len + block_size - 1) // block_size)
        self.cache = PagedKVCache(cfg.num_hidden_layers, num_blocks, block_size, self.nkv, self.d, max_batch,
                                  max_seq_len, dtype=dt, device=dev)
        self.max_batch = max_batch
        self.max_seq_len = max_seq_len
        self.cos, self.sin = T.rope_tables(max(max_seq_len, cfg.max_position_embeddings), self.d, cfg.rope_theta,
                                           interleaved=False, device=dev)
        self.use_graph = use_graph and dev.type == "cuda"
        self._graph = None
        # static decode-step buffers
        self._tok = torch.zeros(max_batch, dtype=torch.long, device=dev)
        self._pos = torch.zeros(max_batch, dtype=torch.int32, device=dev)
        self._lens = torch.zeros(max_batch, dtype=torch.int32, device=dev)
        # the KV-cache write's sequence index per decode row: static, so no arange / int32 cast per layer per step
        self._slots = torch.arange(max_batch, dtype=torch.int32, device=dev)
        self._logits = None
        import os

        self.weight_layout = (weight_layout or os.environ.get("PADDLE2_AMD_SERVING_LAYOUT")
                              or ("nk" if dev.type == "cuda" else "kn"))
        self._wt = {}

    def _mm_part(self, x, param):
        """x @ W for decode rows that run the split-K kernel, as its unreduced partials (weight_only.DecodePartials,
        summed by the residual-add + RMSNorm that consumes them: _norm); the plain product otherwise."""
        if self.weight_layout == "nk" and x.numel() <= 16 * x.shape[-1]:
            wt = self._wt_of(param)
            if wt is not None:
                from ..ops import weight_only as WO

                K = x.shape[-1]
                p = WO.decode_matmul_partials(x.reshape(-1, K), wt, tuple(x.shape[:-1]) + (wt.shape[0],))
                if p is not None:
                    return p
        return self._mm(x, param)

    def _norm(self, x, weight, residual):
        """Residual-add + RMSNorm of the layer stream; x may be a decode GEMM's unreduced partials."""
        from ..ops import weight_only as WO

        if isinstance(x, WO.DecodePartials):
            if residual is None:
                x = x.materialize()
            else:
                return T.rms_norm_partials(x, weight, self.cfg.rms_norm_eps, residual)
        if residual is None:
            return T.rms_norm(x, weight, self.cfg.rms_norm_eps), x
        return T.rms_norm(x, weight, self.cfg.rms_norm_eps, residual)

    def _wt_of(self, param):
        """The cached W^T of a projection ("nk" layout), refreshed in place when the parameter changed; None when the
        transposed copies do not fit (the layout then falls back to "kn")."""
        w = param._t
        key = id(param)
        ent = self._wt.get(key)
        if ent is None:
            if not self._wt and not self._nk_fits():
                self.weight_layout = "kn"
                return None
            ent = self._wt[key] = [w.data_ptr(), w._version, T.transpose2d(w)]
        elif ent[0] != w.data_ptr() or ent[1] != w._version:
            if ent[2].shape == (w.shape[1], w.shape[0]) and ent[2].dtype == w.dtype:
                ent[2].copy_(w.t())
            else:
                ent[2] = T.transpose2d(w)
                self._graph = None
            ent[0], ent[1] = w.data_ptr(), w._version
        return ent[2]

    def _mm(self, x, param):
        """x @ W for a Paddle-layout W [K, N]; with the "nk" layout through a cached contiguous W^T.

        A parameter whose storage or version changed (set_state_dict, an in-place update) is re-transposed INTO
        the cached buffer, so a captured decode graph that reads that buffer stays valid and sees the new
        weights; only a shape change replaces the buffer, and then the graph is dropped and re-captured."""
        w = param._t
        if self.weight_layout != "nk":
            return torch.matmul(x, w)
        key = id(param)
        ent = self._wt.get(key)
        if ent is None:
            if not self._wt and not self._nk_fits():
                self.weight_layout = "kn"  # no room for a transposed copy of every projection
                return torch.matmul(x, w)
            ent = self._wt[key] = [w.data_ptr(), w._version, T.transpose2d(w)]
        elif ent[0] != w.data_ptr() or ent[1] != w._version:
            if ent[2].shape == (w.shape[1], w.shape[0]) and ent[2].dtype == w.dtype:
                ent[2].copy_(w.t())
            else:
                ent[2] = T.transpose2d(w)
                self._graph = None
            ent[0], ent[1] = w.data_ptr(), w._version
        K = x.shape[-1]
        if x.numel() <= 64 * K:
            # decode ([B, 1, K] hidden states, B <= 64): the rows flattened to one [B, K] operand so the native
            # weight-streaming kernel sees them (ops/weight_only.decode_ok picks it or hipBLASLt per shape)
            from ..ops import weight_only as WO

            y = WO.decode_matmul(x.reshape(-1, K), ent[2])
            return y.view(*x.shape[:-1], y.shape[-1])
        return torch.matmul(x, ent[2].t())

    def _nk_fits(self):
        """The transposed copies (one per projection weight) fit in free device memory with a 10 % margin."""
        if self.dev.type != "cuda":
            return True
        need = 0
        for layer in self.model.llama.layers:
            for lin in (layer.self_attn.qkv_proj, layer.self_attn.o_proj, layer.mlp.gate_up_fused_proj,
                        layer.mlp.down_proj):
                need += lin.weight._t.numel() * lin.weight._t.element_size()
        need += self.model.lm_head.weight._t.numel() * self.model.lm_head.weight._t.element_size()
        free, _ = torch.cuda.mem_get_info(self.dev)
        return need * 1.1 < free

    # ------------------------------------------------------------------ layer pieces
    def _layer_qkv(self, layer, x, residual):
        h, residual = self._norm(x, layer.input_layernorm.weight._t, residual)
        qkv = self._mm(h, layer.self_attn.qkv_proj.weight)
        return qkv, residual

    def _layer_out(self, layer, o, residual, partials=False):
        # decode step (``partials``): the o / down projections hand their split-K partials to the next residual-add +
        # norm, which sums them (no reduce launch); the returned stream x may then be a DecodePartials
        a = self._mm_part(o, layer.self_attn.o_proj.weight) if partials else self._mm(o, layer.self_attn.o_proj.weight)
        h, residual = self._norm(a, layer.post_attention_layernorm.weight._t, residual)
        gu = self._mm(h, layer.mlp.gate_up_fused_proj.weight)
        down = self._mm_glu(gu, layer.mlp.down_proj.weight, partials=partials)   # SwiGLU inside the down GEMM
        if down is not None:
            return down, residual
        return self._mm(T.swiglu(gu), layer.mlp.down_proj.weight), residual

    def _mm_glu(self, gu, param, partials=False):
        """swiglu(gu) @ W on the SwiGLU-staged decode GEMM (<= 16 rows, cached W^T), else None; ``partials``: as the
        unreduced split-K partials (weight_only.DecodePartials) when available."""
        if self.weight_layout != "nk" or gu.numel() > 16 * gu.shape[-1]:
            return None
        from ..ops import weight_only as WO

        w = param._t
        ent = self._wt.get(id(param))
        if ent is None or ent[0] != w.data_ptr() or ent[1] != w._version:
            return None   # let _mm (re)build the cached W^T first
        gu2 = gu.reshape(-1, gu.shape[-1])
        if not WO.decode_glu_ok(gu2, ent[2]):
            return None
        if partials:
            p = WO.decode_glu_partials(gu2, ent[2], tuple(gu.shape[:-1]) + (ent[2].shape[0],))
            if p is not None:
                return p
        y = WO.decode_glu_matmul(gu2, ent[2])
        return y.view(*gu.shape[:-1], y.shape[-1])

    def _logits_of(self, h, residual):
        out, _ = self._norm(h, self.model.llama.norm.weight._t, residual)
        return self._mm(out, self.model.lm_head.weight)

    # ------------------------------------------------------------------ prefill
    @torch.no_grad()
    def prefill(self, slot, ids):
        """Run prompt ``ids`` (1-D LongTensor) for sequence ``slot``; returns last-token logits [V]."""
        n = ids.numel()
        self.cache.allocate(slot, n + 1)
        nh, nkv, d = self.nh, self.nkv, self.d
        x = self.model.llama.embed_tokens.weight._t[ids.to(self.dev)][None]  # [1, n, h]
        pos = torch.arange(n, device=self.dev)
        residual = None
        for li, layer in enumerate(self.model.llama.layers):
            qkv, residual = self._layer_qkv(layer, x, residual)
            qkv = qkv.view(1, n, nh + 2 * nkv, d)
            q = T.rope(qkv[:, :, :nh], self.cos, self.sin, None, style=0)
            k = T.rope(qkv[:, :, nh:nh + nkv], self.cos, self.sin, None, style=0)
            v = qkv[:, :, nh + nkv:]
            write_kv(k[0].contiguous(), v[0].contiguous(), self.cache.k[li], self.cache.v[li],
                     torch.full((n,), slot, device=self.dev), pos, self.cache.block_table)
            o, _ = T.flash_attention(q, k, v, causal=True)
            x, residual = self._layer_out(layer, o.reshape(1, n, nh * d), residual)
        self.cache.seq_lens[slot] = n
        return self._logits_of(x[:, -1:], residual[:, -1:])[0, 0]

    @torch.no_grad()
    def prefill_batch(self, slots, prompts):
        """Run several prompts as ONE packed token batch (the reference's batched encoder pass of
        block_multihead_attention, seq_lens_encoder): every projection GEMM sees all prompts' tokens — M = the
        summed lengths instead of one prompt's, so a 1024-token prompt no longer under-fills the 256 CUs — and
        attention is the varlen flash kernel over cu_seqlens.  Returns the last-token logits [len(prompts), V]."""
        lens = [len(p) for p in prompts]
        total = sum(lens)
        nh, nkv, d = self.nh, self.nkv, self.d
        for s, n in zip(slots, lens):
            self.cache.allocate(s, n + 1)
        ids = torch.as_tensor([int(t) for p in prompts for t in p], dtype=torch.long).to(self.dev)
        pos = torch.cat([torch.arange(n, dtype=torch.int32) for n in lens]).to(self.dev)
        tok_batch = torch.cat([torch.full((n,), s, dtype=torch.int32) for s, n in zip(slots, lens)]).to(self.dev)
        cu = torch.zeros(len(lens) + 1, dtype=torch.int32)
        cu[1:] = torch.cumsum(torch.as_tensor(lens, dtype=torch.int32), 0)
        last = (cu[1:] - 1).to(torch.long).to(self.dev)
        cu = cu.to(self.dev)
        pos_l = pos.long()[None]
        x = self.model.llama.embed_tokens.weight._t[ids][None]  # [1, total, h]
        residual = None
        for li, layer in enumerate(self.model.llama.layers):
            qkv, residual = self._layer_qkv(layer, x, residual)
            qkv = qkv.view(1, total, nh + 2 * nkv, d)
            qk = T.rope(qkv[:, :, :nh + nkv], self.cos, self.sin, pos_l, style=0)   # per-token positions
            q, k, v = qk[0, :, :nh], qk[0, :, nh:], qkv[0, :, nh + nkv:]
            write_kv(k, v, self.cache.k[li], self.cache.v[li], tok_batch, pos, self.cache.block_table)
            o, _ = T.flash_attention_varlen(q.contiguous(), k.contiguous(), v.contiguous(), cu, cu, max(lens),
                                            max(lens), causal=True)
            x, residual = self._layer_out(layer, o.reshape(1, total, nh * d), residual)
        for s, n in zip(slots, lens):
            self.cache.seq_lens[s] = n
        return self._logits_of(x[:, last], residual[:, last])[0]

    # ------------------------------------------------------------------ decode
    def _decode_body(self):
        nh, nkv, d = self.nh, self.nkv, self.d
        B = self.max_batch
        x = self.model.llama.embed_tokens.weight._t[self._tok][:, None]  # [B, 1, h]
        pos = self._pos.long()
        residual = None
        for li, layer in enumerate(self.model.llama.layers):
            qkv, residual = self._layer_qkv(layer, x, residual)
            qkv = qkv.view(B, 1, nh + 2 * nkv, d)
            # q and k are adjacent heads of qkv: one RoPE launch over both
            qk = T.rope(qkv[:, :, :nh + nkv], self.cos, self.sin, pos[:, None], style=0)
            q, k = qk[:, :, :nh], qk[:, :, nh:]
            # k and v stay strided views (the cache write takes row strides): no per-layer copies
            write_kv(k[:, 0], qkv[:, 0, nh + nkv:], self.cache.k[li], self.cache.v[li],
                     self._slots[:B], self._pos, self.cache.block_table)
            o = decode_attention(q[:, 0], self.cache.k[li], self.cache.v[li], self._lens, self.cache.block_table)
            x, residual = self._layer_out(layer, o.reshape(B, 1, nh * d), residual, partials=True)
        return self._logits_of(x, residual)[:, 0]

    @torch.no_grad()
    def decode_step(self, tokens, positions):
        """tokens/positions: [max_batch] (inactive slots may hold anything valid) -> logits [B, V]."""
        self._tok.copy_(tokens)
        self._pos.copy_(positions)
        self._lens.copy_(positions + 1)
        if not self.use_graph:
            return self._decode_body()
        if self._graph is None:
            from ..device.context import get_context

            s = get_context().capture_stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):  # warm up allocations outside the graph
                    self._decode_body()
            torch.cuda.current_stream().wait_stream(s)
            from ..ops import fp8

            fp8.before_capture()
            self._graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._graph):
                self._logits = self._decode_body()
        self._graph.replay()
        return self._logits

    # ------------------------------------------------------------------ generate
    @torch.no_grad()
    def generate(self, prompts, max_new_tokens=32, temperature=0.0, top_k=0, top_p=1.0, eos_token_id=None,
                 seed=0):
        """prompts: list of 1-D id sequences (<= max_batch). Returns list of generated id lists."""
        assert len(prompts) <= self.max_batch
        gen = torch.Generator(device=self.dev).manual_seed(seed) if self.dev.type == "cuda" else \
            torch.Generator().manual_seed(seed)
        B = self.max_batch
        toks = torch.zeros(B, dtype=torch.long, device=self.dev)
        pos = torch.zeros(B, dtype=torch.int32, device=self.dev)
        outs = [[] for _ in prompts]
        done = [False] * len(prompts)
        # one packed prefill for all prompts (per-prompt when a single one is given)
        first = (self.prefill_batch(list(range(len(prompts))), prompts) if len(prompts) > 1 else
                 self.prefill(0, torch.as_tensor(prompts[0], dtype=torch.long))[None]) if prompts else None
        for i, p in enumerate(prompts):
            t = sample_logits(first[i:i + 1], temperature, top_k, top_p, gen)[0]
            toks[i] = t
            pos[i] = len(p)
            outs[i].append(int(t))
            self.cache.allocate(i, len(p) + max_new_tokens + 1)
        for i in range(len(prompts), B):  # idle slots decode a dummy token at position 0
            self.cache.allocate(i, max_new_tokens + 2)
        for _ in range(max_new_tokens - 1):
            logits = self.decode_step(toks, pos)
            nxt = sample_logits(logits, temperature, top_k, top_p, gen)
            pos = pos + 1
            for i in range(len(prompts)):
                if done[i]:
                    continue
                ti = int(nxt[i])
                outs[i].append(ti)
                if eos_token_id is not None and ti == eos_token_id:
                    done[i] = True
            toks = nxt
            if all(done):
                break
        for i in range(B):
            self.cache.free(i)
        return outs


def greedy_reference(model, prompt, max_new_tokens):
    """Full-recompute greedy decoding with the training forward (test oracle)."""
    ids = torch.as_tensor(prompt, dtype=torch.long, device=model.llama.embed_tokens.weight._t.device)[None]
    out = []
    with torch.no_grad():
        for _ in range(max_new_tokens):
            logits = model(Tensor._wrap(ids))._t[0, -1]
            t = int(logits.argmax())
            out.append(t)
            ids = torch.cat([ids, torch.tensor([[t]], device=ids.device)], 1)
    return out
