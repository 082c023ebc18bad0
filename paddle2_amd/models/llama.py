"""Llama-2 for causal LM pretraining, built on paddle2_amd's Paddle-style API.

Structure follows the reference's Llama test/auto-parallel models
(test/auto_parallel/hybrid_strategy/semi_auto_parallel_llama_model.py:55-640: RMSNorm ->
q/k/v proj -> RoPE -> flash_attn -> o_proj -> RMSNorm -> gate/up -> swiglu -> down) with the
fused variants PaddleNLP uses (``fuse_attention_qkv``, ``fuse_attention_ffn``, fused residual
RMSNorm).  MI355X mapping of every op:

  RMSNorm (+ residual add)   -> csrc/kernels/norm.hip        (wave-per-row, fused residual)
  QKV / gate-up / o / down   -> hipBLASLt GEMM (plain library GEMMs, bf16 MFMA)
  RoPE                       -> csrc/kernels/elementwise.hip (rotate-half, fp32 cos/sin table)
  causal attention (GQA)     -> csrc/kernels/flash_attn.hip  (MFMA 32x32x16 fwd + bwd)
  SwiGLU                     -> csrc/kernels/elementwise.hip (packed [gate|up] input)
  embedding / softmax-CE     -> csrc/kernels/loss_embed.hip  (one-pass online LSE)

Tensor parallelism: when ``config.tensor_parallel_degree > 1`` the projections become
Column/RowParallelLinear and the embedding / LM head vocab-parallel (paddle2_amd.distributed.fleet).
Fused weights are laid out per mp rank: rank r's shard of ``qkv_proj`` is ``[q_r | k_r | v_r]`` and
of ``gate_up_fused_proj`` is ``[gate_r | up_r]``, so the local views need no reshuffle.
"""
from __future__ import annotations

import contextlib
import dataclasses
import math

import torch

from .. import nn
from ..framework.tensor import Tensor
from ..nn import functional as F
from ..nn import initializer as I
from ..ops import torch_ops as T

_wrap = Tensor._wrap


@dataclasses.dataclass
class LlamaConfig:
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    initializer_range: float = 0.02
    tie_word_embeddings: bool = False
    fuse_attention_qkv: bool = True
    fuse_attention_ffn: bool = True
    use_flash_attention: bool = True
    dtype: str = "bfloat16"
    tensor_parallel_degree: int = 1
    sequence_parallel: bool = False
    # context parallelism over the fleet ``sep`` axis: "ulysses" (head<->sequence all-to-all) or "ring"
    # (zigzag ring flash attention); inputs arrive as this rank's shard (shard_sequence)
    sep_parallel_degree: int = 1
    context_parallel: str = "ulysses"
    recompute: bool = False
    pad_token_id: int = 0
    ignore_index: int = -100

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads

    @classmethod
    def llama2_7b(cls, **kw):
        return cls(**kw)

    @classmethod
    def llama2_13b(cls, **kw):
        d = dict(hidden_size=5120, intermediate_size=13824, num_hidden_layers=40, num_attention_heads=40,
                 num_key_value_heads=40)
        d.update(kw)
        return cls(**d)

    @classmethod
    def tiny(cls, **kw):
        d = dict(vocab_size=512, hidden_size=256, intermediate_size=688, num_hidden_layers=2, num_attention_heads=2,
                 num_key_value_heads=2, max_position_embeddings=256)
        d.update(kw)
        return cls(**d)


def _linear(cfg, fin, fout, kind):
    """kind: 'col' (output-sharded) | 'row' (input-sharded) | None."""
    init = I.Normal(0.0, cfg.initializer_range)
    attr = nn.ParamAttr(initializer=init)
    if cfg.tensor_parallel_degree > 1 and kind is not None:
        from ..distributed.fleet.layers.mpu import ColumnParallelLinear, RowParallelLinear

        if kind == "col":
            return ColumnParallelLinear(fin, fout, weight_attr=attr, has_bias=False, gather_output=False)
        return RowParallelLinear(fin, fout, weight_attr=attr, has_bias=False, input_is_parallel=True)
    return nn.Linear(fin, fout, weight_attr=attr, bias_attr=False)


class LlamaRotaryEmbedding:
    """cos/sin tables (fp32, [max_pos, head_dim], rotate-half layout) cached per device."""

    def __init__(self, dim, max_pos, base):
        self.dim, self.max_pos, self.base = dim, max_pos, base
        self._cache = {}

    def tables(self, device, seq_len):
        n = max(seq_len, self.max_pos)
        key = (device, n)
        if key not in self._cache:
            self._cache[key] = T.rope_tables(n, self.dim, self.base, interleaved=False, device=device)
        return self._cache[key]


class LlamaRMSNorm(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.eps = config.rms_norm_eps
        self.weight = self.create_parameter([config.hidden_size], dtype=config.dtype,
                                            default_initializer=I.Constant(1.0))

    def forward(self, x, residual=None):
        if residual is None:
            return _wrap(T.rms_norm(x._t, self.weight._t, self.eps))
        y, h = T.rms_norm(x._t, self.weight._t, self.eps, residual._t)
        return _wrap(y), _wrap(h)


class LlamaAttention(nn.Layer):
    def __init__(self, config, rope):
        super().__init__()
        self.config = config
        tp = config.tensor_parallel_degree
        self.num_heads = config.num_attention_heads // tp
        self.num_kv = config.num_key_value_heads // tp
        self.head_dim = config.head_dim
        h = config.hidden_size
        self.rope = rope
        if config.fuse_attention_qkv:
            self.qkv_proj = _linear(config, h, h + 2 * config.num_key_value_heads * self.head_dim, "col")
        else:
            self.q_proj = _linear(config, h, h, "col")
            self.k_proj = _linear(config, h, config.num_key_value_heads * self.head_dim, "col")
            self.v_proj = _linear(config, h, config.num_key_value_heads * self.head_dim, "col")
        self.o_proj = _linear(config, h, h, "row")

    def _sep_group(self):
        from ..distributed import fleet

        return fleet.get_hybrid_communicate_group().get_sep_parallel_group()

    def forward(self, x, position_ids=None):
        b, s = x.shape[0], x.shape[1]
        nh, nkv, d = self.num_heads, self.num_kv, self.head_dim
        sep = self.config.sep_parallel_degree
        cos, sin = self.rope.tables(x._t.device, s * sep)
        pos = None if position_ids is None else position_ids._t
        if sep > 1:
            # context parallel: RoPE at the shard's global positions, then the sep-group attention exchange
            from ..distributed.fleet.meta_parallel import context_parallel as CP

            if self.config.fuse_attention_qkv:
                qkv = self.qkv_proj(x)._t.view(b, s, nh + 2 * nkv, d)
                q, k, v = qkv[:, :, :nh], qkv[:, :, nh:nh + nkv], qkv[:, :, nh + nkv:]
            else:
                q = self.q_proj(x)._t.view(b, s, nh, d)
                k = self.k_proj(x)._t.view(b, s, nkv, d)
                v = self.v_proj(x)._t.view(b, s, nkv, d)
            q = T.rope(q, cos, sin, pos, style=0)
            k = T.rope(k, cos, sin, pos, style=0)
            attn = CP.ring_flash_attention if self.config.context_parallel == "ring" else CP.ulysses_attention
            o = attn(q, k, v, self._sep_group(), causal=True)
            return self.o_proj(_wrap(o.reshape(b, s, nh * d)))
        if self.config.fuse_attention_qkv and type(self.qkv_proj) is nn.Linear and not (
                self.qkv_proj._forward_pre_hooks or self.qkv_proj._forward_post_hooks):
            w = self.qkv_proj.weight._t
            bias = None if self.qkv_proj.bias is None else self.qkv_proj.bias._t
            if T.qkv_rope_linear_ok(x._t, w, bias, d, pos):
                # RoPE in the QKV GEMM epilogue, attention on the rotated qkv in place
                c128 = cos.reshape(-1, d)[:s].float().contiguous()
                s128 = sin.reshape(-1, d)[:s].float().contiguous()
                if T._ROPE_BWD_IN_FLASH:
                    # one node: backward un-rotates dQ / dK inside the flash backward
                    o = T.qkv_proj_rope_attention(x._t, w, c128, s128, nh, nkv, s)
                else:
                    qkv = T._QKVRopeLinearFn.apply(x._t, w, c128, s128, nh + nkv, s).view(b, s, nh + 2 * nkv, d)
                    o = T.qkv_attention(qkv, nh, nkv, causal=True)
                return self.o_proj(_wrap(o.reshape(b, s, nh * d)))
        if self.config.fuse_attention_qkv:
            # one autograd node: strided q/k/v views -> RoPE -> flash attention; backward fills one dQKV
            qkv = self.qkv_proj(x)._t.view(b, s, nh + 2 * nkv, d)
            o = T.qkv_rope_attention(qkv, nh, nkv, cos, sin, pos, causal=True)
            return self.o_proj(_wrap(o.reshape(b, s, nh * d)))
        else:
            q = self.q_proj(x)._t.view(b, s, nh, d)
            k = self.k_proj(x)._t.view(b, s, nkv, d)
            v = self.v_proj(x)._t.view(b, s, nkv, d)
        q = T.rope(q, cos, sin, pos, style=0)
        k = T.rope(k, cos, sin, pos, style=0)
        o, _ = T.flash_attention(q, k, v, causal=True)
        return self.o_proj(_wrap(o.reshape(b, s, nh * d)))


class LlamaMLP(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.config = config
        h, f = config.hidden_size, config.intermediate_size
        if config.fuse_attention_ffn:
            self.gate_up_fused_proj = _linear(config, h, 2 * f, "col")
        else:
            self.gate_proj = _linear(config, h, f, "col")
            self.up_proj = _linear(config, h, f, "col")
        self.down_proj = _linear(config, f, h, "row")

    def forward(self, x):
        if self.config.fuse_attention_ffn and type(self.gate_up_fused_proj) is nn.Linear:
            gu, dn = self.gate_up_fused_proj, self.down_proj
            if (type(dn) is nn.Linear and gu.bias is None and dn.bias is None and not (
                    gu._forward_pre_hooks or gu._forward_post_hooks or dn._forward_pre_hooks
                    or dn._forward_post_hooks) and T.swiglu_mlp_ok(x._t, gu.weight._t, dn.weight._t)):
                # one node: the SwiGLU backward runs in the down projection's dgrad epilogue
                return _wrap(T.swiglu_mlp(x._t, gu.weight._t, dn.weight._t))
            a = T.swiglu_linear(x._t, self.gate_up_fused_proj.weight._t)  # one node: GEMM + SwiGLU (+dY^T)
        elif self.config.fuse_attention_ffn:
            a = T.swiglu(self.gate_up_fused_proj(x)._t)  # per-rank [gate_r | up_r]
        else:
            a = T.swiglu(self.gate_proj(x)._t, self.up_proj(x)._t)
        return self.down_proj(_wrap(a))


class LlamaDecoderLayer(nn.Layer):
    def __init__(self, config, rope):
        super().__init__()
        self.self_attn = LlamaAttention(config, rope)
        self.mlp = LlamaMLP(config)
        self.input_layernorm = LlamaRMSNorm(config)
        self.post_attention_layernorm = LlamaRMSNorm(config)

    def forward(self, hidden, residual=None, position_ids=None):
        """Returns (mlp_out, residual) so the next layer can fuse ``residual + mlp_out`` into its norm."""
        if residual is None:
            residual = hidden
            x = self.input_layernorm(hidden)
        else:
            x, residual = self.input_layernorm(hidden, residual)
        attn = self.self_attn(x, position_ids)
        x, residual = self.post_attention_layernorm(attn, residual)
        return self.mlp(x), residual


class LlamaModel(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.config = config
        init = nn.ParamAttr(initializer=I.Normal(0.0, config.initializer_range))
        if config.tensor_parallel_degree > 1:
            from ..distributed.fleet.layers.mpu import VocabParallelEmbedding

            self.embed_tokens = VocabParallelEmbedding(config.vocab_size, config.hidden_size, weight_attr=init)
        else:
            self.embed_tokens = nn.Embedding(config.vocab_size, config.hidden_size, weight_attr=init)
        rope = LlamaRotaryEmbedding(config.head_dim, config.max_position_embeddings, config.rope_theta)
        self.layers = nn.LayerList([LlamaDecoderLayer(config, rope) for _ in range(config.num_hidden_layers)])
        self.norm = LlamaRMSNorm(config)

    def forward(self, input_ids, position_ids=None):
        h = self.embed_tokens(input_ids)
        if position_ids is None and self.config.sep_parallel_degree > 1:
            from ..distributed import fleet
            from ..distributed.fleet.meta_parallel.context_parallel import context_positions

            hcg = fleet.get_hybrid_communicate_group()
            b, s = input_ids.shape[0], input_ids.shape[1]
            pos = context_positions(s, hcg.get_sep_parallel_world_size(), hcg.get_sep_parallel_rank(),
                                    self.config.context_parallel, device=h._t.device)
            position_ids = _wrap(pos[None].expand(b, s))
        residual = None
        for layer in self.layers:
            if self.config.recompute and self.training:
                from ..distributed.fleet.recompute import recompute

                h, residual = recompute(layer, h, residual, position_ids)
            else:
                h, residual = layer(h, residual, position_ids)
        out, _ = self.norm(h, residual)
        return out


class LlamaLMHead(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.config = config
        tp = config.tensor_parallel_degree
        vocab = config.vocab_size // tp
        self._mp_group = None
        ctx = contextlib.nullcontext()
        if tp > 1:
            from ..distributed.fleet.layers.mpu.mp_layers import _init_ctx, _mp_info

            self._mp_group = _mp_info(None)[0]
            ctx = _init_ctx(tp)
        with ctx:
            self.weight = self.create_parameter([config.hidden_size, vocab], dtype=config.dtype,
                                                default_initializer=I.Normal(0.0, config.initializer_range))
        if tp > 1:
            self.weight.is_distributed = True
            self.weight.split_axis = 1

    def forward(self, h):
        if self._mp_group is not None:
            # vocab-sharded logits; dX all-reduced over mp overlapping the dW GEMM
            from ..distributed.fleet.layers.mpu.mp_ops import _ColumnLinear

            return _wrap(_ColumnLinear.apply(h._t, self.weight._t, None, self._mp_group))
        return _wrap(T.linear(h._t, self.weight._t))


class LlamaPretrainingCriterion(nn.Layer):
    """Token-mean softmax cross entropy (vocab-parallel when TP > 1)."""

    def __init__(self, config):
        super().__init__()
        self.config = config

    def forward(self, logits, labels):
        if self.config.tensor_parallel_degree > 1:
            from ..distributed.fleet.layers.mpu import ParallelCrossEntropy

            loss = ParallelCrossEntropy(ignore_index=self.config.ignore_index)(logits, labels)._t
        else:
            loss = T.softmax_cross_entropy(logits._t, labels._t, self.config.ignore_index)
        valid = (labels._t != self.config.ignore_index).sum().clamp_min(1)
        return _wrap(loss.sum() / valid)


class LlamaForCausalLM(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.llama = LlamaModel(config)
        self.lm_head = LlamaLMHead(config)
        self.criterion = LlamaPretrainingCriterion(config)
        if config.dtype in ("bfloat16", "float16"):
            self.to(dtype=config.dtype)

    def forward(self, input_ids, labels=None, position_ids=None):
        h = self.llama(input_ids, position_ids)
        logits = self.lm_head(h)
        if labels is None:
            return logits
        return self.criterion(logits, labels)


def llama_flops_per_token(cfg: LlamaConfig, seq_len: int) -> float:
    """Training FLOPs/token: 6 * N_matmul_params + causal attention (fwd 2*2*s*h/2 per layer, x3 for bwd)."""
    h, f, L, V = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers, cfg.vocab_size
    kvh = cfg.num_key_value_heads * cfg.head_dim
    per_layer = h * (h + 2 * kvh) + h * h + 3 * h * f
    n = L * per_layer + h * V
    attn = L * 2 * 2 * seq_len * h / 2  # QK^T + PV, causal half, fwd
    return 6.0 * n + 3.0 * attn


# ============================================================================ pipeline-parallel form
class LlamaEmbeddingPipe(nn.Layer):
    """Stage-0 head of the pipeline: token ids -> hidden states."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        init = nn.ParamAttr(initializer=I.Normal(0.0, config.initializer_range))
        if config.tensor_parallel_degree > 1:
            from ..distributed.fleet.layers.mpu import VocabParallelEmbedding

            self.embed_tokens = VocabParallelEmbedding(config.vocab_size, config.hidden_size, weight_attr=init)
        else:
            self.embed_tokens = nn.Embedding(config.vocab_size, config.hidden_size, weight_attr=init)
        if config.dtype in ("bfloat16", "float16"):
            self.to(dtype=config.dtype)

    def forward(self, input_ids):
        return self.embed_tokens(input_ids)


class LlamaDecoderLayerPipe(LlamaDecoderLayer):
    """Decoder layer exchanging ``(hidden, residual)`` between pipeline stages (the first layer gets
    the bare embedding output)."""

    def __init__(self, config, layer_idx=0):
        rope = LlamaRotaryEmbedding(config.head_dim, config.max_position_embeddings, config.rope_theta)
        super().__init__(config, rope)
        self.config = config
        if config.dtype in ("bfloat16", "float16"):
            self.to(dtype=config.dtype)

    def forward(self, hidden, residual=None):
        if self.config.recompute and self.training:
            from ..distributed.fleet.recompute import recompute

            return recompute(super().forward, hidden, residual, None)
        return super().forward(hidden, residual, None)


class LlamaNormPipe(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.norm = LlamaRMSNorm(config)
        if config.dtype in ("bfloat16", "float16"):
            self.to(dtype=config.dtype)

    def forward(self, hidden, residual=None):
        if residual is None:
            return self.norm(hidden)
        out, _ = self.norm(hidden, residual)
        return out


class LlamaLMHeadPipe(LlamaLMHead):
    def __init__(self, config):
        super().__init__(config)
        if config.dtype in ("bfloat16", "float16"):
            self.to(dtype=config.dtype)


def LlamaForCausalLMPipe(config, num_stages=None, topology=None, seg_method="layer:LlamaDecoderLayerPipe",
                         num_virtual_pipeline_stages=None, recompute_interval=0):
    """Llama as a ``PipelineLayer`` (reference pattern: PaddleNLP LlamaForCausalLMPipe on
    fleet.meta_parallel.PipelineLayer): embedding | decoder layers | norm | LM head, loss =
    LlamaPretrainingCriterion; segmentation balances decoder layers across stages."""
    from ..distributed.fleet.meta_parallel import LayerDesc, PipelineLayer

    descs = [LayerDesc(LlamaEmbeddingPipe, config)]
    descs += [LayerDesc(LlamaDecoderLayerPipe, config, i) for i in range(config.num_hidden_layers)]
    descs += [LayerDesc(LlamaNormPipe, config), LayerDesc(LlamaLMHeadPipe, config)]
    crit = LlamaPretrainingCriterion(config)
    return PipelineLayer(descs, num_stages=num_stages, topology=topology, loss_fn=crit, seg_method=seg_method,
                         num_virtual_pipeline_stages=num_virtual_pipeline_stages,
                         recompute_interval=recompute_interval)
