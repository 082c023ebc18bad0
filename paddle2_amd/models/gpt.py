"""GPT-3 style decoder (learned positions, LayerNorm, GELU MLP) with TP, Megatron sequence
parallelism and fp8 linears.

Reference model structure: the GPT test models in the reference
(test/auto_parallel/get_gpt_model.py, test/legacy_test/auto_parallel_gpt_model.py: embeddings ->
[LN -> fused QKV -> attention -> out proj -> LN -> fc1 -> GELU -> fc2] x L -> LN -> tied/untied
head) and SURVEY config 5 ("GPT-3 13B fp8 + sequence parallel + sharding-3").

MI355X mapping: LayerNorm fwd/bwd and the residual add run in the fused norm kernel
(csrc/kernels/norm.hip, layernorm path), attention in the MFMA flash kernels, projections in
hipBLASLt GEMMs (bf16) or fp8 GEMMs with delayed scaling (``use_fp8``).  With
``sequence_parallel`` activations between TP regions are sharded on the sequence dim ([s, b, h]
layout): column linears all-gather their input, row linears reduce-scatter their output, and the
LayerNorm params are SP-marked so their grads are summed over the mp group.
"""
from __future__ import annotations

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
class GPTConfig:
    vocab_size: int = 50304
    hidden_size: int = 5120
    num_hidden_layers: int = 40
    num_attention_heads: int = 40
    intermediate_size: int = 20480
    max_position_embeddings: int = 2048
    layer_norm_eps: float = 1e-5
    initializer_range: float = 0.02
    hidden_dropout_prob: float = 0.0
    attention_dropout_prob: float = 0.0
    dtype: str = "bfloat16"
    tensor_parallel_degree: int = 1
    sequence_parallel: bool = False
    use_fp8: bool = False
    recompute: bool = False
    tie_word_embeddings: bool = True
    ignore_index: int = -100

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads

    @classmethod
    def gpt3_13b(cls, **kw):
        return cls(**kw)

    @classmethod
    def gpt3_6_7b(cls, **kw):
        d = dict(hidden_size=4096, num_hidden_layers=32, num_attention_heads=32, intermediate_size=16384)
        d.update(kw)
        return cls(**d)

    @classmethod
    def gpt3_1_3b(cls, **kw):
        d = dict(hidden_size=2048, num_hidden_layers=24, num_attention_heads=16, intermediate_size=8192)
        d.update(kw)
        return cls(**d)

    @classmethod
    def tiny(cls, **kw):
        d = dict(vocab_size=512, hidden_size=128, num_hidden_layers=2, num_attention_heads=4, intermediate_size=512,
                 max_position_embeddings=128)
        d.update(kw)
        return cls(**d)


def _proj(cfg, fin, fout, kind, bias=True):
    """kind 'col' | 'row'; picks TP / SP / fp8 variants."""
    attr = nn.ParamAttr(initializer=I.Normal(0.0, cfg.initializer_range))
    tp = cfg.tensor_parallel_degree
    fp8 = True if cfg.use_fp8 else None   # TP / SP linears: fp8 local GEMMs, bf16 collectives
    if tp > 1:
        if cfg.sequence_parallel:
            from ..distributed.fleet.utils.sequence_parallel_utils import (ColumnSequenceParallelLinear,
                                                                           RowSequenceParallelLinear)

            if kind == "col":
                return ColumnSequenceParallelLinear(fin, fout, weight_attr=attr, has_bias=bias, gather_output=False,
                                                    fp8=fp8)
            return RowSequenceParallelLinear(fin, fout, weight_attr=attr, has_bias=bias, input_is_parallel=True,
                                             fp8=fp8)
        from ..distributed.fleet.layers.mpu import ColumnParallelLinear, RowParallelLinear

        if kind == "col":
            return ColumnParallelLinear(fin, fout, weight_attr=attr, has_bias=bias, gather_output=False, fp8=fp8)
        return RowParallelLinear(fin, fout, weight_attr=attr, has_bias=bias, input_is_parallel=True, fp8=fp8)
    if cfg.use_fp8:
        from ..incubate.fp8 import Float8Linear

        return Float8Linear(fin, fout, weight_attr=attr, bias_attr=None if bias else False)
    return nn.Linear(fin, fout, weight_attr=attr, bias_attr=None if bias else False)


class GPTLayerNorm(nn.Layer):
    def __init__(self, config):
        super().__init__()
        h = config.hidden_size
        self.eps = config.layer_norm_eps
        self.weight = self.create_parameter([h], default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([h], is_bias=True, default_initializer=I.Constant(0.0))
        if config.sequence_parallel and config.tensor_parallel_degree > 1:
            from ..distributed.fleet.utils.sequence_parallel_utils import mark_as_sequence_parallel_parameter

            mark_as_sequence_parallel_parameter(self.weight)
            mark_as_sequence_parallel_parameter(self.bias)

    def forward(self, x, residual=None):
        if residual is None:
            return _wrap(T.layer_norm(x._t, self.weight._t, self.bias._t, self.eps))
        y, h = T.layer_norm(x._t, self.weight._t, self.bias._t, self.eps, residual._t)
        return _wrap(y), _wrap(h)


class GPTAttention(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.config = config
        tp = config.tensor_parallel_degree
        self.nh = config.num_attention_heads // tp
        self.d = config.head_dim
        h = config.hidden_size
        self.qkv_proj = _proj(config, h, 3 * h, "col")   # per mp rank: [q_r | k_r | v_r]
        self.out_proj = _proj(config, h, h, "row")

    def forward(self, x):
        cfg = self.config
        qkv = self.qkv_proj(x)._t
        if cfg.sequence_parallel and cfg.tensor_parallel_degree > 1:
            s, b = qkv.shape[0], qkv.shape[1]
            qkv = qkv.transpose(0, 1)  # [b, s, ...] for attention
        else:
            b, s = qkv.shape[0], qkv.shape[1]
        qkv = qkv.reshape(b, s, 3 * self.nh, self.d)
        o = T.qkv_attention(qkv, self.nh, self.nh, causal=True)
        o = o.reshape(b, s, self.nh * self.d)
        if cfg.sequence_parallel and cfg.tensor_parallel_degree > 1:
            o = o.transpose(0, 1).contiguous()
        return self.out_proj(_wrap(o))


class GPTMLP(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.fc1 = _proj(config, config.hidden_size, config.intermediate_size, "col")
        self.fc2 = _proj(config, config.intermediate_size, config.hidden_size, "row")

    def forward(self, x):
        f1, f2 = self.fc1, self.fc2
        if (type(f1) is nn.Linear and type(f2) is nn.Linear and not (f1._forward_pre_hooks or f1._forward_post_hooks
                                                                     or f2._forward_pre_hooks or f2._forward_post_hooks)):
            args = (x._t, f1.weight._t, None if f1.bias is None else f1.bias._t, f2.weight._t,
                    None if f2.bias is None else f2.bias._t)
            if T.gelu_mlp_ok(*args):
                # one autograd node with GELU in the GEMM epilogues (forward GELU_AUX_BIAS, backward dGELU)
                return _wrap(T._GeluMLPFn.apply(*args, True))
        return self.fc2(F.gelu(self.fc1(x), approximate=True))


class GPTDecoderLayer(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.ln_1 = GPTLayerNorm(config)
        self.attn = GPTAttention(config)
        self.ln_2 = GPTLayerNorm(config)
        self.mlp = GPTMLP(config)

    def forward(self, hidden, residual=None):
        """Pre-LN block returning (mlp_out, residual); the next LN fuses the residual add."""
        if residual is None:
            residual = hidden
            x = self.ln_1(hidden)
        else:
            x, residual = self.ln_1(hidden, residual)
        a = self.attn(x)
        x, residual = self.ln_2(a, residual)
        return self.mlp(x), residual


class GPTModel(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.config = config
        init = nn.ParamAttr(initializer=I.Normal(0.0, config.initializer_range))
        if config.tensor_parallel_degree > 1:
            from ..distributed.fleet.layers.mpu import VocabParallelEmbedding

            self.word_embeddings = VocabParallelEmbedding(config.vocab_size, config.hidden_size, weight_attr=init)
        else:
            self.word_embeddings = nn.Embedding(config.vocab_size, config.hidden_size, weight_attr=init)
        self.position_embeddings = nn.Embedding(config.max_position_embeddings, config.hidden_size, weight_attr=init)
        self.layers = nn.LayerList([GPTDecoderLayer(config) for _ in range(config.num_hidden_layers)])
        self.final_norm = GPTLayerNorm(config)

    def forward(self, input_ids, position_ids=None):
        cfg = self.config
        b, s = input_ids.shape
        if position_ids is None:
            position_ids = _wrap(torch.arange(s, device=input_ids._t.device).unsqueeze(0).expand(b, s))
        h = self.word_embeddings(input_ids) + self.position_embeddings(position_ids)
        sp = cfg.sequence_parallel and cfg.tensor_parallel_degree > 1
        if sp:
            from ..distributed.fleet.utils.sequence_parallel_utils import ScatterOp

            h = ScatterOp.apply(_wrap(h._t.transpose(0, 1).contiguous()))  # [s/mp, b, h]
        residual = None
        for layer in self.layers:
            if cfg.recompute and self.training:
                from ..distributed.fleet.recompute import recompute

                h, residual = recompute(layer, h, residual)
            else:
                h, residual = layer(h, residual)
        out, _ = self.final_norm(h, residual)
        if sp:
            from ..distributed.fleet.utils.sequence_parallel_utils import GatherOp

            out = _wrap(GatherOp.apply(out)._t.transpose(0, 1).contiguous())
        return out


class GPTForCausalLM(nn.Layer):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.gpt = GPTModel(config)
        tp = config.tensor_parallel_degree
        if not config.tie_word_embeddings:
            self.lm_head = self.create_parameter([config.hidden_size, config.vocab_size // tp],
                                                 default_initializer=I.Normal(0.0, config.initializer_range))
            if tp > 1:
                self.lm_head.is_distributed = True
                self.lm_head.split_axis = 1
        else:
            self.lm_head = None
        if config.dtype in ("bfloat16", "float16"):
            self.to(dtype=config.dtype)

    def _sharding_root_params(self):
        """Stage-3 sharding: the tied word embedding is read again by the logits, outside its own layer."""
        return [self.gpt.word_embeddings.weight] if self.lm_head is None else []

    def _logits(self, h):
        cfg = self.config
        if cfg.tensor_parallel_degree > 1:
            from ..distributed.fleet.layers.mpu.mp_ops import _ColumnLinear
            from ..distributed.fleet.layers.mpu.mp_layers import _mp_info

            g = _mp_info(None)[0]
            w = self.gpt.word_embeddings.weight._t.t() if self.lm_head is None else self.lm_head._t
            return _wrap(_ColumnLinear.apply(h._t, w, None, g))
        if self.lm_head is None:   # tied: h @ E^T on the TN GEMM with E as stored
            return _wrap(T.tied_logits(h._t, self.gpt.word_embeddings.weight._t))
        return _wrap(T.linear(h._t, self.lm_head._t))

    def forward(self, input_ids, labels=None, position_ids=None):
        logits = self._logits(self.gpt(input_ids, position_ids))
        if labels is None:
            return logits
        cfg = self.config
        if cfg.tensor_parallel_degree > 1:
            from ..distributed.fleet.layers.mpu import ParallelCrossEntropy

            loss = ParallelCrossEntropy(ignore_index=cfg.ignore_index)(logits, labels)._t.squeeze(-1)
        else:
            loss = T.softmax_cross_entropy(logits._t, labels._t, cfg.ignore_index)
        valid = (labels._t != cfg.ignore_index).sum().clamp_min(1)
        return _wrap(loss.sum() / valid)


def gpt_flops_per_token(cfg: GPTConfig, seq_len: int) -> float:
    h, f, L, V = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers, cfg.vocab_size
    n = L * (4 * h * h + 2 * h * f) + h * V
    attn = L * 2 * 2 * seq_len * h / 2
    return 6.0 * n + 3.0 * attn
