"""Tensor-parallel layers (reference: fleet/layers/mpu/mp_layers.py — ``VocabParallelEmbedding`` :49,
``ColumnParallelLinear`` :336, ``RowParallelLinear`` :543, ``ParallelCrossEntropy`` :744).

Weights are stored Paddle-style ([in, out]) and already sharded: column-parallel shards the
output dim, row-parallel the input dim, vocab-parallel the vocab rows.  Distributed params carry
``is_distributed=True`` / ``split_axis`` so the hybrid optimizer and checkpoint code know they
are not replicated.  Shard initialisation draws from the tracker's ``model_parallel_rng`` state
so shards differ across the mp group while replicated params match.
"""
from __future__ import annotations

import contextlib

import torch

from ..... import nn
from .....framework.tensor import Tensor
from .....nn import initializer as I
from . import mp_ops
from .random import MODEL_PARALLEL_RNG, get_rng_state_tracker

_wrap = Tensor._wrap


def _mp_info(mp_group):
    if mp_group is not None:
        return mp_group, mp_group.nranks, max(mp_group.rank, 0)
    from .... import fleet

    hcg = fleet.get_hybrid_communicate_group()
    if hcg is None:
        return None, 1, 0
    return hcg.get_model_parallel_group(), hcg.get_model_parallel_world_size(), hcg.get_model_parallel_rank()


def _init_ctx(world):
    tr = get_rng_state_tracker()
    if world > 1 and MODEL_PARALLEL_RNG in tr.states_:
        return tr.rng_state(MODEL_PARALLEL_RNG)
    return contextlib.nullcontext()


class _Fp8Local:
    """fp8 local GEMM of a tensor-parallel linear (``fp8=True`` or a DelayedScaling recipe): the shard's matmul
    runs as e4m3 forward / e5m2-gradient GEMMs with per-layer delayed scaling (ops/fp8.py fp8_linear, the
    Float8Linear recipe) while the TP / SP collectives around it stay bf16 — each rank scales its own weight shard
    and gradient, the gathered activation is the same bytes on every rank (reference: fp8 GEMMs inside
    ColumnSequenceParallelLinear / RowSequenceParallelLinear, sequence_parallel_utils.py:429,564)."""

    def _init_fp8(self, fp8):
        self._fp8 = fp8
        self._fp8_metas = None

    def _fp8_on(self):
        return bool(getattr(self, "_fp8", None))

    def _fp8_mm(self, x, b):
        from .....ops import fp8 as F8

        dev = x.device
        if self._fp8_metas is None or self._fp8_metas[0].amax.device != dev:
            from .....incubate.fp8 import DelayedScaling

            r = self._fp8 if isinstance(self._fp8, DelayedScaling) else DelayedScaling()
            bwd = F8.E5M2 if r.fp8_format == "HYBRID" else F8.E4M3
            self._fp8_metas = (F8.FP8TensorMeta(F8.E4M3, r.amax_history_len, r.margin, dev),
                               F8.FP8TensorMeta(F8.E4M3, r.amax_history_len, r.margin, dev),
                               F8.FP8TensorMeta(bwd, r.amax_history_len, r.margin, dev))
        mx, mw, mg = self._fp8_metas
        return F8.fp8_linear(x, self.weight._t, b, mx, mw, mg)


class VocabParallelEmbedding(nn.Layer):
    def __init__(self, num_embeddings, embedding_dim, weight_attr=None, mp_group=None, name=None):
        super().__init__()
        self.model_parallel_group, self.world_size, self.rank = _mp_info(mp_group)
        self.origin_num_embeddings = num_embeddings
        self.is_mp = self.world_size > 1
        assert num_embeddings % self.world_size == 0, "vocab size must be divisible by mp degree"
        per = num_embeddings // self.world_size
        self.vocab_start_index = self.rank * per
        self._dtype = self._helper_dtype()
        with _init_ctx(self.world_size):
            self.weight = self.create_parameter([per, embedding_dim], attr=weight_attr, dtype=self._dtype,
                                                default_initializer=I.XavierNormal())
        self.weight.is_distributed = self.is_mp
        self.weight.split_axis = 0

    @staticmethod
    def _helper_dtype():
        from .....framework.dtype import get_default_dtype

        return get_default_dtype()

    def forward(self, x):
        out = mp_ops._c_lookup_table(self.weight, x, start_index=self.vocab_start_index)
        if self.is_mp:
            out = mp_ops._mp_allreduce(out, group=self.model_parallel_group)
        return out


class ColumnParallelLinear(nn.Layer, _Fp8Local):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=None, gather_output=True,
                 fuse_matmul_bias=False, mp_group=None, name=None, fp8=None):
        super().__init__()
        self._init_fp8(fp8)
        self.model_parallel_group, self.world_size, self.rank = _mp_info(mp_group)
        self.is_mp = self.world_size > 1
        assert out_features % self.world_size == 0, "out_features must be divisible by mp degree"
        self.output_size_per_partition = out_features // self.world_size
        self.gather_output = gather_output
        self.in_features, self.out_features = in_features, out_features
        dt = VocabParallelEmbedding._helper_dtype()
        with _init_ctx(self.world_size):
            self.weight = self.create_parameter([in_features, self.output_size_per_partition], attr=weight_attr,
                                                dtype=dt, default_initializer=I.XavierUniform())
        self.weight.is_distributed = self.is_mp
        self.weight.split_axis = 1
        if has_bias is None or has_bias:
            self.bias = self.create_parameter([self.output_size_per_partition], dtype=dt, is_bias=True,
                                              default_initializer=I.Constant(0.0))
            self.bias.is_distributed = self.is_mp
            self.bias.split_axis = 0
        else:
            self.bias = None

    def forward(self, x):
        b = None if self.bias is None else self.bias._t
        if self._fp8_on():
            xt = mp_ops._Identity.apply(x._t, self.model_parallel_group) if self.is_mp else x._t
            y = self._fp8_mm(xt, b)
        elif self.is_mp:
            y = mp_ops._ColumnLinear.apply(x._t, self.weight._t, b, self.model_parallel_group)
        else:
            from .....ops import torch_ops as T

            y = T.linear(x._t, self.weight._t, b)
        out = _wrap(y)
        if self.gather_output and self.is_mp:
            out = mp_ops._c_concat(out, group=self.model_parallel_group)
        return out


class RowParallelLinear(nn.Layer, _Fp8Local):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=True, input_is_parallel=False,
                 fuse_matmul_bias=False, mp_group=None, name=None, fp8=None):
        super().__init__()
        self._init_fp8(fp8)
        self.model_parallel_group, self.world_size, self.rank = _mp_info(mp_group)
        self.is_mp = self.world_size > 1
        assert in_features % self.world_size == 0, "in_features must be divisible by mp degree"
        self.input_size_per_partition = in_features // self.world_size
        self.input_is_parallel = input_is_parallel
        self.in_features, self.out_features = in_features, out_features
        dt = VocabParallelEmbedding._helper_dtype()
        with _init_ctx(self.world_size):
            self.weight = self.create_parameter([self.input_size_per_partition, out_features], attr=weight_attr,
                                                dtype=dt, default_initializer=I.XavierUniform())
        self.weight.is_distributed = self.is_mp
        self.weight.split_axis = 0
        self.bias = self.create_parameter([out_features], dtype=dt, is_bias=True,
                                          default_initializer=I.Constant(0.0)) if has_bias else None

    def forward(self, x):
        if self.is_mp and not self.input_is_parallel:
            x = mp_ops._c_split(x, group=self.model_parallel_group)
        from .....ops import torch_ops as T

        # the Linear node (native GEMMs, fp32 main-grad accumulation) then the mp all-reduce of the partials
        y = _wrap(self._fp8_mm(x._t, None) if self._fp8_on() else T.linear(x._t, self.weight._t))
        if self.is_mp:
            y = mp_ops._mp_allreduce(y, group=self.model_parallel_group)
        if self.bias is not None:
            y = _wrap(y._t + self.bias._t)
        return y


class ParallelCrossEntropy(nn.Layer):
    """Softmax CE over vocab-sharded logits (per-token loss, shape [..., 1] like the reference)."""

    def __init__(self, mp_group=None, name=None, ignore_index=-100):
        super().__init__()
        self.model_parallel_group, self.world_size, self.rank = _mp_info(mp_group)
        self.ignore_index = ignore_index

    def forward(self, input, label):
        lab = label._t
        if lab.dim() == input._t.dim():
            lab = lab.squeeze(-1)
        loss = mp_ops._VocabParallelCE.apply(input._t, lab, self.model_parallel_group, self.ignore_index)
        return _wrap(loss.unsqueeze(-1))
