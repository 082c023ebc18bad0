"""Fused layers (reference: python/paddle/incubate/nn/layer/)."""
from __future__ import annotations

from ...nn import Layer
from ...nn import initializer as I
from . import functional as F


class FusedLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, transpose_weight=False, name=None):
        super().__init__()
        shape = [out_features, in_features] if transpose_weight else [in_features, out_features]
        self.transpose_weight = transpose_weight
        self.weight = self.create_parameter(shape, attr=weight_attr, default_initializer=I.XavierUniform())
        self.bias = self.create_parameter([out_features], attr=bias_attr, is_bias=True)

    def forward(self, x):
        return F.fused_linear(x, self.weight, self.bias, self.transpose_weight)


class FusedDropoutAdd(Layer):
    def __init__(self, p=0.5, mode="upscale_in_train", name=None):
        super().__init__()
        self.p, self.mode = p, mode

    def forward(self, x, y):
        return F.fused_dropout_add(x, y, self.p, self.training, self.mode)


class FusedMultiTransformer(Layer):
    """Inference decoder stack with KV cache (reference: incubate/nn/layer/fused_transformer.py)."""

    def __init__(self, embed_dim, num_heads, dim_feedforward, dropout_rate=0.0, activation="gelu",
                 normalize_before=True, num_layers=1, epsilon=1e-5, norm_type="layernorm", gqa_group_size=-1,
                 **kwargs):
        super().__init__()
        from ...serving import FusedMultiTransformerImpl

        self.impl = FusedMultiTransformerImpl(self, embed_dim, num_heads, dim_feedforward, activation, num_layers,
                                              epsilon, norm_type, gqa_group_size)

    def forward(self, src, attn_mask=None, caches=None, seq_lens=None, time_step=None, **kwargs):
        return self.impl.forward(src, attn_mask, caches, seq_lens, time_step)
