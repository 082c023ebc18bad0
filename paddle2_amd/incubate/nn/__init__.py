"""paddle.incubate.nn (fused layers)."""
from . import functional  # noqa: F401
from .layers import FusedLinear, FusedMultiTransformer, FusedDropoutAdd  # noqa: F401

from . import attn_bias  # noqa: E402,F401
from .memory_efficient_attention import memory_efficient_attention, memory_efficient_attention_op  # noqa: E402,F401
