"""paddle.incubate.nn (fused layers)."""
from . import functional  # noqa: F401
from .layers import FusedLinear, FusedMultiTransformer, FusedDropoutAdd  # noqa: F401
