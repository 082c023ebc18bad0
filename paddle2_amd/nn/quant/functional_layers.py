"""Layer wrappers for functional ops so quantization passes can see them
(reference: python/paddle/nn/quant/functional_layers.py)."""
from __future__ import annotations

from ..layer.layers import Layer


class FloatFunctionalLayer(Layer):
    def __init__(self):
        super().__init__()


def _mk(name, fn_name):
    def forward(self, *args, **kwargs):
        import paddle2_amd as paddle

        return getattr(paddle, fn_name)(*args, **kwargs)

    return type(name, (FloatFunctionalLayer,), {"forward": forward})


add = _mk("add", "add")
subtract = _mk("subtract", "subtract")
multiply = _mk("multiply", "multiply")
divide = _mk("divide", "divide")
reshape = _mk("reshape", "reshape")
transpose = _mk("transpose", "transpose")
concat = _mk("concat", "concat")
flatten = _mk("flatten", "flatten")
matmul = _mk("matmul", "matmul")
