"""Kernels of the ops the PIR passes introduce into executed programs (pir/lowering.py)."""
from __future__ import annotations

from ..static.graph import graph_op


@graph_op
def fused_gemm_epilogue(x, w, bias=None, activation="identity"):
    """act(x @ W + bias) (reference paddle/phi/kernels/fusion/gpu/fused_gemm_epilogue_kernel.cu): the Linear GEMM
    node (native MFMA GEMM on the MI355X, bias in its epilogue when there is no activation) plus, with an
    activation, the fused bias-activation kernel — one pass over the output instead of three."""
    from ..ops import fused as FU
    from ..ops import torch_ops as T

    if activation == "identity":
        return T.linear(x, w, bias)
    return FU.bias_act(T.linear(x, w), bias, activation)


def alias(x):
    """Re-binds a value under another variable id (a fetch target whose producer CSE merged away)."""
    return x
