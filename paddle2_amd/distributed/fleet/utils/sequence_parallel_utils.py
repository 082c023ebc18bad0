"""Megatron-style sequence parallelism inside the TP group (reference:
fleet/utils/sequence_parallel_utils.py — ``ScatterOp/GatherOp/AllGatherOp/ReduceScatterOp`` :85-138,
``mark_as_sequence_parallel_parameter`` :149, ``register_sequence_parallel_allreduce_hooks`` :170,
``ColumnSequenceParallelLinear`` :429, ``RowSequenceParallelLinear`` :560).

Activations outside the TP regions are sharded on the sequence dim (dim 0, ``[s, b, h]``).
Column linears all-gather their input; row linears reduce-scatter their output; the backward
reduce-scatter of dX overlaps the dW GEMM (RCCL on its own stream, ``async_op``).
"""
from __future__ import annotations

import torch

from .... import nn
from ....framework.tensor import Tensor
from ....nn import initializer as I
from ..layers.mpu import mp_ops
from ..layers.mpu.mp_layers import _Fp8Local, _init_ctx, _mp_info

_wrap = Tensor._wrap


def _mp_group():
    from ... import fleet

    hcg = fleet.get_hybrid_communicate_group()
    return None if hcg is None else hcg.get_model_parallel_group()


class _Scatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return mp_ops._split_dim(x, group, 0)

    @staticmethod
    def backward(ctx, g):
        return mp_ops._allgather_dim(g, ctx.group, 0), None


class _Gather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return mp_ops._allgather_dim(x, group, 0)

    @staticmethod
    def backward(ctx, g):
        return mp_ops._split_dim(g, ctx.group, 0), None


class _AllGather(torch.autograd.Function):
    """fwd all-gather on dim 0, bwd reduce-scatter (the pair used around TP regions)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return mp_ops._allgather_dim(x, group, 0)

    @staticmethod
    def backward(ctx, g):
        return mp_ops._reduce_scatter_dim0(g, ctx.group)[0], None


class _ReduceScatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return mp_ops._reduce_scatter_dim0(x, group)[0]

    @staticmethod
    def backward(ctx, g):
        return mp_ops._allgather_dim(g, ctx.group, 0), None


class _OpBase:
    fn = None

    @classmethod
    def apply(cls, x, group=None):
        group = group if group is not None else _mp_group()
        return _wrap(cls.fn.apply(x._t, group))


class ScatterOp(_OpBase):
    fn = _Scatter


class GatherOp(_OpBase):
    fn = _Gather


class AllGatherOp(_OpBase):
    fn = _AllGather


class ReduceScatterOp(_OpBase):
    fn = _ReduceScatter


def scatter(x, group=None):
    return ScatterOp.apply(x, group)


def all_gather(x, group=None):
    return AllGatherOp.apply(x, group)


def reduce_scatter(x, group=None):
    return ReduceScatterOp.apply(x, group)


def mark_as_sequence_parallel_parameter(parameter):
    parameter.sequence_parallel = True


def is_sequence_parallel_parameter(parameter):
    return getattr(parameter, "sequence_parallel", False)


def register_sequence_parallel_allreduce_hooks(model, accumulation_steps=1, fuse_sequence_parallel_allreduce=False):
    """All-reduce grads of SP-marked params over the mp group once their grad is final."""
    import torch.distributed as dist

    group = _mp_group()
    if group is None or group.nranks <= 1:
        return
    params = [p for p in model.parameters() if is_sequence_parallel_parameter(p)]

    def hook(t):
        if t.grad is not None:
            dist.all_reduce(t.grad, group=group.pg)

    for p in params:
        p._t.register_post_accumulate_grad_hook(hook)


class ColumnSequenceParallelLinear(nn.Layer, _Fp8Local):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=None, gather_output=True,
                 fuse_matmul_bias=False, mp_group=None, name=None, fp8=None):
        super().__init__()
        self._init_fp8(fp8)
        self.model_parallel_group, self.world_size, self.rank = _mp_info(mp_group)
        assert not gather_output, "ColumnSequenceParallelLinear requires gather_output=False"
        assert out_features % self.world_size == 0
        self.output_size_per_partition = out_features // self.world_size
        from ....framework.dtype import get_default_dtype

        dt = get_default_dtype()
        with _init_ctx(self.world_size):
            self.weight = self.create_parameter([in_features, self.output_size_per_partition], attr=weight_attr,
                                                dtype=dt, default_initializer=I.XavierUniform())
        self.weight.is_distributed = self.world_size > 1
        self.weight.split_axis = 1
        if has_bias is None or has_bias:
            self.bias = self.create_parameter([self.output_size_per_partition], dtype=dt, is_bias=True,
                                              default_initializer=I.Constant(0.0))
            self.bias.is_distributed = self.world_size > 1
            self.bias.split_axis = 0
        else:
            self.bias = None

    def forward(self, x):
        b = None if self.bias is None else self.bias._t
        if self._fp8_on():
            # all-gather of the sequence shards (bwd: reduce-scatter of dX), then the fp8 GEMM on the full sequence
            xf = _AllGather.apply(x._t, self.model_parallel_group) if self.world_size > 1 else x._t
            return _wrap(self._fp8_mm(xf, b))
        return _wrap(mp_ops._SeqColumnLinear.apply(x._t, self.weight._t, b, self.model_parallel_group))


class RowSequenceParallelLinear(nn.Layer, _Fp8Local):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=True, input_is_parallel=True,
                 fuse_matmul_bias=False, mp_group=None, name=None, fp8=None):
        super().__init__()
        self._init_fp8(fp8)
        self.model_parallel_group, self.world_size, self.rank = _mp_info(mp_group)
        assert input_is_parallel, "RowSequenceParallelLinear requires input_is_parallel=True"
        assert in_features % self.world_size == 0
        self.input_size_per_partition = in_features // self.world_size
        from ....framework.dtype import get_default_dtype

        dt = get_default_dtype()
        with _init_ctx(self.world_size):
            self.weight = self.create_parameter([self.input_size_per_partition, out_features], attr=weight_attr,
                                                dtype=dt, default_initializer=I.XavierUniform())
        self.weight.is_distributed = self.world_size > 1
        self.weight.split_axis = 0
        if has_bias:
            self.bias = self.create_parameter([out_features], dtype=dt, is_bias=True,
                                              default_initializer=I.Constant(0.0))
            mark_as_sequence_parallel_parameter(self.bias)
        else:
            self.bias = None

    def forward(self, x):
        if self._fp8_on():
            # fp8 GEMM of the partial sums, then their reduce-scatter onto the sequence shards (bwd: all-gather)
            y = self._fp8_mm(x._t, None)
            y = _ReduceScatter.apply(y, self.model_parallel_group) if self.world_size > 1 else y
        else:
            y = mp_ops._SeqRowLinear.apply(x._t, self.weight._t, self.model_parallel_group)
        if self.bias is not None:
            y = y + self.bias._t
        return _wrap(y)
