"""Tensor-parallel communication ops (reference: fleet/layers/mpu/mp_ops.py — ``_c_identity``
:39, ``_c_concat`` :110, ``_c_split`` :173, ``_mp_allreduce`` :231, ``_c_lookup_table`` :325,
``_c_softmax_with_cross_entropy`` :418, ``split`` :640).

Every op is a ``torch.autograd.Function`` whose collective runs on the mp group's RCCL
communicator (gloo on CPU).  The reference's ``c_softmax_with_cross_entropy`` CUDA op
(phi/kernels/gpu/c_softmax_with_cross_entropy_kernel.cu) becomes: one pass of our
``ce_stats`` HIP kernel over the local vocab shard (row max, sum-exp, target logit with the
shard's vocab offset), ONE packed all-reduce of 2 floats/row (max-rescaled sum-exp | target)
after a MAX all-reduce of the row max, and the ``ce_bwd`` kernel with the same offset.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .....framework.tensor import Tensor
from .....ops import _native as N
from .....ops import torch_ops as T
from ....collective import _get_default_group

_wrap = Tensor._wrap


def _grp(group):
    return group if group is not None else _get_default_group()


def _nr(group):
    return _grp(group).nranks


def _allreduce_(t, group, op=dist.ReduceOp.SUM, async_op=False):
    g = _grp(group)
    if g.nranks == 1:
        return None
    return dist.all_reduce(t, op=op, group=g.pg, async_op=async_op)


def _allgather_dim(t, group, dim):
    g = _grp(group)
    if g.nranks == 1:
        return t
    t = t.contiguous()
    if dim == 0:
        out = torch.empty((t.shape[0] * g.nranks,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=g.pg)
        return out
    parts = [torch.empty_like(t) for _ in range(g.nranks)]
    dist.all_gather(parts, t, group=g.pg)
    return torch.cat(parts, dim=dim)


def _split_dim(t, group, dim):
    g = _grp(group)
    if g.nranks == 1:
        return t
    return t.chunk(g.nranks, dim=dim)[g.rank].contiguous()


def _reduce_scatter_dim0(t, group, async_op=False):
    g = _grp(group)
    if g.nranks == 1:
        return t, None
    t = t.contiguous()
    out = torch.empty((t.shape[0] // g.nranks,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    w = dist.reduce_scatter_tensor(out, t, op=dist.ReduceOp.SUM, group=g.pg, async_op=async_op)
    return out, w


# ----------------------------------------------------------------------------- autograd ops
class _Identity(torch.autograd.Function):
    """fwd: identity; bwd: all-reduce(sum) over mp."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        _allreduce_(g, ctx.group)
        return g, None


class _AllReduce(torch.autograd.Function):
    """fwd: all-reduce(sum) over mp; bwd: identity."""

    @staticmethod
    def forward(ctx, x, group):
        y = x.contiguous().clone()
        _allreduce_(y, group)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None


class _Concat(torch.autograd.Function):
    """fwd: all-gather along the last dim; bwd: take this rank's slice."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _allgather_dim(x, group, x.dim() - 1)

    @staticmethod
    def backward(ctx, g):
        return _split_dim(g, ctx.group, g.dim() - 1), None


class _Split(torch.autograd.Function):
    """fwd: take this rank's slice of the last dim; bwd: all-gather."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _split_dim(x, group, x.dim() - 1)

    @staticmethod
    def backward(ctx, g):
        return _allgather_dim(g, ctx.group, g.dim() - 1), None


def _c_identity(tensor, group=None, skip_c_identity_dynamic=False):
    return _wrap(_Identity.apply(tensor._t, group))


def _mp_allreduce(tensor, op=None, group=None, use_calc_stream=True, use_model_parallel=True,
                  skip_c_identity_dynamic=False):
    return _wrap(_AllReduce.apply(tensor._t, group))


def _c_concat(tensor, group=None):
    return _wrap(_Concat.apply(tensor._t, group))


def _c_split(tensor, group=None):
    return _wrap(_Split.apply(tensor._t, group))


def _c_lookup_table(table, index, start_index=0, vocab_size=-1, name=None):
    """Embedding over a vocab shard: rows outside [start, start+V_local) give 0 (c_embedding)."""
    from .....ops import torch_ops as T

    return _wrap(T.embedding(index._t, table._t, None, start_index))


# ----------------------------------------------------------------------------- overlapped linears
class _ColumnLinear(torch.autograd.Function):
    """y = x @ W_shard (+ b_shard); bwd: dx = dy W^T all-reduced over mp *asynchronously* while the
    dW / db GEMMs run (the reference's ``mp_async_allreduce`` / ``InnerOverlapLinear``, mp_layers.py:190)."""

    @staticmethod
    def forward(ctx, x, w, b, group):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.save_for_backward(x2, w)
        ctx.group, ctx.has_b, ctx.xshape = group, b is not None, x.shape
        ctx.gt = getattr(w, "_p2_gt", None)
        return T.mm(x2, w, b).view(*x.shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dx = T.mm_t(dy2, w).view(ctx.xshape)
        work = _allreduce_(dx, ctx.group, async_op=True)
        dw = T.weight_grad(x2, dy2, ctx.gt) if ctx.needs_input_grad[1] else None
        db = T.bias_grad(dy2) if ctx.has_b and ctx.needs_input_grad[2] else None
        if work is not None:
            work.wait()
        return dx, dw, db, None


class _SeqColumnLinear(torch.autograd.Function):
    """Sequence-parallel column linear (sequence_parallel_utils.py:429): x is seq-sharded on dim 0.
    fwd: all-gather(x) -> GEMM.  bwd: dx_full = dy W^T reduce-scattered asynchronously while the
    dW GEMM runs (``SPInnerOverlapLinear`` :257).  The gathered input is kept (288 GB HBM) instead
    of re-gathered in backward."""

    @staticmethod
    def forward(ctx, x, w, b, group):
        xf = _allgather_dim(x, group, 0)
        x2 = xf.reshape(-1, xf.shape[-1])
        ctx.save_for_backward(x2, w)
        ctx.group, ctx.has_b, ctx.xfshape = group, b is not None, xf.shape
        ctx.gt = getattr(w, "_p2_gt", None)
        return T.mm(x2, w, b).view(*xf.shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dxf = T.mm_t(dy2, w).view(ctx.xfshape)
        dx, work = _reduce_scatter_dim0(dxf, ctx.group, async_op=True)
        dw = T.weight_grad(x2, dy2, ctx.gt) if ctx.needs_input_grad[1] else None
        db = T.bias_grad(dy2) if ctx.has_b and ctx.needs_input_grad[2] else None
        if work is not None:
            work.wait()
        return dx, dw, db, None


class _SeqRowLinear(torch.autograd.Function):
    """Sequence-parallel row linear (sequence_parallel_utils.py:560): GEMM -> reduce-scatter on dim 0;
    bwd: all-gather(dy) -> dx, dW."""

    @staticmethod
    def forward(ctx, x, w, group):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.save_for_backward(x2, w)
        ctx.group, ctx.xshape = group, x.shape
        ctx.gt = getattr(w, "_p2_gt", None)
        y = T.mm(x2, w).view(*x.shape[:-1], w.shape[1])
        out, _ = _reduce_scatter_dim0(y, group)
        return out

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dyf = _allgather_dim(dy, ctx.group, 0)
        dy2 = dyf.reshape(-1, dyf.shape[-1]).contiguous()
        dx = T.mm_t(dy2, w).view(ctx.xshape)
        dw = T.weight_grad(x2, dy2, ctx.gt) if ctx.needs_input_grad[1] else None
        return dx, dw, None


# ----------------------------------------------------------------------------- vocab-parallel CE
class _VocabParallelCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, group, ignore_index):
        g = _grp(group)
        Vl = logits.shape[-1]
        start = g.rank * Vl if g.nranks > 1 else 0
        x2 = logits.reshape(-1, Vl).contiguous()
        lab = labels.reshape(-1).to(torch.int64).contiguous()
        Nr = x2.shape[0]
        native = N.use_native(x2) and x2.dtype in (torch.float32, torch.bfloat16, torch.float16)
        if native:
            from .....ops.torch_ops import _DT

            C = N.native()
            mx = torch.empty(Nr, dtype=torch.float32, device=x2.device)
            se = torch.empty_like(mx)
            tgt = torch.empty_like(mx)
            C.ce_stats(_DT[x2.dtype], x2.data_ptr(), lab.data_ptr(), mx.data_ptr(), se.data_ptr(), tgt.data_ptr(), Nr,
                       Vl, start, N.stream())
        else:
            xf = x2.float()
            mx = xf.max(-1).values
            se = torch.exp(xf - mx[:, None]).sum(-1)
            local = lab - start
            ok = (local >= 0) & (local < Vl)
            tgt = torch.where(ok, xf.gather(1, local.clamp(0, Vl - 1)[:, None]).squeeze(1), torch.zeros_like(mx))
        gmx = mx.clone()
        _allreduce_(gmx, g, op=dist.ReduceOp.MAX)
        packed = torch.stack([se * torch.exp(mx - gmx), tgt])
        _allreduce_(packed, g)
        lse = gmx + torch.log(packed[0])
        valid = lab != ignore_index
        loss = torch.where(valid, lse - packed[1], torch.zeros_like(lse))
        ctx.save_for_backward(x2, lab, lse)
        ctx.meta = (start, ignore_index, native, logits.shape)
        return loss.reshape(labels.shape)

    @staticmethod
    def backward(ctx, dloss):
        x2, lab, lse = ctx.saved_tensors
        start, ignore, native, shape = ctx.meta
        Nr, Vl = x2.shape
        dl = dloss.reshape(-1).float().contiguous()
        if native:
            from .....ops.torch_ops import _DT

            C = N.native()
            dx = torch.empty_like(x2)
            C.ce_bwd(_DT[x2.dtype], x2.data_ptr(), lab.data_ptr(), lse.data_ptr(), dl.data_ptr(), dx.data_ptr(), Nr, Vl,
                     start, ignore, 0, N.stream())
        else:
            p = torch.exp(x2.float() - lse[:, None])
            local = lab - start
            ok = (local >= 0) & (local < Vl) & (lab != ignore)
            rows = torch.arange(Nr, device=x2.device)[ok]
            p[rows, local[ok]] -= 1.0
            valid = (lab != ignore).float()
            dx = (p * (dl * valid)[:, None]).to(x2.dtype)
        return dx.reshape(shape), None, None, None


def _c_softmax_with_cross_entropy(logits, label, group=None, return_softmax=False, ignore_index=-100):
    lab = label._t
    squeeze = lab.dim() == logits._t.dim()
    if squeeze:
        lab = lab.squeeze(-1)
    loss = _VocabParallelCE.apply(logits._t, lab, group, ignore_index).unsqueeze(-1)
    if return_softmax:
        g = _grp(group)
        lf = logits._t.float()
        gm = lf.max(-1, keepdim=True).values
        _allreduce_(gm, g, op=dist.ReduceOp.MAX)
        e = torch.exp(lf - gm)
        s = e.sum(-1, keepdim=True)
        _allreduce_(s, g)
        return _wrap(loss), _wrap((e / s).to(logits._t.dtype))
    return _wrap(loss)


def _linear(x, weight, bias=None, name=None):
    from .....nn import functional as F

    return F.linear(x, weight, bias)


def split(x, size, operation, axis=0, num_partitions=1, gather_out=True, weight_attr=None, bias_attr=None,
          name=None):
    """paddle.distributed.split (mp_ops.py:640): builds a parallel embedding / linear layer over the
    mp group and applies it to ``x``."""
    from .mp_layers import ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding

    if operation == "embedding":
        layer = VocabParallelEmbedding(size[0], size[1], weight_attr=weight_attr)
        return layer(x)
    if operation == "linear":
        if axis == 0:
            layer = RowParallelLinear(size[0], size[1], weight_attr=weight_attr, has_bias=bias_attr is not False,
                                      input_is_parallel=False)
        else:
            layer = ColumnParallelLinear(size[0], size[1], weight_attr=weight_attr, has_bias=bias_attr is not False,
                                         gather_output=gather_out)
        return layer(x)
    raise ValueError(f"unsupported operation {operation}")
