"""Expert-parallel token exchange (reference: python/paddle/distributed/utils/moe_utils.py —
``global_scatter`` :20, ``global_gather`` :153; CUDA op fluid/operators/collective/
global_scatter_op.cu.cc:129-165 issues one NCCL send/recv per (expert, rank) pair).

MI355X design: ONE ``all_to_all_single`` with per-rank split sizes moves every token (RCCL turns
it into a single grouped p2p exchange over the xGMI links), instead of n_expert x world grouped
send/recv rounds.  The reference's output order (expert-major, then source rank) is restored by
one row permutation on the receiver, and undone before the return trip.

Count convention (same as the reference): ``local_count[i]`` = rows this rank sends to local expert
``i % n_expert`` of rank ``i // n_expert``; ``global_count[i]`` = rows this rank receives from rank
``i // n_expert`` for its local expert ``i % n_expert``.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ...framework.tensor import Tensor
from ..collective import _get_default_group

_wrap = Tensor._wrap


def _counts(t):
    if isinstance(t, Tensor):
        t = t._t
    return [int(v) for v in t.detach().cpu().tolist()]


def _recv_perm(gcount, world, n_expert, device):
    """Row order of the all_to_all output is (src rank j, expert e); reference order is (e, j)."""
    starts, off = {}, 0
    for j in range(world):
        for e in range(n_expert):
            starts[(j, e)] = off
            off += gcount[j * n_expert + e]
    idx = []
    for e in range(n_expert):
        for j in range(world):
            s = starts[(j, e)]
            idx.extend(range(s, s + gcount[j * n_expert + e]))
    return torch.tensor(idx, dtype=torch.long, device=device)


def _a2a(x, send_split, recv_split, group):
    g = group if group is not None else _get_default_group()
    out = torch.empty((sum(recv_split),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    if g.nranks == 1:
        out.copy_(x)
        return out
    dist.all_to_all_single(out, x.contiguous(), recv_split, send_split, group=g.pg)
    return out


def _scatter_raw(x, lcount, gcount, group):
    g = group if group is not None else _get_default_group()
    world = g.nranks
    n_expert = len(lcount) // world
    send = [sum(lcount[j * n_expert:(j + 1) * n_expert]) for j in range(world)]
    recv = [sum(gcount[j * n_expert:(j + 1) * n_expert]) for j in range(world)]
    y = _a2a(x, send, recv, g)
    if n_expert > 1 and world > 1:
        y = y.index_select(0, _recv_perm(gcount, world, n_expert, y.device))
    return y


def _gather_raw(y, lcount, gcount, group):
    g = group if group is not None else _get_default_group()
    world = g.nranks
    n_expert = len(lcount) // world
    if n_expert > 1 and world > 1:
        perm = _recv_perm(gcount, world, n_expert, y.device)
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(perm.numel(), device=perm.device)
        y = y.index_select(0, inv)
    send = [sum(gcount[j * n_expert:(j + 1) * n_expert]) for j in range(world)]
    recv = [sum(lcount[j * n_expert:(j + 1) * n_expert]) for j in range(world)]
    return _a2a(y, send, recv, g)


class _GlobalScatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, lcount, gcount, group):
        ctx.meta = (lcount, gcount, group)
        return _scatter_raw(x, lcount, gcount, group)

    @staticmethod
    def backward(ctx, dy):
        lcount, gcount, group = ctx.meta
        return _gather_raw(dy, lcount, gcount, group), None, None, None


class _GlobalGather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, lcount, gcount, group):
        ctx.meta = (lcount, gcount, group)
        return _gather_raw(y, lcount, gcount, group)

    @staticmethod
    def backward(ctx, dx):
        lcount, gcount, group = ctx.meta
        return _scatter_raw(dx, lcount, gcount, group), None, None, None


def global_scatter(x, local_count, global_count, group=None, use_calc_stream=True):
    return _wrap(_GlobalScatter.apply(x._t, _counts(local_count), _counts(global_count), group))


def global_gather(x, local_count, global_count, group=None, use_calc_stream=True):
    return _wrap(_GlobalGather.apply(x._t, _counts(local_count), _counts(global_count), group))


def exchange_counts(local_count, group=None):
    """global_count from local_count: all-to-all of the per-expert counts (moe utils ``count_by_gate``)."""
    g = group if group is not None else _get_default_group()
    lc = local_count._t if isinstance(local_count, Tensor) else local_count
    if g.nranks == 1:
        return lc.clone()
    n_expert = lc.numel() // g.nranks
    out = torch.empty_like(lc)
    dist.all_to_all_single(out, lc.contiguous(), [n_expert] * g.nranks, [n_expert] * g.nranks, group=g.pg)
    return out
