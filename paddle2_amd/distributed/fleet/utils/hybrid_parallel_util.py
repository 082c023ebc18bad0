"""Hybrid-parallel parameter/gradient sync helpers (reference: fleet/utils/hybrid_parallel_util.py —
``broadcast_mp_parameters`` :218, ``broadcast_dp_parameters`` :229, ``broadcast_sharding_parameters``
:296, ``fused_allreduce_gradients`` :254-291, ``sharding_reduce_gradients``).

Gradient all-reduce packs grads into flat buckets per dtype (≤ ``bucket_mb``, default 256 MB —
large buckets suit xGMI rings, where per-message latency, not bandwidth, limits small
collectives), all-reduces each bucket with AVG and scatters back in place.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ....framework.tensor import Tensor
from ...parallel import sync_params_buffers


def broadcast_mp_parameters(model, hcg):
    g = hcg.get_model_parallel_group()
    sync_params_buffers(model, g, src_rank=0, is_model_parallel=True)


def broadcast_dp_parameters(model, hcg):
    g = hcg.get_data_parallel_group()
    sync_params_buffers(model, g, src_rank=0, is_model_parallel=False)


def broadcast_sharding_parameters(model, hcg):
    g = hcg.get_sharding_parallel_group()
    sync_params_buffers(model, g, src_rank=0, is_model_parallel=False)


def broadcast_sep_parameters(model, hcg):
    g = hcg.get_sep_parallel_group()
    if g is not None:
        sync_params_buffers(model, g, src_rank=0, is_model_parallel=False)


def _grad_tensor(p):
    mg = getattr(p, "main_grad", None)
    if mg is not None:
        return mg._t if isinstance(mg, Tensor) else mg
    return p._t.grad


def _allreduce_flat(grads, group, avg=True, bucket_mb=256):
    if group is None or group.nranks <= 1 or not grads:
        return
    by = {}
    for g in grads:
        by.setdefault((g.dtype, g.device), []).append(g)
    limit = bucket_mb << 20
    for ts in by.values():
        bucket, size = [], 0
        for t in ts + [None]:
            if t is not None:
                bucket.append(t)
                size += t.numel() * t.element_size()
            if (t is None or size >= limit) and bucket:
                flat = torch.cat([b.reshape(-1) for b in bucket]) if len(bucket) > 1 else bucket[0].reshape(-1)
                if group.backend == "nccl" and avg:
                    dist.all_reduce(flat, op=dist.ReduceOp.AVG, group=group.pg)
                else:
                    dist.all_reduce(flat, group=group.pg)
                    if avg:
                        flat.div_(group.nranks)
                if len(bucket) > 1 or flat.data_ptr() != bucket[0].data_ptr():
                    off = 0
                    for b in bucket:
                        n = b.numel()
                        b.copy_(flat[off:off + n].view_as(b))
                        off += n
                bucket, size = [], 0


def fused_allreduce_gradients(parameter_list, hcg, bucket_mb=256):
    """AVG all-reduce of grads over the dp (x sep) group."""
    if hcg is None:
        from ... import collective as C

        group = C._get_default_group()
    else:
        group = hcg.get_data_sep_parallel_group() if hcg.get_sep_parallel_world_size() > 1 else \
            hcg.get_data_parallel_group()
    grads = [_grad_tensor(p) for p in parameter_list]
    _allreduce_flat([g for g in grads if g is not None], group, True, bucket_mb)


def fused_allreduce_gradients_with_group(parameter_list, group, bucket_size=128 * 1024 * 1024, scale=None):
    grads = [_grad_tensor(p) for p in parameter_list]
    _allreduce_flat([g for g in grads if g is not None], group, scale is None, max(1, bucket_size >> 20))
    if scale is not None:
        for g in grads:
            if g is not None:
                g.mul_(scale)


def sharding_reduce_gradients(parameter_list, hcg):
    fused_allreduce_gradients_with_group(parameter_list, hcg.get_sharding_parallel_group())


def unwrap_optimizer(optimizer, optimizer_instances=()):
    inner = optimizer
    while hasattr(inner, "_inner_opt") and (not optimizer_instances or not isinstance(inner, optimizer_instances)):
        inner = inner._inner_opt
    return inner
