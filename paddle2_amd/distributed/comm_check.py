"""Collective argument checks (reference: phi/core/distributed/check/static_check.h:25-34 and
nccl_dynamic_check.h:34-56).

* static (always on, host only): rank membership, dtype/shape agreement between the input and
  output buffers of one call (all_gather_into_tensor, reduce_scatter, alltoall), divisibility.
* dynamic (``FLAGS_enable_nccl_dynamic_check``): before the real collective, every rank
  all-gathers a tiny int64 descriptor (dtype code, ndim, numel, dims...) over the same group and
  compares it with its own — a mismatched shape/dtype across ranks raises a readable error on
  every rank instead of hanging or silently corrupting inside RCCL.  Costs one extra small
  collective per call, so it is a debugging mode like the reference's.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.float64: 3, torch.int32: 4, torch.int64: 5,
       torch.int8: 6, torch.uint8: 7, torch.bool: 8, torch.float8_e4m3fn: 9, torch.float8_e5m2: 10}
_MAXD = 8


class CommCheckError(RuntimeError):
    pass


def static_check(op, group, inp, out=None, *, root=None):
    n = group.nranks
    if group.rank < 0:
        raise CommCheckError(f"{op}: this rank is not a member of {group}")
    if root is not None and not (0 <= root < n):
        raise CommCheckError(f"{op}: root {root} out of range for a group of {n} ranks")
    if out is None:
        return
    if inp.dtype != out.dtype:
        raise CommCheckError(f"{op}: input dtype {inp.dtype} != output dtype {out.dtype}")
    if op == "all_gather_into_tensor" and out.numel() != inp.numel() * n:
        raise CommCheckError(f"{op}: output numel {out.numel()} != input numel {inp.numel()} x {n} ranks")
    if op == "reduce_scatter" and inp.numel() != out.numel() * n:
        raise CommCheckError(f"{op}: input numel {inp.numel()} != output numel {out.numel()} x {n} ranks")
    if op == "alltoall" and (inp.numel() % n or out.numel() != inp.numel()):
        raise CommCheckError(f"{op}: numel {inp.numel()} -> {out.numel()} not splittable across {n} ranks")


def _descriptor(t):
    d = torch.full((3 + _MAXD,), -1, dtype=torch.int64)
    d[0], d[1], d[2] = _DT.get(t.dtype, 99), t.dim(), t.numel()
    for i, s in enumerate(list(t.shape)[:_MAXD]):
        d[3 + i] = s
    return d


def dynamic_check(op, group, t, *, same_shape=True):
    from ..framework import flags

    if not flags.flag("FLAGS_enable_nccl_dynamic_check", False) or group.nranks <= 1 or group.pg is None:
        return
    dev = t.device if dist.get_backend(group.pg) == "nccl" else torch.device("cpu")
    mine = _descriptor(t).to(dev)
    allv = torch.empty(group.nranks * mine.numel(), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allv, mine, group=group.pg)
    allv = allv.cpu().view(group.nranks, -1)
    ref = allv[0]
    for r in range(1, group.nranks):
        a = allv[r]
        bad = a[0] != ref[0] or (same_shape and not torch.equal(a, ref))
        if bad:
            inv = {v: k for k, v in _DT.items()}

            def fmt(x):
                return f"dtype={inv.get(int(x[0]), '?')} shape={[int(s) for s in x[3:3 + int(x[1])]]}"

            raise CommCheckError(f"{op} on {group}: rank {group.ranks[r]} has {fmt(a)} but rank {group.ranks[0]} "
                                 f"has {fmt(ref)} (FLAGS_enable_nccl_dynamic_check)")
