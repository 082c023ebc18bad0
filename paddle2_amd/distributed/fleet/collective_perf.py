"""Collective performance check (reference: python/paddle/distributed/fleet/fleet.py:572-672
``collective_perf`` / ``_collective_perf_impl`` and the *_perf helpers).

Times ``round`` back-to-back collectives of each message size on the data-parallel (or sharding)
group for allreduce / reduce / broadcast and on the model-parallel group for allgather /
reduce_scatter, reports algorithm and bus bandwidth (nccl-tests conventions: allreduce bus =
alg x 2(n-1)/n, allgather / reduce_scatter bus = alg x (n-1)/n), and warns when a size exceeds
its time threshold.  Returns the measurements so callers can pick bucket sizes for the xGMI
topology.
"""
from __future__ import annotations

import logging
import time

import torch
import torch.distributed as dist

from .. import collective as C

logger = logging.getLogger("paddle2_amd.fleet")

_BUS = {"allreduce": lambda n: 2 * (n - 1) / n, "reduce": lambda n: 1.0, "broadcast": lambda n: 1.0,
        "allgather": lambda n: (n - 1) / n, "reduce_scatter": lambda n: (n - 1) / n}


def _run(comm_type, x, group):
    pg = group.pg
    n = group.nranks
    if comm_type == "allreduce":
        dist.all_reduce(x, group=pg)
    elif comm_type == "reduce":
        dist.reduce(x, dst=group.ranks[0], group=pg)
    elif comm_type == "broadcast":
        dist.broadcast(x, src=group.ranks[0], group=pg)
    elif comm_type == "allgather":
        out = torch.empty(x.numel() * n, dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x, group=pg)
    elif comm_type == "reduce_scatter":
        out = torch.empty(x.numel() // n, dtype=x.dtype, device=x.device)
        dist.reduce_scatter_tensor(out, x[: out.numel() * n], group=pg)
    else:
        raise ValueError(f"unknown comm_type {comm_type!r}")


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def perf_one(comm_type, nbytes, group, round=50, dtype=torch.float32):
    from ..fleet import _device_for_group

    dev = _device_for_group(group)
    n = group.nranks
    esz = torch.empty(0, dtype=dtype).element_size()
    numel = max(n, nbytes // esz // n * n)
    x = torch.zeros(numel, dtype=dtype, device=dev)
    for _ in range(3):
        _run(comm_type, x, group)
    _sync(dev)
    dist.barrier(group=group.pg)
    t0 = time.perf_counter()
    for _ in range(round):
        _run(comm_type, x, group)
    _sync(dev)
    dt = (time.perf_counter() - t0) / round
    algbw = numel * esz / dt / 1e9
    return {"comm_type": comm_type, "bytes": numel * esz, "nranks": n, "time_ms": dt * 1e3, "algbw_GBs": algbw,
            "busbw_GBs": algbw * _BUS[comm_type](n)}


def collective_perf(comm_type, round=50, size_and_time=None, hcg=None):
    """-> list of measurement dicts.  ``size_and_time`` = {nbytes: threshold_seconds}; empty means a
    1 MB .. 1 GB sweep without thresholds."""
    if hcg is None:
        from . import get_hybrid_communicate_group

        hcg = get_hybrid_communicate_group()
    data_group = hcg.get_data_parallel_group()
    if data_group.nranks <= 1 and hcg.get_sharding_parallel_group().nranks > 1:
        data_group = hcg.get_sharding_parallel_group()
    group = data_group if comm_type in ("allreduce", "reduce", "broadcast") else hcg.get_model_parallel_group()
    if group is None or group.nranks <= 1:
        group = C._get_default_group()
    plan = dict(size_and_time or {})
    if not plan:
        s = 1 << 20
        while s <= 1 << 30:
            plan[s] = None
            s <<= 1
    out = []
    for nbytes, thr in plan.items():
        if nbytes <= 0:
            logger.warning("collective perf size must be positive, got %s", nbytes)
            continue
        r = perf_one(comm_type, nbytes, group, round)
        out.append(r)
        msg = (f"[collective_perf] {comm_type} {r['bytes'] / 2**20:.1f} MB x{r['nranks']}: {r['time_ms']:.3f} ms, "
               f"algbw {r['algbw_GBs']:.1f} GB/s, busbw {r['busbw_GBs']:.1f} GB/s")
        if thr is not None and r["time_ms"] / 1e3 > thr:
            logger.warning(msg + f" (slower than threshold {thr * 1e3:.3f} ms)")
        else:
            logger.info(msg)
    return out
