"""Flat parameter / gradient buffers and fused gradient communication
(reference: python/paddle/distributed/fleet/utils/tensor_fusion_helper.py — HOOK_ACTION :34,
assign_group_by_size :76, flatten_dense_tensors :99, FusedCommBuffer :384 (add_grad :592,
comm_grads :652, _comm_grads :672, scale_grads :736), obtain_storage :749, fused_parameters :925).

MI355X design notes: buffers are one contiguous allocation per (dtype, group) with every
parameter's gradient a view into it, so a bucket's collective is ONE RCCL call on a 128 MB-class
message (xGMI rings are per-link bound; fewer, larger messages amortise the per-collective
latency).  Communication is issued asynchronously the moment the last gradient of a bucket
arrives (gradient hooks) and joined in ``scale_grads`` — overlap with the rest of backward.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ....framework.tensor import Tensor
from ... import collective as C


class HOOK_ACTION:
    ALL_REDUCE = 0
    REDUCE = 1
    REDUCE_SCATTER = 2


alignment = {"gpu": 256, "cpu": 256}   # bytes
align = {torch.float16: 2, torch.bfloat16: 2, torch.float32: 4}


def _t(p):
    return p._t if isinstance(p, Tensor) else p


_pid = id  # FusedCommBuffer's constructor takes an ``id`` argument (reference signature)


def _aligned_numel(numel, dtype, nranks=1):
    """Elements so that every slot starts 256-byte aligned and the buffer splits evenly over ranks."""
    esz = torch.empty(0, dtype=dtype).element_size()
    unit = alignment["gpu"] // esz
    n = -(-numel // unit) * unit
    return n


def assign_group_by_size(parameters, group_size=128 * 1024 * 1024):
    """Greedy size-bounded grouping (per dtype, order preserved) -> {group_idx: [params]}."""
    groups, cur, cur_sz, cur_dt = {}, [], 0, None
    idx = 0
    for p in parameters:
        t = _t(p)
        sz = t.numel() * t.element_size()
        if cur and (t.dtype != cur_dt or cur_sz + sz > group_size):
            groups[idx] = cur
            idx += 1
            cur, cur_sz = [], 0
        cur.append(p)
        cur_sz += sz
        cur_dt = t.dtype
    if cur:
        groups[idx] = cur
    return groups


def flatten_dense_tensors(parameters, use_main_grad=False, fuse_param=True, warp_buffer=False, release_grad=False):
    """One flat buffer for the params (if ``fuse_param``; params become views) and one for their grads
    (fp32 when ``use_main_grad``).  Returns (param_storage, grad_storage)."""
    ts = [_t(p) for p in parameters]
    dtype = ts[0].dtype
    dev = ts[0].device
    offs, total = [], 0
    for t in ts:
        offs.append(total)
        total += _aligned_numel(t.numel(), dtype)
    pbuf = None
    if fuse_param:
        pbuf = torch.zeros(total, dtype=dtype, device=dev)
        for t, o in zip(ts, offs):
            pbuf[o:o + t.numel()].copy_(t.detach().reshape(-1))
            t.data = pbuf[o:o + t.numel()].view(t.shape)
    gdt = torch.float32 if use_main_grad else dtype
    gbuf = None if release_grad else torch.zeros(total, dtype=gdt, device=dev)
    for p, t, o in zip(parameters, ts, offs):
        p._fused_offset = o
    return pbuf, gbuf


def obtain_storage(parameters, use_main_grad=False, clip=True, dist=False, fuse_param=True, comm_overlap=False,
                   act=None, comm_group=None, dst=-1, acc_steps=1, scale_after_comm=False, apply_decay_param_fun=None):
    if not parameters:
        return [], []
    var_groups = assign_group_by_size(parameters)
    storages, buffers = [], []
    for gid, params in var_groups.items():
        if comm_overlap:
            buf = FusedCommBuffer(gid, params, comm_group, acc_steps, act, dst, use_main_grad, fuse_param,
                                  scale_after_comm)
            buffers.append(buf)
            storages.append(buf.param_storage)
        else:
            pbuf, _ = flatten_dense_tensors(params, use_main_grad, fuse_param)
            storages.append(pbuf)
    return storages, buffers


class FusedCommBuffer:
    """Gradient bucket for a list of parameters: grads accumulate into one flat buffer; when every
    param has checked in ``acc_steps`` times the bucket's collective is launched asynchronously."""

    def __init__(self, id, params, comm_group, acc_steps=1, act=None, dst=-1, use_main_grad=None, fuse_param=False,
                 scale_after_comm=True, release_grads=False, use_reduce_avg=False, free_grads_in_comm=False):
        self._id = id
        self._params = list(params)
        self._acc_steps = acc_steps
        self._comm_group = comm_group or C._get_default_group()
        self._act = HOOK_ACTION.ALL_REDUCE if act is None else act
        self._dst = dst
        self._scale_after_comm = scale_after_comm
        self._use_reduce_avg = use_reduce_avg
        ts = [_t(p) for p in self._params]
        self._dtype = ts[0].dtype
        self.use_main_grad = bool(use_main_grad) if use_main_grad is not None else hasattr(self._params[0],
                                                                                           "main_grad")
        gdt = torch.float32 if self.use_main_grad else self._dtype
        n = self._comm_group.nranks
        self._offs, total = [], 0
        for t in ts:
            self._offs.append(total)
            total += _aligned_numel(t.numel(), gdt)
        total = -(-total // max(n, 1)) * max(n, 1)  # reduce-scatter needs an even split
        self.param_storage = None
        if fuse_param:
            self.param_storage, _ = flatten_dense_tensors(self._params, fuse_param=True, release_grad=True)
        self.grad_storage = torch.zeros(total, dtype=gdt, device=ts[0].device)
        self._numel = total
        self._task = None
        self._steps = {_pid(p): 0 for p in self._params}
        self._checked_in = 0
        self._index = {_pid(p): i for i, p in enumerate(self._params)}
        self._shard = None

    @property
    def params(self):
        return self._params

    def _slot(self, i):
        t = _t(self._params[i])
        return self.grad_storage[self._offs[i]:self._offs[i] + t.numel()].view(t.shape)

    def add_grad(self, param, use_comm=True):
        i = self._index[_pid(param)]
        slot = self._slot(i)
        g = getattr(param, "main_grad", None) if self.use_main_grad else None
        g = _t(g) if g is not None else _t(param).grad
        if g is not None and g.data_ptr() != slot.data_ptr():
            slot.add_(g.to(slot.dtype))
        if not self.use_main_grad:
            _t(param).grad = slot  # grads live in the bucket from now on
        self._steps[_pid(param)] += 1
        if self._steps[_pid(param)] == self._acc_steps:
            self._checked_in += 1
        if self._checked_in == len(self._params) and use_comm:
            self.comm_grads()

    def _all_params_checked_in(self):
        return self._checked_in == len(self._params)

    def comm_grads(self):
        assert self._all_params_checked_in(), "not every parameter of the bucket has its gradient yet"
        self._comm_grads()

    def _comm_grads(self):
        g = self._comm_group
        if g.nranks <= 1:
            self._task = None
            return
        pg = g.pg
        avg = self._use_reduce_avg and g.backend == "nccl"
        op = dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM
        self._scale_needed = not avg
        if self._act == HOOK_ACTION.ALL_REDUCE:
            self._task = dist.all_reduce(self.grad_storage, op=op, group=pg, async_op=True)
        elif self._act == HOOK_ACTION.REDUCE:
            dst = self._dst if self._dst >= 0 else 0
            self._task = dist.reduce(self.grad_storage, dst=g.ranks[dst], op=op, group=pg, async_op=True)
        else:
            n = g.nranks
            self._shard = torch.empty(self._numel // n, dtype=self.grad_storage.dtype, device=self.grad_storage.device)
            self._task = dist.reduce_scatter_tensor(self._shard, self.grad_storage, op=op, group=pg, async_op=True)

    def scale_grads(self):
        if self._task is not None:
            self._task.wait()
            self._task = None
        n = self._comm_group.nranks
        if n > 1 and self._scale_after_comm and getattr(self, "_scale_needed", True):
            if self._act == HOOK_ACTION.REDUCE_SCATTER and self._shard is not None:
                self._shard.div_(n)
            else:
                self.grad_storage.div_(n)
        if self._act == HOOK_ACTION.REDUCE_SCATTER and self._shard is not None:
            r = self._comm_group.rank
            seg = self._numel // n
            self.grad_storage[r * seg:(r + 1) * seg].copy_(self._shard)
        if self.use_main_grad:
            for i, p in enumerate(self._params):
                mg = getattr(p, "main_grad", None)
                if mg is not None:
                    _t(mg).copy_(self._slot(i))
        self._reset()

    def _reset(self):
        self._steps = {k: 0 for k in self._steps}
        self._checked_in = 0

    def _clear_grad_storage(self):
        self.grad_storage.zero_()
        self._reset()


def fused_parameters(parameters, use_main_grad=False, fuse_param=True, comm_overlap=False, comm_group=None,
                     act=None, dst=-1, acc_step=1, scale_after_comm=False, apply_decay_param_fun=None):
    """Split params into decay / no-decay groups and build their flat buffers.
    Returns (decay_fused, all_fused, all_buffers)."""
    decay = [p for p in parameters if apply_decay_param_fun is None or apply_decay_param_fun(p.name)]
    other = [p for p in parameters if p not in decay]
    d_st, d_buf = obtain_storage(decay, use_main_grad, fuse_param=fuse_param, comm_overlap=comm_overlap, act=act,
                                 comm_group=comm_group, dst=dst, acc_steps=acc_step, scale_after_comm=scale_after_comm)
    o_st, o_buf = obtain_storage(other, use_main_grad, fuse_param=fuse_param, comm_overlap=comm_overlap, act=act,
                                 comm_group=comm_group, dst=dst, acc_steps=acc_step, scale_after_comm=scale_after_comm)
    return d_st, d_st + o_st, d_buf + o_buf
