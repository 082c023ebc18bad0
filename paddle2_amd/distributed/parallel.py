"""``paddle.DataParallel`` with a zero-copy bucketed gradient reducer.

Reference: python/paddle/distributed/parallel.py:219 (DataParallel, sync_params_buffers :164,
bucket sizes 25 MB + 1 MB :377) and paddle/fluid/distributed/collective/reducer.cc (EagerReducer:
size-grouped buckets, MarkVarReady -> MarkGroupReady -> FusedAllReduceSchedule with concat into a
flat buffer, then split back in FinalizeBackward).

MI355X design:
  * grads live *inside* the bucket: every parameter's ``.grad`` is a view into one flat
    per-bucket buffer, so torch's AccumulateGrad writes straight into the communication buffer —
    the reference's ConcatTensors/SplitTensors copies disappear;
  * a post-accumulate-grad hook counts readiness; a full bucket launches an async RCCL
    all-reduce immediately, overlapping the rest of backward (RCCL runs on its own stream);
  * bucket sizes are chosen for xGMI rings + 288 GB HBM: the first-ready (last-layer) bucket is
    small (8 MB) so communication starts early, the rest 64 MB (fewer, larger collectives on the
    per-link-bound ring);
  * AVG is folded into the collective (RCCL ReduceOp.AVG), a final autograd-engine callback
    waits on outstanding buckets before ``backward()`` returns.
"""
from __future__ import annotations

import contextlib
import math

import torch
import torch.distributed as dist

from ..framework.tensor import Tensor
from ..nn.layer.layers import Layer
from . import collective as C


def sync_params_buffers(model, comm_group=None, src_rank=0, is_model_parallel=False, fuse_params=True):
    g = comm_group or C._get_default_group()
    if g.nranks <= 1:
        return
    objs = list(model.parameters()) + list(model.buffers())
    tensors = [o._t for o in objs if not (is_model_parallel and getattr(o, "is_distributed", False))]
    by_dt = {}
    for t in tensors:
        by_dt.setdefault((t.dtype, t.device), []).append(t)
    for ts in by_dt.values():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        dist.broadcast(flat, src=g.ranks[src_rank], group=g.pg)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


class _Bucket:
    __slots__ = ("params", "buf", "pending", "work", "ready_count", "offsets")

    def __init__(self, params, dtype, device):
        self.params = params
        n = sum(p._t.numel() for p in params)
        self.buf = torch.zeros(n, dtype=dtype, device=device)
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += p._t.numel()
        self.pending = len(params)
        self.work = None
        self.ready_count = 0


class Reducer:
    """Bucketed asynchronous gradient all-reduce over a data-parallel group."""

    def __init__(self, params, group, bucket_bytes=64 << 20, first_bucket_bytes=8 << 20, find_unused=False,
                 grad_scale_avg=True):
        self.group = group
        self.find_unused = find_unused
        self.enabled = True
        self._avg = grad_scale_avg
        self._hooks = []
        self._callback_queued = False
        params = [p for p in params if not p.stop_gradient]
        # reverse registration order ~= gradient arrival order
        order = list(reversed(params))
        self.buckets = []
        cur, cur_bytes, limit = [], 0, first_bucket_bytes
        for p in order:
            nb = p._t.numel() * p._t.element_size()
            if cur and (cur_bytes + nb > limit or p._t.dtype != cur[0]._t.dtype):
                self.buckets.append(cur)
                cur, cur_bytes, limit = [], 0, bucket_bytes
            cur.append(p)
            cur_bytes += nb
        if cur:
            self.buckets.append(cur)
        self.buckets = [_Bucket(b, b[0]._t.dtype, b[0]._t.device) for b in self.buckets]
        self._where = {}
        for bi, b in enumerate(self.buckets):
            for pi, p in enumerate(b.params):
                self._where[id(p._t)] = (bi, pi)
                self._bind_grad(b, pi)
                self._hooks.append(p._t.register_post_accumulate_grad_hook(self._on_grad))

    def _bind_grad(self, b, pi):
        p = b.params[pi]
        off = b.offsets[pi]
        n = p._t.numel()
        p._t.grad = b.buf[off:off + n].view_as(p._t)
        p._keep_grad_storage = True  # optimizer.clear_grad zeroes the bucket view in place

    def rebind(self):
        """Re-point .grad at the bucket views (after user code replaced/cleared grads)."""
        for b in self.buckets:
            for pi, p in enumerate(b.params):
                g = p._t.grad
                off = b.offsets[pi]
                view = b.buf[off:off + p._t.numel()]
                if g is None or g.data_ptr() != view.data_ptr():
                    if g is not None:
                        view.copy_(g.reshape(-1))
                    else:
                        view.zero_()
                    p._t.grad = view.view_as(p._t)

    def _on_grad(self, t):
        if not self.enabled:
            return
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        bi, pi = self._where[id(t)]
        b = self.buckets[bi]
        g = t.grad
        off = b.offsets[pi]
        if g is not None and g.data_ptr() != b.buf[off:off + 1].data_ptr():
            # grad was re-allocated outside the bucket (e.g. set_to_zero=False): copy it in
            b.buf[off:off + t.numel()].copy_(g.reshape(-1))
            t.grad = b.buf[off:off + t.numel()].view_as(t)
        b.ready_count += 1
        if b.ready_count == b.pending:
            self._launch(b)

    def _launch(self, b):
        g = self.group
        if g.nranks <= 1:
            b.work = None
            return
        if g.backend == "nccl" and self._avg:
            b.work = dist.all_reduce(b.buf, op=dist.ReduceOp.AVG, group=g.pg, async_op=True)
        else:
            b.work = dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=g.pg, async_op=True)

    def _finalize(self):
        self._callback_queued = False
        for b in self.buckets:
            if b.ready_count < b.pending:
                if not self.find_unused:
                    # unused parameters: reduce the bucket anyway (their grads are zero)
                    pass
                self._launch(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None
                if not (self.group.backend == "nccl" and self._avg) and self._avg:
                    b.buf.div_(self.group.nranks)
            b.ready_count = 0

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()


class DataParallel(Layer):
    def __init__(self, layers, strategy=None, comm_buffer_size=64, last_comm_buffer_size=8,
                 find_unused_parameters=False, group=None):
        super().__init__()
        self._layers = layers
        self.find_unused_parameters = find_unused_parameters
        self.group = group or C._get_default_group()
        self._grad_need_sync = True
        if self.group.nranks > 1:
            sync_params_buffers(layers, self.group)
        self._reducer = Reducer(layers.parameters(), self.group, int(comm_buffer_size * (1 << 20)),
                                int(last_comm_buffer_size * (1 << 20)), find_unused_parameters)

    def forward(self, *inputs, **kwargs):
        self._reducer.rebind()
        self._reducer.enabled = self._grad_need_sync
        return self._layers(*inputs, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._grad_need_sync
        self._grad_need_sync = False
        try:
            yield
        finally:
            self._grad_need_sync = prev

    def scale_loss(self, loss):
        return loss

    def apply_collective_grads(self):
        pass

    def state_dict(self, destination=None, include_sublayers=True, structured_name_prefix="", use_hook=True):
        return self._layers.state_dict(destination, include_sublayers, structured_name_prefix, use_hook)

    def set_state_dict(self, state_dict, use_structured_name=True):
        return self._layers.set_state_dict(state_dict, use_structured_name)

    set_dict = set_state_dict
    load_dict = set_state_dict

    def parameters(self, include_sublayers=True):
        return self._layers.parameters(include_sublayers)

    def named_parameters(self, prefix="", include_sublayers=True, remove_duplicate=True):
        return self._layers.named_parameters(prefix, include_sublayers, remove_duplicate)
