"""Group-sharded data parallelism, stages 1 / 2 / 3 (ZeRO-style).

Reference: python/paddle/distributed/sharding/group_sharded.py:50 ``group_sharded_parallel``
(levels ``os`` / ``os_g`` / ``p_g_os``), fleet/meta_parallel/sharding/group_sharded_stage3.py:85
(ForwardPreHooks :851 all-gather + prefetch, ForwardPostHooks :901 release, per-param full-grad
``all_reduce`` then slice :743-805), group_sharded_stage2.py:46, group_sharded_optimizer_stage2.py:53,
and save_group_sharded_model :199.

MI355X design:
  * parameters are grouped into *units* (each decoder layer / embedding / head), flattened into
    one padded flat buffer per unit; every rank owns a contiguous 1/N slice (bf16 param shard,
    fp32 master shard, fp32 moments, fp32 grad shard) — 288 GB HBM leaves room for generous
    unit sizes and prefetch;
  * stage 3: a unit is materialised by ONE ``all_gather_into_tensor`` of its flat shard into a
    flat buffer the parameters view (no per-param collectives); the next unit's gather is issued
    asynchronously before the current unit computes (RCCL runs on its own stream, so the xGMI
    transfer overlaps the GEMMs), in forward and in backward (triggered by a hook on the unit's
    output gradient);
  * gradients: ONE ``reduce_scatter_tensor`` (ReduceOp.AVG) of the unit's flat grad straight into
    the owned slice — not the reference's per-param full all-reduce + slice (half the bytes);
  * the optimizer steps only the owned slices with the fused multi-tensor AdamW kernel (one
    launch), global-norm clipping all-reduces one scalar;
  * stage 1/2 keep parameters replicated; after the sharded update each unit's slices are
    all-gathered back (one collective per unit).
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from ...framework.param import Parameter
from ...framework.tensor import Tensor
from ...nn.layer.common import LayerList
from ...nn.layer.layers import Layer
from .. import collective as C

_EMPTY = {}


def _empty(dtype, device):
    key = (dtype, device)
    if key not in _EMPTY:
        _EMPTY[key] = torch.empty(0, dtype=dtype, device=device)
    return _EMPTY[key]


def _find_units(model: Layer):
    """Units = children of LayerLists + other layers that own parameters directly."""
    units, claimed = [], set()

    def visit(layer, inside_unit):
        if isinstance(layer, LayerList):
            for child in layer._sub_layers.values():
                if child is not None:
                    units.append(child)
                    for p in child.parameters():
                        claimed.add(id(p))
            return
        own = [p for p in layer._parameters.values() if p is not None and id(p) not in claimed]
        if own and not inside_unit:
            units.append(layer)
            for p in layer.parameters():
                claimed.add(id(p))
            return
        for child in layer._sub_layers.values():
            if child is not None:
                visit(child, inside_unit)

    visit(model, False)
    # anything still unclaimed (e.g. params registered on a container) forms a root unit
    rest = [p for p in model.parameters() if id(p) not in claimed]
    return units, rest


class _Unit:
    def __init__(self, idx, layer, params, group, stage, decay_fn, lr_ratio_fn):
        self.idx = idx
        self.layer = layer
        self.params = [p for p in params if not p.stop_gradient] + [p for p in params if p.stop_gradient]
        self.group = group
        self.stage = stage
        self.N = group.nranks
        self.rank = group.rank
        p0 = self.params[0]._t
        self.dtype, self.device = p0.dtype, p0.device
        self.numels = [p._t.numel() for p in self.params]
        self.shapes = [tuple(p._t.shape) for p in self.params]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n
        self.total = off
        self.padded = int(math.ceil(off / self.N)) * self.N
        self.S = self.padded // self.N
        flat = torch.zeros(self.padded, dtype=self.dtype, device=self.device)
        for p, o, n in zip(self.params, self.offsets, self.numels):
            flat[o:o + n].copy_(p._t.detach().reshape(-1))
        lo = self.rank * self.S
        self.shard = flat[lo:lo + self.S].clone()
        self.master = self.shard.float().clone() if self.dtype in (torch.bfloat16, torch.float16) else None
        self.grad_shard = torch.zeros(self.S, dtype=torch.float32, device=self.device)
        self.grad_clean = True   # grad_shard logically zero (next accumulate overwrites instead of adding)
        self.full = None
        self.work = None
        self.rs_work = None
        self.rs_buf = None
        self.flat_grad = None
        self.ready = 0
        self.n_trainable = sum(1 for p in self.params if not p.stop_gradient)
        self.bw_gathered = False
        # optimizer pieces: (param, shard offset, length) for every param overlapping my slice
        self.pieces = []
        for p, o, n in zip(self.params, self.offsets, self.numels):
            a, b = max(o, lo), min(o + n, lo + self.S)
            if a < b and not p.stop_gradient:
                self.pieces.append((p, a - lo, b - a, decay_fn(p), lr_ratio_fn(p)))
        if stage == 3:
            self.full = flat
            self._bind(flat)
            self.release()
        else:
            self.full = flat
            self._bind(flat)

    # ------------------------------------------------------------ materialisation
    def _bind(self, flat):
        for p, o, n, s in zip(self.params, self.offsets, self.numels, self.shapes):
            p._t.data = flat[o:o + n].view(s)

    def gather(self, async_op=True):
        if self.full is not None or self.work is not None:
            return
        if self.N == 1:
            # the single shard IS the full flat buffer: bind the parameters to it, no copy
            self.full = self.shard
            self._bind(self.shard)
            return
        buf = torch.empty(self.padded, dtype=self.dtype, device=self.device)
        self.work = dist.all_gather_into_tensor(buf, self.shard, group=self.group.pg, async_op=async_op)
        self._pending = buf
        if not async_op:
            self.work = None
            self.full = buf
            self._bind(buf)

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
            self.full = self._pending
            self._pending = None
            self._bind(self.full)
        elif self.full is None:
            self.gather(async_op=False)

    def release(self):
        if self.stage != 3:
            return
        for p in self.params:
            p._t.data = _empty(self.dtype, self.device)
        self.full = None

    # ------------------------------------------------------------ gradients
    def on_param_grad(self):
        self.ready += 1
        if self.ready == self.n_trainable:
            self.reduce_grads()

    def _accumulate(self, g):
        """grad_shard (fp32) += g, or = g when the shard was lazily cleared (no zero-fill pass)."""
        if self.grad_clean:
            self.grad_shard.copy_(g)
            self.grad_clean = False
        else:
            self.grad_shard.add_(g)

    def reduce_grads(self):
        # one flat buffer per unit; only the gaps (missing grads, padding tail) are zero-filled
        flat = torch.empty(self.padded, dtype=self.dtype, device=self.device)
        if self.padded > self.total:
            flat[self.total:].zero_()
        for p, o, n in zip(self.params, self.offsets, self.numels):
            g = p._t.grad
            if g is not None:
                flat[o:o + n].copy_(g.reshape(-1))
                p._t.grad = None
            else:
                flat[o:o + n].zero_()
        if self.N == 1:
            self._accumulate(flat[: self.S])
            self.flat_grad = None
        else:
            out = torch.empty(self.S, dtype=self.dtype, device=self.device)
            op = dist.ReduceOp.AVG if self.group.backend == "nccl" else dist.ReduceOp.SUM
            self.rs_work = dist.reduce_scatter_tensor(out, flat, op=op, group=self.group.pg, async_op=True)
            self.rs_buf = out
            self.flat_grad = flat  # keep alive until the collective completes
        self.release()

    def finish_grads(self):
        if self.ready < self.n_trainable and self.ready > 0:
            self.reduce_grads()
        if self.rs_work is not None:
            self.rs_work.wait()
            g = self.rs_buf
            if self.group.backend != "nccl":
                g = g.float().div_(self.N)
            self._accumulate(g)
            self.rs_work = None
            self.rs_buf = None
            self.flat_grad = None
        self.ready = 0
        self.bw_gathered = False

    # ------------------------------------------------------------ after the optimizer
    def refresh_params(self):
        """Stage 1/2: all-gather the updated slices into the replicated parameters."""
        if self.stage == 3:
            return
        if self.N == 1:
            self.full[: self.S].copy_(self.shard)
            return
        dist.all_gather_into_tensor(self.full, self.shard, group=self.group.pg)


class GroupShardedModel(Layer):
    """Wraps a Layer; owns the units and the forward/backward gather/release hooks."""

    def __init__(self, layer, group, stage, optimizer, prefetch=True):
        super().__init__()
        self._layer = layer
        self._group = group
        self._stage = stage
        self._prefetch = prefetch
        decay_fn = getattr(optimizer, "_decay_of", lambda p: 0.0)
        lr_fn = getattr(optimizer, "_lr_ratio_of", lambda p: 1.0)
        unit_layers, rest = _find_units(layer)
        self._units = []
        for i, l in enumerate(unit_layers):
            ps = l.parameters()
            if ps:
                self._units.append(_Unit(len(self._units), l, ps, group, stage, decay_fn, lr_fn))
        if rest:
            self._units.append(_Unit(len(self._units), None, rest, group, stage, decay_fn, lr_fn))
        self._order = []       # unit call order in forward
        self._by_layer = {id(u.layer): u for u in self._units if u.layer is not None}
        self._cb_queued = False
        self._hooks = []
        for u in self._units:
            if u.layer is not None:
                self._hooks.append(u.layer.register_forward_pre_hook(self._make_pre(u)))
                self._hooks.append(u.layer.register_forward_post_hook(self._make_post(u)))
            for p in u.params:
                if not p.stop_gradient:
                    self._hooks.append(p._t.register_post_accumulate_grad_hook(self._make_grad_hook(u)))

    # ------------------------------------------------------------ hooks
    def _make_pre(self, u):
        def pre(layer, inputs):
            if self._stage == 3:
                u.wait()
                if u.idx not in self._order_set():
                    self._order.append(u.idx)
                if self._prefetch:
                    nxt = self._next_in_order(u.idx, +1)
                    if nxt is not None:
                        nxt.gather(async_op=True)
            return None

        return pre

    def _order_set(self):
        return set(self._order)

    def _next_in_order(self, idx, step):
        if idx not in self._order:
            return None
        i = self._order.index(idx) + step
        if 0 <= i < len(self._order):
            return self._units[self._order[i]]
        return None

    def _make_post(self, u):
        def post(layer, inputs, outputs):
            if self._stage == 3 and torch.is_grad_enabled():
                outs = outputs if isinstance(outputs, (tuple, list)) else [outputs]
                hooked = False
                for o in outs:
                    t = o._t if isinstance(o, Tensor) else o
                    if isinstance(t, torch.Tensor) and t.requires_grad:
                        t.register_hook(self._make_bw_pre(u))
                        hooked = True
                if hooked:
                    u.release()
            elif self._stage == 3:
                u.release()
            return None

        return post

    def _make_bw_pre(self, u):
        def hook(grad):
            if not u.bw_gathered:
                u.bw_gathered = True
                self._queue_cb()
                u.wait()
                if self._prefetch:
                    prv = self._next_in_order(u.idx, -1)
                    if prv is not None and not prv.bw_gathered:
                        prv.gather(async_op=True)
            return None

        return hook

    def _make_grad_hook(self, u):
        def hook(t):
            self._queue_cb()
            if self._stage == 3 and u.full is None:
                u.wait()
            u.on_param_grad()

        return hook

    def _queue_cb(self):
        if not self._cb_queued:
            self._cb_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize_backward)

    def _finalize_backward(self):
        self._cb_queued = False
        for u in self._units:
            u.finish_grads()
            if self._stage == 3:
                u.release()

    # ------------------------------------------------------------ module API
    def forward(self, *args, **kwargs):
        if self._stage == 3:
            for u in self._units:
                if u.layer is None:
                    u.wait()  # root unit: keep gathered for the whole step
        return self._layer(*args, **kwargs)

    def gather_all(self):
        for u in self._units:
            u.wait()

    def release_all(self):
        for u in self._units:
            u.release()

    def state_dict(self, destination=None, include_sublayers=True, structured_name_prefix="", use_hook=True):
        """Full (gathered) parameters, like save_group_sharded_model."""
        self.gather_all()
        sd = self._layer.state_dict(destination, include_sublayers, structured_name_prefix, use_hook)
        sd = {k: Tensor._wrap(v._t.detach().clone()) for k, v in sd.items()}
        if self._stage == 3:
            self.release_all()
        return sd

    def set_state_dict(self, state_dict, use_structured_name=True):
        self.gather_all()
        r = self._layer.set_state_dict(state_dict, use_structured_name)
        for u in self._units:
            lo = u.rank * u.S
            u.shard.copy_(u.full[lo:lo + u.S])
            if u.master is not None:
                u.master.copy_(u.shard.float())
        if self._stage == 3:
            self.release_all()
        return r

    def parameters(self, include_sublayers=True):
        return self._layer.parameters(include_sublayers)


class GroupShardedOptimizer:
    """Steps the owned slices with the fused multi-tensor AdamW (or the wrapped optimizer's math)."""

    def __init__(self, optimizer, model: GroupShardedModel):
        self._inner = optimizer
        self._model = model
        self._table = None
        self._m = {}
        self._v = {}

    @property
    def _parameter_list(self):
        return self._inner._parameter_list

    def get_lr(self):
        return self._inner.get_lr()

    def set_lr(self, v):
        self._inner.set_lr(v)

    def _pieces(self):
        out = []
        for u in self._model._units:
            for (p, o, n, dec, lrr) in u.pieces:
                out.append((u, p, o, n, dec, lrr))
        return out

    def _materialize_grads(self):
        for u in self._model._units:
            if u.grad_clean:      # no gradient reached this unit since clear_grad: it is zero
                u.grad_shard.zero_()
                u.grad_clean = False

    def _global_sq_norm(self):
        sq = torch.zeros(1, dtype=torch.float32, device=self._model._units[0].device)
        for u in self._model._units:
            sq += torch.dot(u.grad_shard, u.grad_shard)
        g = self._model._group
        if g.nranks > 1:
            dist.all_reduce(sq, group=g.pg)
        return sq

    @torch.no_grad()
    def step(self):
        inner = self._inner
        inner._step += 1
        self._materialize_grads()
        clip = inner._grad_clip
        coef = None
        if clip is not None and hasattr(clip, "clip_norm"):
            norm = torch.sqrt(self._global_sq_norm())
            coef = torch.clamp(clip.clip_norm / torch.clamp(norm, min=1e-6), max=1.0).float().reshape(1)
        lr = inner.get_lr()
        b1, b2 = getattr(inner, "_beta1", 0.9), getattr(inner, "_beta2", 0.999)
        eps = getattr(inner, "_epsilon", 1e-8)
        bc1, bc2 = 1 - b1 ** inner._step, 1 - b2 ** inner._step
        pieces = self._pieces()
        from ...ops import _native as N

        dev = self._model._units[0].device
        if self._table is None:
            params, grads, ms, vs, masters, lrrs, decs = [], [], [], [], [], [], []
            for (u, p, o, n, dec, lrr) in pieces:
                params.append(u.shard[o:o + n])
                grads.append(u.grad_shard[o:o + n])
                key = (u.idx, o)
                self._m[key] = torch.zeros(n, dtype=torch.float32, device=dev)
                self._v[key] = torch.zeros(n, dtype=torch.float32, device=dev)
                ms.append(self._m[key])
                vs.append(self._v[key])
                masters.append(None if u.master is None else u.master[o:o + n])
                lrrs.append(lrr)
                decs.append(dec)
            use_native = dev.type == "cuda" and N.available() and all(
                t.data_ptr() % 16 == 0 for t in params + grads + [m for m in masters if m is not None])
            if use_native and params:
                from ...optimizer.multi_tensor import MultiTensorTable

                groups = {}
                for i in range(len(params)):
                    groups.setdefault((params[i].dtype, masters[i] is not None), []).append(i)
                tabs = []
                for _, idx in groups.items():
                    tabs.append(MultiTensorTable([params[i] for i in idx], [grads[i] for i in idx],
                                                 [ms[i] for i in idx], [vs[i] for i in idx],
                                                 [masters[i] for i in idx] if masters[idx[0]] is not None else None,
                                                 [lrrs[i] for i in idx], [decs[i] for i in idx]))
                self._table = ("native", tabs)
            else:
                self._table = ("ref", list(zip(params, grads, ms, vs, masters, lrrs, decs)))
        kind, tabs = self._table
        if kind == "native":
            # clip coefficient folded into the fused AdamW pass (device scalar, no extra grad pass)
            for t in tabs:
                t.adamw(lr, b1, b2, eps, bc1, bc2, getattr(inner, "_found_inf", None), coef)
        else:
            if coef is not None:
                for u in self._model._units:
                    u.grad_shard.mul_(coef)
            for (p, g, m, v, mw, lrr, dec) in tabs:
                m.mul_(b1).add_(g, alpha=1 - b1)
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                tgt = mw if mw is not None else p
                lr_t = lr * lrr
                upd = tgt.float() * (1 - lr_t * dec) - (lr_t / bc1) * m / (v.sqrt() / math.sqrt(bc2) + eps)
                tgt.copy_(upd.to(tgt.dtype))
                if mw is not None:
                    p.copy_(mw)
        for u in self._model._units:
            u.refresh_params()

    def clear_grad(self, set_to_zero=True):
        for u in self._model._units:
            if set_to_zero:
                u.grad_clean = True  # lazy zero: the next reduce overwrites the shard
            else:
                u.grad_shard.zero_()
            for p in u.params:
                p._t.grad = None

    clear_gradients = clear_grad

    def state_dict(self):
        sd = {"step": self._inner._step}
        for k in self._m:
            sd[f"unit{k[0]}_off{k[1]}_moment1"] = Tensor._wrap(self._m[k])
            sd[f"unit{k[0]}_off{k[1]}_moment2"] = Tensor._wrap(self._v[k])
        for u in self._model._units:
            if u.master is not None:
                sd[f"unit{u.idx}_master"] = Tensor._wrap(u.master)
        return sd

    def set_state_dict(self, sd):
        self._inner._step = int(sd.get("step", 0))
        for k in list(self._m):
            a = sd.get(f"unit{k[0]}_off{k[1]}_moment1")
            if a is not None:
                self._m[k].copy_(a._t)
                self._v[k].copy_(sd[f"unit{k[0]}_off{k[1]}_moment2"]._t)

    def minimize(self, loss, *a, **k):
        self.step()


def group_sharded_parallel(model, optimizer, level, scaler=None, group=None, offload=False, sync_buffers=False,
                           buffer_max_size=2 ** 23, segment_size=2 ** 20, sync_comm=False, dp_group=None,
                           exclude_layer=None):
    """level: 'os' (stage 1), 'os_g' (stage 2), 'p_g_os' (stage 3)."""
    stage = {"os": 1, "os_g": 2, "p_g_os": 3}[level]
    g = group or C._get_default_group()
    if g.nranks > 1:
        from ..parallel import sync_params_buffers

        sync_params_buffers(model, g)
    sm = GroupShardedModel(model, g, stage, optimizer, prefetch=not sync_comm)
    so = GroupShardedOptimizer(optimizer, sm)
    return sm, so, scaler


def save_group_sharded_model(model, output, optimizer=None):
    import os

    from ...framework.io import save

    os.makedirs(output, exist_ok=True)
    sd = model.state_dict()
    if C.get_rank(model._group if isinstance(model, GroupShardedModel) else None) == 0:
        save(sd, os.path.join(output, "model.pdmodel"))
        if optimizer is not None:
            save(optimizer.state_dict(), os.path.join(output, "model.pdopt"))
