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


def force_comm():
    """PADDLE2_AMD_STAGE3_FORCE_COMM=1: a 1-rank sharding group still takes the N > 1 code path — real
    all_gather_into_tensor / reduce_scatter_tensor on the group's process group (comm stream included), the fp32
    flat-gradient pool, prefetch and retire_rs — so one GPU exercises what an 8-GPU node runs (collective.py then
    initialises a 1-rank process group)."""
    import os

    return os.environ.get("PADDLE2_AMD_STAGE3_FORCE_COMM", "0") == "1"


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
    # parameters the model also reads outside their own layer (tied input/output embeddings: GPT's logits use
    # word_embeddings.weight) cannot be released after that layer's forward: their layers join the root unit,
    # which stays gathered for the whole step
    shared = getattr(model, "_sharding_root_params", None)
    shared = shared() if callable(shared) else (shared or [])
    if shared:
        sid = {id(p) for p in shared}
        units = [u for u in units if not any(id(p) in sid for p in u.parameters())]
        claimed = {id(p) for u in units for p in u.parameters()}
    # anything still unclaimed (e.g. params registered on a container) forms a root unit
    rest = [p for p in model.parameters() if id(p) not in claimed]
    return units, rest


def _excluded_params(model, exclude_layer):
    """ids of the parameters of every sublayer named in ``exclude_layer`` (class names or id(layer))."""
    if not exclude_layer:
        return set()
    names = {e for e in exclude_layer if isinstance(e, str)}
    ids = {e for e in exclude_layer if isinstance(e, int)}
    out = set()
    for _, sub in model.named_sublayers(include_self=True):
        if type(sub).__name__ in names or id(sub) in ids:
            out.update(id(p) for p in sub.parameters())
    return out


class _Unit:
    def __init__(self, idx, layer, params, group, stage, decay_fn, lr_ratio_fn):
        self.idx = idx
        self.layer = layer
        self.params = [p for p in params if not p.stop_gradient] + [p for p in params if p.stop_gradient]
        self.group = group
        self.stage = stage
        self.N = group.nranks
        self.rank = group.rank
        # collectives on (N > 1, or forced on a 1-rank group that has a process group): see force_comm
        self.comm = self.N > 1 or (force_comm() and getattr(group, "pg", None) is not None)
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
        self.written = set()
        self.flat32 = None
        self.rs_add = False
        self.model = None
        self.n_trainable = sum(1 for p in self.params if not p.stop_gradient)
        self.bw_gathered = False
        self.n_gathers = 0   # all-gathers issued (the comm path), for tests and the comm model
        for i, p in enumerate(self.params):
            if not p.stop_gradient and p._t.dim() == 2:
                p._t._p2_gt = (self, i)  # weight-gradient GEMMs write straight into the fp32 target
            elif not p.stop_gradient and p._t.dim() == 1 and not getattr(p, "sequence_parallel", False):
                p._t._p2_bt = (self, i)  # bias / norm-weight column sums likewise (ops.torch_ops.main_slot)
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
        if not self.comm:
            # the single shard IS the full flat buffer: bind the parameters to it, no copy
            self.full = self.shard
            self._bind(self.shard)
            return
        buf = torch.empty(self.padded, dtype=self.dtype, device=self.device)
        self.n_gathers += 1
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
    # Every trainable parameter's gradient lands ONCE per backward in an fp32 target: a view of the
    # owned grad shard (N == 1: the shard is the whole flat unit) or of a per-backward flat fp32 unit
    # buffer (N > 1) that one reduce_scatter(SUM) then folds into the owned shard.  Linear weights are
    # written directly by their weight-gradient GEMM (fp32 accumulate, ops.torch_ops._main_grad_accumulate);
    # the rest (norm weights, embeddings) arrive through autograd and are copied in by the grad hook.
    # The same SUM + fp32 1/N scale runs on RCCL and gloo (the scale is folded into the optimizer).
    def _flat(self):
        """This unit's fp32 flat gradient buffer for the running backward (N > 1), from the model's bounded pool."""
        if self.flat32 is None:
            self.flat32 = self.model._acquire_flat(self) if self.model is not None else \
                torch.empty(self.padded, dtype=torch.float32, device=self.device)
        return self.flat32

    def grad_target(self, i):
        """-> (fp32 view of param i's gradient slot, beta): beta 0 = overwrite, 1 = accumulate."""
        o, n, shp = self.offsets[i], self.numels[i], self.shapes[i]
        if not self.comm:
            buf = self.grad_shard
            beta = 0 if (self.grad_clean and i not in self.written) else 1
        else:
            buf = self._flat()
            beta = 0 if i not in self.written else 1
        return buf[o:o + n].view(shp), beta

    def param_grad_done(self, i):
        self.written.add(i)
        if self.model is not None:
            self.model._queue_cb()
        if len(self.written) == self.n_trainable:
            self.reduce_grads()

    def on_param_grad(self, i):
        """autograd-path gradient (p.grad) -> fp32 target, then drop p.grad."""
        p = self.params[i]
        g = p._t.grad
        if g is None:
            return
        spg = self.model._sp_group if self.model is not None else None
        if spg is not None and getattr(p, "sequence_parallel", False):
            # a sequence-parallel parameter (norm weights / row-linear bias inside TP + SP) saw only this rank's
            # sequence shard: its gradient is the sum over the mp group (HybridParallelOptimizer's SP sync, done
            # here because stage 3 consumes the gradient before any optimizer hook runs)
            dist.all_reduce(g, group=spg.pg)
        view, beta = self.grad_target(i)
        if beta == 0:
            view.copy_(g.reshape(view.shape))
        else:
            view.add_(g.reshape(view.shape))
        p._t.grad = None
        self.param_grad_done(i)

    def _zero_unwritten(self, buf):
        for i, (o, n) in enumerate(zip(self.offsets, self.numels)):
            if i not in self.written:
                buf[o:o + n].zero_()
        if self.padded > self.total:
            buf[self.total:].zero_()

    def reduce_grads(self):
        if not self.comm:
            if self.grad_clean:
                self._zero_unwritten(self.grad_shard)
                self.grad_clean = False
        else:
            flat = self._flat()
            self._zero_unwritten(flat)
            if self.grad_clean:
                out, self.rs_add = self.grad_shard, False
            else:
                out, self.rs_add = torch.empty(self.S, dtype=torch.float32, device=self.device), True
            self.rs_work = dist.reduce_scatter_tensor(out, flat, op=dist.ReduceOp.SUM, group=self.group.pg,
                                                      async_op=True)
            self.rs_buf = out
            self.flat_grad = flat  # keep alive until the collective completes (then back to the pool)
            self.flat32 = None
            self.grad_clean = False
            if self.model is not None:
                self.model._rs_issued(self)
        self.written = set()
        self.release()

    def retire_rs(self):
        """Complete this unit's reduce-scatter: fold an accumulation step's partial into the owned fp32 shard and
        hand the flat buffer back; -> the freed flat buffer (or None)."""
        flat = None
        if self.rs_work is not None:
            self.rs_work.wait()
            if self.rs_add:
                self.grad_shard.add_(self.rs_buf)
            self.rs_work = None
            self.rs_buf = None
            flat, self.flat_grad = self.flat_grad, None
        return flat

    def finish_grads(self):
        if self.written:
            self.reduce_grads()
        if self.model is not None:
            self.model._retire_all()
        else:
            self.retire_rs()
        self.bw_gathered = False

    # ------------------------------------------------------------ after the optimizer
    def refresh_params(self):
        """Stage 1/2: all-gather the updated slices into the replicated parameters."""
        if self.stage == 3:
            return
        if not self.comm:
            self.full[: self.S].copy_(self.shard)
            return
        dist.all_gather_into_tensor(self.full, self.shard, group=self.group.pg)


class GroupShardedModel(Layer):
    """Wraps a Layer; owns the units and the forward/backward gather/release hooks."""

    def __init__(self, layer, group, stage, optimizer, prefetch=True, exclude_layer=None):
        super().__init__()
        self._layer = layer
        self._group = group
        self._stage = stage
        self._prefetch = prefetch
        decay_fn = getattr(optimizer, "_decay_of", lambda p: 0.0)
        lr_fn = getattr(optimizer, "_lr_ratio_of", lambda p: 1.0)
        excluded = _excluded_params(layer, exclude_layer) if stage == 3 else set()
        unit_layers, rest = _find_units(layer)
        self._units = []
        for i, l in enumerate(unit_layers):
            ps = [p for p in l.parameters() if id(p) not in excluded]
            if ps:
                self._units.append(_Unit(len(self._units), l, ps, group, stage, decay_fn, lr_fn))
        rest = [p for p in rest if id(p) not in excluded]
        if rest:
            self._units.append(_Unit(len(self._units), None, rest, group, stage, decay_fn, lr_fn))
        if excluded:
            # exclude_layer (group_sharded_stage3.py:98): those parameters stay whole on every rank; their
            # gradients and optimizer state are still reduce-scattered / sharded (one replicated unit)
            ps = [p for p in layer.parameters() if id(p) in excluded]
            self._units.append(_Unit(len(self._units), None, ps, group, 2, decay_fn, lr_fn))
        # tensor parallelism inside the sharded model: _mp_group (the clip norm sums the TP-sharded parameters over
        # it); _sp_group (the same group when sequence-parallel parameters exist: their grads are summed over it)
        self._mp_group = self._sp_group = None
        try:
            from .. import fleet

            hcg = fleet.get_hybrid_communicate_group()
            if hcg is not None and hcg.get_model_parallel_world_size() > 1:
                self._mp_group = hcg.get_model_parallel_group()
                if any(getattr(p, "sequence_parallel", False) for p in layer.parameters()):
                    self._sp_group = self._mp_group
        except Exception:   # noqa: BLE001 - no fleet: plain sharding
            self._mp_group = self._sp_group = None
        self._order = []       # unit call order in forward
        self._order_done = False  # a full forward has recorded _order (the last unit stays gathered for backward)
        self._by_layer = {id(u.layer): u for u in self._units if u.layer is not None}
        self._cb_queued = False
        self._hooks = []
        # stage-3 N > 1 gradient buffers: at most MAX_LIVE_FLAT fp32 flat unit buffers exist at a time (the ones
        # being written + the ones whose reduce-scatter is in flight); acquiring one more first retires the oldest
        # reduce-scatter (group_sharded_stage3.py:743-805 keeps one full fp32 grad per PARAM alive instead)
        self.max_live_flat = 2
        self._rs_queue = []       # units with a reduce-scatter in flight, oldest first
        self._flat_pool = {}      # numel -> [free fp32 buffers]
        self._live_flat = 0
        self.peak_live_flat = 0
        self.prefetch_depth = 2
        self.keep_gathered = self._keep_gathered_policy()
        # units left gathered by a grad-enabled forward for the backward (the turn unit, or all with keep_gathered);
        # cleared by _finalize_backward — a forward that never gets a backward (eval without no_grad) would
        # otherwise hold them gathered for good, so the next forward releases whatever is still listed
        self._kept = set()
        for u in self._units:
            if u.layer is not None:
                self._hooks.append(u.layer.register_forward_pre_hook(self._make_pre(u)))
                self._hooks.append(u.layer.register_forward_post_hook(self._make_post(u)))
            u.model = self
            for i, p in enumerate(u.params):
                if not p.stop_gradient:
                    self._hooks.append(p._t.register_post_accumulate_grad_hook(self._make_grad_hook(u, i)))

    def _keep_gathered_policy(self):
        """Stage 3 at N > 1 keeps every unit gathered from its forward to its backward (no backward re-gather: one
        of the step's three collectives per unit) when the whole bf16 model is a small share of HBM — on MI355X
        the 288 GB card holds Llama-2-7B's 13.5 GB of gathered parameters beside a ~170 GiB per-rank peak at
        N = 8 (profiles/r5_stage3_force_comm.md).  PADDLE2_AMD_STAGE3_KEEP_GATHERED = auto | 1 | 0."""
        import os

        mode = os.environ.get("PADDLE2_AMD_STAGE3_KEEP_GATHERED", "auto")
        if self._stage != 3 or mode == "0":
            return False
        comm = [u for u in self._units if u.comm]
        if not comm:
            return False
        if mode == "1":
            return True
        if force_comm() or self._group.nranks <= 1:
            return False   # the 1-GPU rehearsal holds the whole optimizer state: no room for a second copy
        dev = comm[0].device
        if dev.type != "cuda":
            return False
        full = sum(u.padded * torch.tensor([], dtype=u.dtype).element_size() for u in comm)
        return full <= 0.08 * torch.cuda.get_device_properties(dev).total_memory

    # ------------------------------------------------------------ bounded fp32 grad buffers (N > 1)
    def _acquire_flat(self, unit):
        while self._live_flat >= self.max_live_flat and self._rs_queue:
            self._retire_oldest()
        pool = self._flat_pool.get(unit.padded)
        buf = pool.pop() if pool else torch.empty(unit.padded, dtype=torch.float32, device=unit.device)
        self._live_flat += 1
        self.peak_live_flat = max(self.peak_live_flat, self._live_flat)
        return buf

    def _release_flat(self, buf):
        if buf is not None:
            self._flat_pool.setdefault(buf.numel(), []).append(buf)
            self._live_flat -= 1

    def _rs_issued(self, unit):
        self._rs_queue.append(unit)

    def _retire_oldest(self):
        u = self._rs_queue.pop(0)
        self._release_flat(u.retire_rs())

    def _retire_all(self):
        while self._rs_queue:
            self._retire_oldest()

    def release_grad_pool(self):
        """Free the recycled fp32 flat buffers (they are kept across steps by default)."""
        self._flat_pool.clear()

    # ------------------------------------------------------------ hooks
    def _make_pre(self, u):
        def pre(layer, inputs):
            if self._stage == 3:
                u.wait()
                if u.idx not in self._order_set():
                    self._order.append(u.idx)
                if self._prefetch:
                    # prefetch depth 2: the next two units' all-gathers are in flight while this one computes
                    for d in range(1, self.prefetch_depth + 1):
                        nxt = self._next_in_order(u.idx, +d)
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
                # the last unit of the forward is the first of the backward: keep it gathered across the turn
                # (every unit, with keep_gathered: the backward then issues no all-gather at all)
                last = self._order_done and self._order and u.idx == self._order[-1]
                if hooked and not last and not self.keep_gathered:
                    u.release()
                elif hooked:
                    self._kept.add(u.idx)
                else:
                    u.release()   # no output needs a gradient: no backward will come for this unit
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
                    for d in range(1, self.prefetch_depth + 1):
                        prv = self._next_in_order(u.idx, -d)
                        if prv is not None and not prv.bw_gathered:
                            prv.gather(async_op=True)
            return None

        return hook

    def _make_grad_hook(self, u, i):
        def hook(t):
            self._queue_cb()
            u.on_param_grad(i)

        return hook

    def _queue_cb(self):
        if not self._cb_queued:
            self._cb_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize_backward)

    def _finalize_backward(self):
        self._cb_queued = False
        self._kept.clear()
        for u in self._units:
            u.finish_grads()
            if self._stage == 3:
                u.release()
        self._retire_all()
        self._order_done = True

    # ------------------------------------------------------------ module API
    def forward(self, *args, **kwargs):
        if self._stage == 3:
            if self._kept:
                # kept gathered by the previous forward, whose backward never ran: release before re-gathering
                for i in sorted(self._kept):
                    self._units[i].release()
                self._kept.clear()
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
    """Steps the owned slices with the fused multi-tensor AdamW (or the wrapped optimizer's math).

    Optimizer state per unit: fp32 moments (and the fp32 master of 16-bit params) for the owned slice
    only, as flat shard-sized buffers the per-parameter pieces view.  ``offload=True``
    (group_sharded_stage3.py:98 ``offload``): master weights and moments live in pinned host memory and
    the AdamW update of the owned slice runs on the CPU; only the fp32 grad shard goes down and the
    updated 16-bit param shard comes back up each step.

    ``state_dict()`` is the plain optimizer's per-parameter layout (``{name}_moment1_0``,
    ``{name}_moment2_0``, ``{name}_beta{1,2}_pow_acc_0``, ``master_weights``, ``LR_Scheduler``) with
    full, unsharded tensors, so a checkpoint reloads at any sharding degree and into an unsharded run
    (and vice versa)."""

    def __init__(self, optimizer, model: GroupShardedModel, offload=False):
        self._inner = optimizer
        self._model = model
        self._offload = offload
        self._table = None
        self._state = {}   # unit idx -> (m, v, master)  flat, shard-sized

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

    def _unit_state(self, u):
        st = self._state.get(u.idx)
        if st is None:
            if self._offload:
                mk = lambda: torch.zeros(u.S, dtype=torch.float32).pin_memory() if torch.cuda.is_available() \
                    else torch.zeros(u.S, dtype=torch.float32)  # noqa: E731
                m, v = mk(), mk()
                master = mk()
                master.copy_(u.shard.float().cpu())
                u.master = None  # the device master is not kept when offloading
            else:
                m = torch.zeros(u.S, dtype=torch.float32, device=u.device)
                v = torch.zeros(u.S, dtype=torch.float32, device=u.device)
                master = u.master
            st = (m, v, master)
            self._state[u.idx] = st
        return st

    def _materialize_grads(self):
        for u in self._model._units:
            if u.grad_clean:      # no gradient reached this unit since clear_grad: it is zero
                u.grad_shard.zero_()
                u.grad_clean = False

    def _global_sq_norm(self):
        from ...ops import _native as N

        mpg = self._model._mp_group
        if mpg is not None:
            # TP inside: a TP-sharded parameter's norm is the sum over the mp group, a replicated one (norms, SP
            # parameters after their mp sum) counts once — every mp rank then clips with the same coefficient
            dev = self._model._units[0].device
            sq = torch.zeros(2, dtype=torch.float32, device=dev)
            for u in self._model._units:
                for (p, o, n, _, _) in u.pieces:
                    seg = u.grad_shard[o:o + n]
                    sq[0 if getattr(p, "is_distributed", False) else 1] += torch.dot(seg, seg)
            if self._model._units[0].comm:
                dist.all_reduce(sq, group=self._model._group.pg)
            sd = sq[:1].clone()
            dist.all_reduce(sd, group=mpg.pg)
            return sd + sq[1:]
        shards = [u.grad_shard for u in self._model._units]
        if shards[0].is_cuda and N.use_native(shards[0]) and all(g.dtype == shards[0].dtype for g in shards):
            # one multi-tensor launch over every unit's fp32 grad shard (csrc/kernels/optim.hip sqnorm_mt)
            key = tuple(g.data_ptr() for g in shards)
            if getattr(self, "_sq_key", None) != key:
                from ...optimizer.multi_tensor import MultiTensorTable

                self._sq_table, self._sq_key = MultiTensorTable.for_grads(shards), key
            sq = self._sq_table.sqnorm()
        else:
            sq = torch.zeros(1, dtype=torch.float32, device=self._model._units[0].device)
            for g in shards:
                sq += torch.dot(g, g)
        g = self._model._group
        if self._model._units[0].comm:
            dist.all_reduce(sq, group=g.pg)
        return sq

    def _build_table(self):
        from ...ops import _native as N

        params, grads, ms, vs, masters, lrrs, decs = [], [], [], [], [], [], []
        for (u, p, o, n, dec, lrr) in self._pieces():
            m, v, master = self._unit_state(u)
            params.append(u.shard[o:o + n])
            grads.append(u.grad_shard[o:o + n])
            ms.append(m[o:o + n])
            vs.append(v[o:o + n])
            masters.append(None if master is None else master[o:o + n])
            lrrs.append(lrr)
            decs.append(dec)
        dev = self._model._units[0].device
        if self._offload:
            return ("cpu", None)
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
            return ("native", tabs)
        return ("ref", list(zip(params, grads, ms, vs, masters, lrrs, decs)))

    @staticmethod
    def _adamw_ref(p, g, m, v, mw, lr_t, dec, b1, b2, eps, bc1, bc2):
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        tgt = mw if mw is not None else p
        upd = tgt.float() * (1 - lr_t * dec) - (lr_t / bc1) * m / (v.sqrt() / math.sqrt(bc2) + eps)
        tgt.copy_(upd.to(tgt.dtype))
        if mw is not None:
            p.copy_(mw)

    @torch.no_grad()
    def step(self):
        inner = self._inner
        inner._step += 1
        self._materialize_grads()
        clip = inner._grad_clip
        coef = None
        nr = self._model._group.nranks
        inv = 1.0 / nr  # grads were reduce-scattered with SUM: the mean's 1/N is folded in here
        if clip is not None and hasattr(clip, "clip_norm"):
            norm = torch.sqrt(self._global_sq_norm()) * inv
            coef = (torch.clamp(clip.clip_norm / torch.clamp(norm, min=1e-6), max=1.0) * inv).float().reshape(1)
        elif nr > 1:
            coef = torch.full((1,), inv, dtype=torch.float32, device=self._model._units[0].device)
        lr = inner.get_lr()
        b1, b2 = getattr(inner, "_beta1", 0.9), getattr(inner, "_beta2", 0.999)
        eps = getattr(inner, "_epsilon", 1e-8)
        bc1, bc2 = 1 - b1 ** inner._step, 1 - b2 ** inner._step
        if self._table is None:
            self._table = self._build_table()
        kind, tabs = self._table
        if kind == "native":
            # clip coefficient folded into the fused AdamW pass (device scalar, no extra grad pass)
            for t in tabs:
                t.adamw(lr, b1, b2, eps, bc1, bc2, getattr(inner, "_found_inf", None), coef)
        elif kind == "cpu":
            self._step_offload(lr, b1, b2, eps, bc1, bc2, coef)
        else:
            if coef is not None:
                for u in self._model._units:
                    u.grad_shard.mul_(coef)
            for (p, g, m, v, mw, lrr, dec) in tabs:
                self._adamw_ref(p, g, m, v, mw, lr * lrr, dec, b1, b2, eps, bc1, bc2)
        for u in self._model._units:
            u.refresh_params()

    def _step_offload(self, lr, b1, b2, eps, bc1, bc2, coef):
        """Owned-slice AdamW on the host: grad shard D2H, update the pinned fp32 master, 16-bit shard H2D."""
        c = None if coef is None else float(coef.reshape(-1)[0])
        for u in self._model._units:
            m, v, master = self._unit_state(u)
            g = u.grad_shard.to("cpu", non_blocking=False)
            if c is not None:
                g.mul_(c)
            for (p, o, n, dec, lrr) in u.pieces:
                self._adamw_ref(master[o:o + n], g[o:o + n], m[o:o + n], v[o:o + n], None, lr * lrr, dec,
                                b1, b2, eps, bc1, bc2)
            u.shard.copy_(master.to(u.shard.dtype), non_blocking=True)

    def clear_grad(self, set_to_zero=True):
        for u in self._model._units:
            if set_to_zero:
                u.grad_clean = True  # lazy zero: the next reduce overwrites the shard
            else:
                u.grad_shard.zero_()
            u.written = set()
            for p in u.params:
                p._t.grad = None

    clear_gradients = clear_grad

    # ------------------------------------------------------------ checkpoint (any sharding degree)
    def _gather_full(self, u, shard):
        """owned fp32 slice -> full padded flat (host), one all_gather per unit."""
        src = shard.to(u.device)
        if u.N == 1:
            return src.detach().cpu().clone()
        full = torch.empty(u.padded, dtype=src.dtype, device=u.device)
        dist.all_gather_into_tensor(full, src.contiguous(), group=u.group.pg)
        return full.cpu()

    def state_dict(self):
        from ...optimizer.lr import LRScheduler

        inner = self._inner
        sd = {}
        masters = {}
        for u in self._model._units:
            m, v, master = self._unit_state(u)
            fm, fv = self._gather_full(u, m), self._gather_full(u, v)
            fmw = self._gather_full(u, master) if master is not None else None
            for p, o, n, shp in zip(u.params, u.offsets, u.numels, u.shapes):
                if p.stop_gradient:
                    continue
                sd[f"{p.name}_moment1_0"] = Tensor._wrap(fm[o:o + n].view(shp).clone())
                sd[f"{p.name}_moment2_0"] = Tensor._wrap(fv[o:o + n].view(shp).clone())
                sd[f"{p.name}_beta1_pow_acc_0"] = Tensor._wrap(torch.tensor([getattr(inner, "_beta1", 0.9) ** inner._step]))
                sd[f"{p.name}_beta2_pow_acc_0"] = Tensor._wrap(torch.tensor([getattr(inner, "_beta2", 0.999) ** inner._step]))
                if fmw is not None:
                    masters[p.name] = Tensor._wrap(fmw[o:o + n].view(shp).clone())
        if masters:
            sd["master_weights"] = masters
        if isinstance(inner._learning_rate, LRScheduler):
            sd["LR_Scheduler"] = inner._learning_rate.state_dict()
        return sd

    def set_state_dict(self, sd):
        from ...optimizer.lr import LRScheduler

        inner = self._inner
        b1 = getattr(inner, "_beta1", 0.9)
        masters = sd.get("master_weights", {})
        for u in self._model._units:
            m, v, master = self._unit_state(u)
            lo = u.rank * u.S
            for (p, o, n, dec, lrr) in u.pieces:
                pi = next(i for i, q in enumerate(u.params) if q is p)
                po = o + lo - u.offsets[pi]  # offset of this piece inside the parameter
                for key, dst in ((f"{p.name}_moment1_0", m), (f"{p.name}_moment2_0", v)):
                    t = sd.get(key)
                    if t is not None:
                        tt = t._t if isinstance(t, Tensor) else torch.as_tensor(t)
                        dst[o:o + n].copy_(tt.reshape(-1)[po:po + n].to(dst.device, torch.float32))
                mw = masters.get(p.name)
                if mw is not None and master is not None:
                    tt = mw._t if isinstance(mw, Tensor) else torch.as_tensor(mw)
                    master[o:o + n].copy_(tt.reshape(-1)[po:po + n].to(master.device, torch.float32))
                bp = sd.get(f"{p.name}_beta1_pow_acc_0")
                if bp is not None:
                    val = float((bp._t if isinstance(bp, Tensor) else torch.as_tensor(bp)).reshape(-1)[0])
                    if 0 < val < 1:
                        inner._step = int(round(math.log(val) / math.log(b1)))
        if "step" in sd:
            inner._step = int(sd["step"])
        if "LR_Scheduler" in sd and isinstance(inner._learning_rate, LRScheduler):
            inner._learning_rate.set_state_dict(sd["LR_Scheduler"])

    def minimize(self, loss, *a, **k):
        self.step()


def group_sharded_parallel(model, optimizer, level, scaler=None, group=None, offload=False, sync_buffers=False,
                           buffer_max_size=2 ** 23, segment_size=2 ** 20, sync_comm=False, dp_group=None,
                           exclude_layer=None):
    """level: 'os' (stage 1), 'os_g' (stage 2), 'p_g_os' (stage 3).  ``offload``: optimizer state and
    update on the host (pinned memory).  ``exclude_layer``: class names / id(layer) whose parameters stay
    unsharded under stage 3 (reference python/paddle/distributed/sharding/group_sharded.py:50)."""
    stage = {"os": 1, "os_g": 2, "p_g_os": 3}[level]
    g = group or C._get_default_group()
    if g.nranks > 1:
        from ..parallel import sync_params_buffers

        sync_params_buffers(model, g)
    sm = GroupShardedModel(model, g, stage, optimizer, prefetch=not sync_comm, exclude_layer=exclude_layer)
    so = GroupShardedOptimizer(optimizer, sm, offload=offload)
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
