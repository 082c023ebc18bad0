"""Passes over a static auto-parallel ``dist_main_program`` (reference python/paddle/distributed/passes/
auto_parallel_amp.py, auto_parallel_data_parallel_optimization.py (fused + coalesced gradient all-reduce),
auto_parallel_gradient_merge.py, auto_parallel_recompute.py, auto_parallel_sharding.py (stage 1)).

Every pass rewrites ``DistMainProgram.program`` in place (a static Program: ops over VarRefs) and leaves a program
the framework's static ``Executor`` runs:

* ``amp_pass`` — ops of the white list (linear / matmul / mm / bmm / addmm / conv / einsum) read their floating
  inputs through ``cast`` ops to bf16 (the fp32 parameters stay the masters: the cast's backward returns their
  gradient in fp32) and their results are cast back for the fp32 rest of the program;
* ``fuse_allreduce_pass`` — the per-use gradient all-reduces of replicated parameters (``c_identity`` ops of the
  data-parallel plan) become identities, and ONE bucketed, coalesced all-reduce of the parameter gradients runs
  right after ``backward`` (buckets sized for xGMI rings: few, large collectives);
* ``gradient_merge_pass`` — the optimizer step runs every ``k`` executions on the gradients summed (or averaged)
  over them; the other executions only accumulate;
* ``recompute_pass`` — op ranges become one op that runs them under activation checkpointing (their intermediates
  are recomputed in backward instead of kept);
* ``sharding_pass`` (stage 1) — the optimizer state is sharded over a mesh dimension: each rank steps only the
  parameters it owns (its accumulators exist only for those) and broadcasts them to the others.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.utils._pytree as pytree

from .completion import op_key

AMP_WHITE = {"linear", "matmul", "mm", "bmm", "addmm", "conv2d", "conv1d", "einsum", "baddbmm"}


def _new_var(prog, shape, dtype):
    return prog.new_var(torch.empty(list(shape), dtype=dtype, device="meta"))


def _named(fn, name, **tags):
    fn.__name__ = fn.__qualname__ = name
    for k, v in tags.items():
        setattr(fn, k, v)
    return fn


# ------------------------------------------------------------------------------------------------ AMP
def amp_pass(dmp, dtype=torch.bfloat16, white=AMP_WHITE):
    """-> number of ops moved to ``dtype``."""
    from ....static.graph import Op, VarRef

    prog = dmp.program
    ops, n = [], 0
    cast_to = _named(lambda x: x.to(dtype), "cast", amp=True)
    cast_back = _named(lambda x: x.float(), "cast", amp=True)
    for op in prog.ops:
        if op.kind not in ("torch", "native") or op_key(op) not in white:
            ops.append(op)
            continue
        leaves, spec = pytree.tree_flatten((op.args, op.kwargs))
        new = []
        for x in leaves:
            if isinstance(x, VarRef) and prog.vars[x.vid].dtype == torch.float32:
                v = _new_var(prog, prog.vars[x.vid].shape, dtype)
                ops.append(Op("torch", cast_to, (x,), {}, [v._vid]))
                new.append(VarRef(v._vid))
            elif isinstance(x, torch.Tensor) and x.dtype == torch.float32 and x.dim() > 0:
                v = _new_var(prog, x.shape, dtype)
                ops.append(Op("torch", cast_to, (x,), {}, [v._vid]))
                new.append(VarRef(v._vid))
            else:
                new.append(x)
        args, kwargs = pytree.tree_unflatten(new, spec)
        outs, backs = [], []
        for vid in op.outs:
            if vid is None or prog.vars[vid].dtype != torch.float32:
                outs.append(vid)
                continue
            v = _new_var(prog, prog.vars[vid].shape, dtype)
            outs.append(v._vid)
            backs.append(Op("torch", cast_back, (VarRef(v._vid),), {}, [vid]))
        ops.append(Op(op.kind, op.fn, tuple(args), kwargs, outs, dict(op.attrs)))
        ops.extend(backs)
        n += 1
    prog.ops = ops
    return n


# ------------------------------------------------------------------------------------------------ DP fusion
class _FusedAllReduce:
    """Sum the gradients of ``params`` over the mesh dims' groups in coalesced buckets of ``bucket_bytes``."""

    def __init__(self, params, mesh, dims, bucket_bytes):
        self.params, self.mesh, self.dims, self.bucket_bytes = params, mesh, dims, bucket_bytes
        self.calls = 0

    def buckets(self):
        out, cur, size = [], [], 0
        for p in self.params:
            nb = p.numel() * p.element_size()
            if cur and size + nb > self.bucket_bytes:
                out.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            out.append(cur)
        return out

    def __call__(self, env):
        from ..reshard import COMM_LOG

        for bucket in self.buckets():
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in bucket]
            flat = torch.cat([g.reshape(-1) for g in grads])
            for d in self.dims:
                dist.all_reduce(flat, group=self.mesh.get_group(d))
                COMM_LOG.append(("fused_all_reduce", d))
            off = 0
            for p, g in zip(bucket, grads):
                n = g.numel()
                p.grad = flat[off:off + n].view_as(g).clone()
                off += n
        self.calls += 1


def fuse_allreduce_pass(dmp, bucket_mb=256):
    """-> the fused all-reduce (its ``buckets()`` / ``calls`` for inspection), or None when nothing was fused."""
    from ....static.graph import Op

    prog = dmp.program
    params, dims = [], set()
    for op in prog.ops:
        fn = op.fn
        if op.kind == "torch" and getattr(fn, "comm", False) and fn.__name__ == "c_identity" and \
                isinstance(op.args[0], torch.Tensor) and op.args[0].requires_grad:
            p = op.args[0]
            dims |= set(getattr(fn, "dims", ()))
            if all(p is not q for q in params):
                params.append(p)
            op.fn = _named(lambda x: x, "identity")
    if not params:
        return None
    fused = _FusedAllReduce(params, dmp._dm, tuple(sorted(dims)), bucket_mb << 20)
    merge = [o for o in prog.ops if o.kind == "call" and "pre_step" in o.attrs]
    if merge:
        # gradient merge: the gradients accumulate over k micro-steps, so the sum runs once, at the k-step boundary
        # just before the optimizer step (reducing the accumulated grad every micro-step would re-add the sums of
        # earlier micro-steps world-fold)
        merge[0].attrs["pre_step"].append(fused)
        return fused
    i = next(k for k, o in enumerate(prog.ops) if o.kind == "backward")
    prog.ops.insert(i + 1, Op("call", None, (), {}, [], {"fn": fused, "name": "fused_allreduce_grads"}))
    return fused


# ------------------------------------------------------------------------------------------------ gradient merge
def gradient_merge_pass(dmp, k_steps, avg=True):
    """The ``optimize`` instruction steps every ``k_steps`` executions on the merged gradients."""
    from ....static.graph import Op

    prog = dmp.program
    # an already-applied fused DP all-reduce moves from behind the backward to the k-step boundary
    pre = [o.attrs["fn"] for o in prog.ops if o.kind == "call" and o.attrs.get("name") == "fused_allreduce_grads"]
    prog.ops = [o for o in prog.ops if not (o.kind == "call" and o.attrs.get("name") == "fused_allreduce_grads")]
    for i, op in enumerate(prog.ops):
        if op.kind != "optimize":
            continue
        opt = op.attrs["optimizer"]
        state = {"n": 0}

        def step(env, opt=opt, state=state, pre=pre):
            state["n"] += 1
            if state["n"] % k_steps:
                return
            for f in pre:   # gradient sums over the DP groups (fuse_allreduce_pass), once per merged step
                f(env)
            with torch.no_grad():
                if avg:
                    for p in opt._parameter_list:
                        if p._t.grad is not None:
                            p._t.grad.div_(k_steps)
                opt.step()
            opt.clear_grad(set_to_zero=False)

        prog.ops[i] = Op("call", None, (), {}, [], {"fn": step, "name": f"gradient_merge_k{k_steps}",
                                                     "optimizer": opt, "pre_step": pre})
    return prog


# ------------------------------------------------------------------------------------------------ recompute
def recompute_pass(dmp, segments):
    """``segments``: [(start, end)] indices into the program's ops (end exclusive, torch / native ops only).
    Each becomes one op running them under ``torch.utils.checkpoint``."""
    from ....static.graph import Op, VarRef

    prog = dmp.program
    ops = prog.ops
    for start, end in sorted(segments, reverse=True):
        seg = ops[start:end]
        assert all(o.kind in ("torch", "native") for o in seg), "recompute segments hold compute ops only"
        produced = {v for o in seg for v in o.outs if v is not None}
        reads = []
        for o in seg:
            for x in pytree.tree_leaves((o.args, o.kwargs)):
                if isinstance(x, VarRef) and x.vid not in produced and x.vid not in reads:
                    reads.append(x.vid)
        used_after = set()
        for o in ops[end:]:
            for x in pytree.tree_leaves((o.args, o.kwargs)):
                if isinstance(x, VarRef):
                    used_after.add(x.vid)
            for k in ("loss",):
                if k in o.attrs:
                    used_after.add(o.attrs[k])
        outs = [v for o in seg for v in o.outs if v is not None and v in used_after]
        outs = outs or [seg[-1].outs[-1]]

        def run(*vals, seg=seg, reads=tuple(reads), outs=tuple(outs)):
            env = dict(zip(reads, vals))

            def res(x):
                return env[x.vid] if isinstance(x, VarRef) else x

            for o in seg:
                r = o.fn(*pytree.tree_map(res, o.args), **pytree.tree_map(res, o.kwargs))
                for vid, val in zip(o.outs, pytree.tree_leaves(r)):
                    if vid is not None:
                        env[vid] = val
            return tuple(env[v] for v in outs)

        def fn(*vals, run=run):
            return torch.utils.checkpoint.checkpoint(run, *vals, use_reentrant=False)

        ops[start:end] = [Op("torch", _named(fn, f"recompute[{start}:{end}]", recompute=True),
                             tuple(VarRef(v) for v in reads), {}, list(outs))]
    prog.ops = ops
    return prog


# ------------------------------------------------------------------------------------------------ sharding
def _row_of(mesh, mesh_dim):
    n = mesh.size(mesh_dim)
    ranks = mesh.mesh.movedim(mesh_dim, -1).reshape(-1, n)
    return next(r for r in ranks.tolist() if dist.get_rank() in r)


def _coalesced_broadcast(tensors, src, group):
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.broadcast(flat, src=src, group=group)
    off = 0
    for t in tensors:
        t.copy_(flat[off:off + t.numel()].view_as(t))
        off += t.numel()


class _Stage3State:
    """Runtime state of the static stage-3 program: per-unit gathers (forward, one unit of prefetch), re-gathers for
    the backward through saved-tensor hooks, the asynchronous reduces to the owners, and a live-bytes meter."""

    def __init__(self, units, owners, row, group, me):
        self.units = units            # [[Parameter, ...]] in forward order
        self.owners, self.row, self.group, self.me = owners, row, group, me
        self.prefetched = {}          # unit -> (works, tensors) issued ahead
        self.bwd_cache = {}           # unit -> re-gathered tensors (backward), dropped by the unit's backward
        self.pending = []             # (work, grad, param) reduces in flight
        self.storage = {}             # storage data_ptr -> (unit, index) of live gathered tensors
        self.live = 0
        self.peak = 0
        self.n_gathers = 0
        self.hooks = None

    # ---- gathers
    def _issue(self, k):
        works, outs = [], []
        for p in self.units[k]:
            o = self.owners[p.name]
            full = torch.empty(self.shapes[p.name], dtype=p._t.dtype, device=p._t.device)
            if o == self.me:
                full.copy_(p._t.detach())
            works.append(dist.broadcast(full, src=self.row[o], group=self.group, async_op=True))
            outs.append(full)
        self.n_gathers += 1
        return works, outs

    def _track(self, k, outs):
        import weakref

        for i, t in enumerate(outs):
            key = t.untyped_storage().data_ptr()
            self.storage[key] = (k, i)
            nb = t.numel() * t.element_size()
            self.live += nb
            weakref.finalize(t, self._untrack, key, nb)
        self.peak = max(self.peak, self.live)

    def _untrack(self, key, nb):
        self.storage.pop(key, None)
        self.live -= nb

    def materialize(self, k):
        works, outs = self.prefetched.pop(k, None) or self._issue(k)
        for w in works:
            w.wait()
        self._track(k, outs)
        return outs

    def prefetch(self, k):
        if 0 <= k < len(self.units) and k not in self.prefetched and k not in self.bwd_cache:
            self.prefetched[k] = self._issue(k)

    # ---- backward re-gather (saved-tensor hooks)
    def pack(self, t):
        if not isinstance(t, torch.Tensor) or t.device.type == "meta":
            return t
        hit = self.storage.get(t.untyped_storage().data_ptr())
        if hit is None:
            return t
        base = t._base if t._base is not None else t
        return ("_p2_stage3", hit[0], hit[1], tuple(t.size()), tuple(t.stride()),
                t.storage_offset() - base.storage_offset(), t.requires_grad)

    def unpack(self, x):
        if not (isinstance(x, tuple) and x and x[0] == "_p2_stage3"):
            return x
        _, k, i, size, stride, off, _rg = x
        if k not in self.bwd_cache:
            self.bwd_cache[k] = self.materialize(k)
            self.prefetch(k - 1)   # one unit ahead in backward order
        return torch.as_strided(self.bwd_cache[k][i], size, stride, off)

    def release_bwd(self, k):
        self.bwd_cache.pop(k, None)

    def reduce_async(self, k, grads):
        for p, g in zip(self.units[k], grads):
            g = torch.zeros(self.shapes[p.name], dtype=p._t.dtype, device=p._t.device) if g is None else g.contiguous()
            w = dist.reduce(g, dst=self.row[self.owners[p.name]], group=self.group, async_op=True)
            self.pending.append((w, g, p))


class _Stage2Buckets:
    """Stage 2's gradient reduces issued FROM the backward: each parameter's post-accumulate hook marks it ready;
    a bucket (one owner's parameters, in reverse order of first forward use, up to ``cap`` bytes) is flattened and
    reduced to its owner asynchronously as soon as all its members are ready, so the reduces overlap the rest of
    the backward; the sharded step waits for them (reference auto_parallel_sharding.py:1192 fused + overlapped
    gradient comm)."""

    def __init__(self, buckets, owners, row, group, me):
        self.buckets, self.owners, self.row, self.group, self.me = buckets, owners, row, group, me
        self.bucket_of = {id(p._t): bi for bi, b in enumerate(buckets) for p in b}
        self.ready = [set() for _ in buckets]
        self.pending = []             # (work, flat, bucket index)
        self.acc = {}                 # owner: parameter name -> reduced gradient summed over backwards
        self.issued = 0
        self.from_backward = 0        # reduces launched by the hooks, i.e. while the backward was still running

    def hook(self, t):
        bi = self.bucket_of.get(id(t))
        if bi is None:
            return
        self.ready[bi].add(id(t))
        if len(self.ready[bi]) == len(self.buckets[bi]):
            self._launch(bi)

    def _launch(self, bi):
        ps = self.buckets[bi]
        with torch.no_grad():
            flat = torch.cat([(p._t.grad if p._t.grad is not None else torch.zeros_like(p._t)).reshape(-1)
                              for p in ps])
            for p in ps:
                p._t.grad = None      # consumed: the next backward (gradient merge) accumulates afresh
        w = dist.reduce(flat, dst=self.row[self.owners[ps[0].name]], group=self.group, async_op=True)
        self.pending.append((w, flat, bi))
        self.ready[bi] = set()
        self.issued += 1

    def settle(self):
        """Wait for every reduce (launching buckets a backward left partly ready, in bucket order — the same on
        every rank), then hand the owners their summed gradients."""
        self.from_backward += len(self.pending)
        for bi, r in enumerate(self.ready):
            if r:
                self._launch(bi)
        for w, flat, bi in self.pending:
            w.wait()
            ps = self.buckets[bi]
            if self.owners[ps[0].name] == self.me:
                off = 0
                for p in ps:
                    k = p._t.numel()
                    g = flat[off:off + k].view_as(p._t)
                    self.acc[p.name] = g if p.name not in self.acc else self.acc[p.name] + g
                    off += k
        self.pending.clear()
        out, self.acc = self.acc, {}
        return out


class _GatherUnit(torch.autograd.Function):
    """Forward: the full parameters of unit k (broadcast from their owners; unit k + 1 is prefetched).  Backward:
    drops the unit's re-gathered copy and issues the gradient reduce to the owners asynchronously (it overlaps the
    rest of the backward; the sharded step waits for it) — the parameters themselves get no autograd gradient."""

    @staticmethod
    def forward(ctx, state, k, *params):
        ctx.state, ctx.k, ctx.n = state, k, len(params)
        outs = state.materialize(k)
        state.prefetch(k + 1)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        ctx.state.release_bwd(ctx.k)
        ctx.state.reduce_async(ctx.k, grads)
        return (None, None) + (None,) * ctx.n


def _stage2_buckets(prog, params, owners, row, group, me, cap=16 << 20):
    """Buckets for _Stage2Buckets: each owner's parameters in reverse order of first forward use (the order the
    backward finishes them), cut at ``cap`` bytes; hooks registered on every parameter."""
    first = {}
    by_id = {id(p._t): p for p in params}
    for i, op in enumerate(prog.ops):
        if op.kind not in ("torch", "native"):
            continue
        for x in pytree.tree_leaves((op.args, op.kwargs)):
            p = by_id.get(id(x)) if isinstance(x, torch.Tensor) else None
            if p is not None and p.name not in first:
                first[p.name] = i
    order = sorted(params, key=lambda p: -first.get(p.name, -1))
    buckets, cur, size = [], {}, {}
    for p in order:
        o = owners[p.name]
        nb = p._t.numel() * p._t.element_size()
        if o in cur and size[o] + nb > cap:
            buckets.append(cur.pop(o))
        cur.setdefault(o, []).append(p)
        size[o] = (size.get(o, 0) if o in cur and len(cur[o]) > 1 else 0) + nb
    buckets.extend(cur.values())
    st = _Stage2Buckets(buckets, owners, row, group, me)
    for p in params:
        if not p.stop_gradient:
            p._t.register_post_accumulate_grad_hook(st.hook)
    return st


def _sharding_stage3(dmp, mesh_dim, group, n, me, row):
    """Stage 3 with per-use parameter gathers (reference auto_parallel_sharding.py:584-700 broadcast-before-use /
    free-after-use, :761 / :938 fused + overlapped parameter comm, :1192 overlapped gradient comm):

    * parameters are grouped into units by their first forward consumer; ONE gather op per unit is inserted right
      before that consumer and every forward use reads its output — a rank holds 1/n of the parameters plus the
      gathered unit(s) in flight (the next unit is prefetched asynchronously), and each gathered copy dies after its
      last forward reader (the executor drops it; the autograd graph keeps a token, not the tensor);
    * the backward re-gathers a unit when its first saved tensor is unpacked (one unit of prefetch in backward
      order) and drops it when the unit's gather node runs, which also issues the gradient reduce to the owners
      asynchronously — overlapped with the rest of the backward;
    * the sharded step waits for the reduces, steps the owned parameters and leaves the others released."""
    from ....static.graph import Op, VarRef

    prog = dmp.program
    i_bwd = next((i for i, o in enumerate(prog.ops) if o.kind in ("backward", "grad")), len(prog.ops))
    opt_ops = [(i, o) for i, o in enumerate(prog.ops) if o.kind == "optimize"]
    owners, shapes, plist = {}, {}, []
    for _, op in opt_ops:
        opt = op.attrs["optimizer"]
        load = [0] * n
        for p in sorted(opt._parameter_list, key=lambda q: -q._t.numel()):
            o = min(range(n), key=lambda r: load[r])
            owners[p.name] = o
            load[o] += p._t.numel()
            shapes[p.name] = tuple(p._t.shape)
            plist.append(p)
    by_id = {id(p._t): p for p in plist}
    # units: parameters grouped by their first forward consumer, in program order
    first, units = {}, []
    for i in range(i_bwd):
        op = prog.ops[i]
        if op.kind not in ("torch", "native"):
            continue
        for x in pytree.tree_leaves((op.args, op.kwargs)):
            p = by_id.get(id(x)) if isinstance(x, torch.Tensor) else None
            if p is not None and p.name not in first:
                first[p.name] = i
    for i in sorted(set(first.values())):
        units.append((i, [p for p in plist if first.get(p.name) == i]))
    state = _Stage3State([u for _, u in units], owners, row, group, me)
    state.shapes = shapes
    # gather ops (inserted back to front so indices stay valid) and forward uses rewired to their outputs
    out_of = {}
    gather_ops = []
    for k, (i, ps) in enumerate(units):
        vs = [_new_var(prog, shapes[p.name], p._t.dtype) for p in ps]
        for p, v in zip(ps, vs):
            out_of[id(p._t)] = v._vid

        def gather(*params, k=k):
            return _GatherUnit.apply(state, k, *params)

        gather_ops.append((i, Op("torch", _named(gather, f"stage3_gather[{k}]", comm=True, stage3=True),
                                 tuple(p._t for p in ps), {}, [v._vid for v in vs])))
    for i in range(i_bwd):
        op = prog.ops[i]
        if op.kind not in ("torch", "native"):
            continue
        swap = lambda x: VarRef(out_of[id(x)]) if isinstance(x, torch.Tensor) and id(x) in out_of else x  # noqa: E731
        op.args = pytree.tree_map(swap, op.args)
        op.kwargs = pytree.tree_map(swap, op.kwargs)

    def hooks_on(env):
        state.hooks = torch.autograd.graph.saved_tensors_hooks(state.pack, state.unpack)
        state.hooks.__enter__()

    def hooks_off(env):
        if state.hooks is not None:
            state.hooks.__exit__(None, None, None)
            state.hooks = None

    for i, op in opt_ops:
        opt = op.attrs["optimizer"]
        mine = [p for p in opt._parameter_list if owners[p.name] == me]

        def step(env, opt=opt, mine=mine):
            full = opt._parameter_list
            with torch.no_grad():
                for w, g, p in state.pending:
                    w.wait()
                    if owners[p.name] == me:
                        p._t.grad = g if p._t.grad is None else p._t.grad + g
                state.pending.clear()
                state.bwd_cache.clear()
                state.prefetched.clear()
                opt._parameter_list, opt._mt_cache = mine, None
                try:
                    opt.step()
                finally:
                    opt._parameter_list, opt._mt_cache = full, None
                for p in full:
                    if owners[p.name] != me and p._t.numel():
                        p._t.data = torch.empty(0, dtype=p._t.dtype, device=p._t.device)
            opt.clear_grad(set_to_zero=False)

        prog.ops[i] = Op("call", None, (), {}, [], {"fn": step, "name": "sharding_stage3_step", "optimizer": opt})
    prog.ops.insert(i_bwd, Op("call", None, (), {}, [], {"fn": hooks_off, "name": "sharding_stage3_hooks_off"}))
    for i, op in sorted(gather_ops, key=lambda t: -t[0]):
        prog.ops.insert(i, op)
    prog.ops.insert(0, Op("call", None, (), {}, [], {"fn": hooks_on, "name": "sharding_stage3_hooks_on"}))

    def gather_params(env=None):
        """re-materialise every parameter from its owner into the parameters themselves (checkpointing)."""
        with torch.no_grad():
            for p in plist:
                if tuple(p._t.shape) != shapes[p.name]:
                    p._t.data = torch.empty(shapes[p.name], dtype=p._t.dtype, device=p._t.device)
            for o in range(n):
                ps = [p._t for p in plist if owners[p.name] == o]
                if ps:
                    _coalesced_broadcast(ps, row[o], group)

    with torch.no_grad():   # stage 3 starts from the released state: a rank holds only its own parameters
        for p in plist:
            if owners[p.name] != me:
                p._t.data = torch.empty(0, dtype=p._t.dtype, device=p._t.device)
    dmp.gather_params = gather_params
    dmp.stage3_state = state
    return owners


def sharding_pass(dmp, mesh_dim=0, stage=1):
    """ZeRO over ``mesh_dim`` (reference python/paddle/distributed/passes/auto_parallel_sharding.py:92-740
    ``ShardingPass``, stages 1 / 2 / 3).  Parameters are assigned to owners greedily by size.

    * stage 1 — optimizer state sharded: each rank steps only its own parameters (accumulators exist only for
      those) and broadcasts them, one coalesced broadcast per owner;
    * stage 2 — + gradients sharded: the per-use gradient all-reduces of the replicated parameters over
      ``mesh_dim`` (the plan's ``c_identity`` ops, or a fused all-reduce from ``fuse_allreduce_pass``) are removed;
      each owner's gradients are reduced to it in buckets issued asynchronously FROM the backward as they become
      ready (_Stage2Buckets; half the bytes of the all-reduce, overlapped with the rest of the backward) and the
      other ranks drop theirs;
    * stage 3 — + parameters sharded, gathered per use (_sharding_stage3): one gather op per unit right before
      its first forward consumer, next unit prefetched, backward re-gathers through saved-tensor hooks, gradient
      reduces to the owners issued asynchronously from the backward; a rank holds 1/n of the parameters plus the
      unit(s) in flight, during the step as between steps.
    -> {param name: owner}; ``dmp.gather_params()`` materialises every parameter (e.g. before a checkpoint)."""
    from ....static.graph import Op

    assert stage in (1, 2, 3)
    prog = dmp.program
    mesh = dmp._dm
    group = mesh.get_group(mesh_dim)
    n = mesh.size(mesh_dim)
    me = mesh.get_local_rank(mesh_dim)
    row = _row_of(mesh, mesh_dim)
    if stage >= 2:
        from .resharder import _grad_allreduce_fn

        for op in prog.ops:
            fn = op.fn
            if op.kind == "torch" and getattr(fn, "comm", False) and fn.__name__ == "c_identity" and \
                    isinstance(op.args[0], torch.Tensor) and op.args[0].requires_grad and mesh_dim in fn.dims:
                rest = tuple(d for d in fn.dims if d != mesh_dim)
                op.fn = _grad_allreduce_fn(fn.mesh, rest) if rest else _named(lambda x: x, "identity")
        prog.ops = [o for o in prog.ops if not (o.kind == "call" and o.attrs.get("name") == "fused_allreduce_grads")]
    if stage == 3:
        return _sharding_stage3(dmp, mesh_dim, group, n, me, row)
    owners, released = {}, []
    for i, op in enumerate(prog.ops):
        if op.kind != "optimize":
            continue
        opt = op.attrs["optimizer"]
        load = [0] * n
        for p in sorted(opt._parameter_list, key=lambda q: -q._t.numel()):
            o = min(range(n), key=lambda r: load[r])
            owners[p.name] = o
            load[o] += p._t.numel()
        mine = [p for p in opt._parameter_list if owners[p.name] == me]
        shapes = {p.name: (tuple(p._t.shape), p._t.dtype, p._t.device) for p in opt._parameter_list}
        bk = None
        if stage == 2:
            bk = _stage2_buckets(prog, opt._parameter_list, owners, row, group, me)
            dmp.stage2_buckets = bk

        def step(env, opt=opt, mine=mine, bk=bk):
            full = opt._parameter_list
            with torch.no_grad():
                if bk is not None:
                    red = bk.settle()
                    for p in full:
                        p._t.grad = red.get(p.name) if owners[p.name] == me else None
                opt._parameter_list, opt._mt_cache = mine, None
                try:
                    opt.step()
                finally:
                    opt._parameter_list, opt._mt_cache = full, None
                if stage < 3:
                    for o in range(n):
                        ps = [p._t for p in full if owners[p.name] == o]
                        if ps:
                            _coalesced_broadcast(ps, row[o], group)
                else:
                    for p in full:
                        if owners[p.name] != me:
                            p._t.data = torch.empty(0, dtype=p._t.dtype, device=p._t.device)
            opt.clear_grad(set_to_zero=False)

        prog.ops[i] = Op("call", None, (), {}, [], {"fn": step, "name": f"sharding_stage{stage}_step",
                                                     "optimizer": opt})
        released.append((opt, shapes))

    def gather_params(env=None):
        """(stage 3) re-materialise every parameter from its owner: one coalesced broadcast per owner."""
        with torch.no_grad():
            for opt, shapes in released:
                for p in opt._parameter_list:
                    shp, dt, dev = shapes[p.name]
                    if tuple(p._t.shape) != shp:
                        p._t.data = torch.empty(shp, dtype=dt, device=dev)
                for o in range(n):
                    ps = [p._t for p in opt._parameter_list if owners[p.name] == o]
                    if ps:
                        _coalesced_broadcast(ps, row[o], group)

    if stage == 3:
        prog.ops.insert(0, Op("call", None, (), {}, [], {"fn": gather_params, "name": "sharding_stage3_gather"}))
        # stage 3 starts from the released state: a rank holds only its own parameters
        with torch.no_grad():
            for opt, _ in released:
                for p in opt._parameter_list:
                    if owners[p.name] != me:
                        p._t.data = torch.empty(0, dtype=p._t.dtype, device=p._t.device)
    dmp.gather_params = gather_params
    return owners


# ------------------------------------------------------------------------------------------------ sequence parallel
# ops whose output row i depends only on input row i of the sequence operand (the other operands are parameters or
# per-row activations of the same length): the reduce-scatter can move in front of them
_ROW_LOCAL = {"add", "sub", "mul", "div", "relu", "gelu", "silu", "sigmoid", "tanh", "swish", "addmm", "mm",
              "matmul", "linear", "scale", "dropout", "rms_norm", "layer_norm", "cast", "pow", "neg", "exp"}


def _consumers(prog):
    from ....static.graph import VarRef

    uses = {}
    for i, op in enumerate(prog.ops):
        for x in pytree.tree_leaves((op.args, op.kwargs)):
            if isinstance(x, VarRef):
                uses.setdefault(x.vid, []).append(i)
        if "loss" in op.attrs:
            uses.setdefault(op.attrs["loss"], []).append(i)
    return uses


# operand positions that carry the sequence (row) dimension, by op: every other position is a weight-like operand
_SP_ROW_POS = {"mm": (0,), "matmul": (0,), "linear": (0,), "addmm": (1,), "rms_norm": (0,), "layer_norm": (0,)}


def _sp_operand_roles(prog, e, cur):
    """Roles of op ``e``'s positional operands for the sequence-parallel rewrite, or None when the op cannot be
    moved onto the sequence shard.  "row": carries the sequence dim (split onto the shard); "param": a weight-like
    graph value (its gradient is all-reduced over the mesh dims once the op sees only the local rows); "const":
    left alone.  The decision comes from the op's operand semantics — for a GEMM only the activation position, for
    an elementwise op only an operand of the output's rank whose leading dim is the row count — never from a shape
    coincidence (a [hidden, hidden] weight with hidden == rows stays a weight).  Keyword operands that are graph
    values or trainable tensors end the chain: they are not rewritten, so moving the op would be wrong."""
    from ....static.graph import VarRef

    for x in pytree.tree_leaves(e.kwargs):
        if isinstance(x, VarRef) or (isinstance(x, torch.Tensor) and (x.requires_grad or x.dim() > 0)):
            return None
    key = op_key(e)
    cur_v = prog.vars[cur]
    rows, nd = cur_v.shape[0], len(cur_v.shape)
    roles = []
    for k, x in enumerate(e.args):
        if key in _SP_ROW_POS:
            if isinstance(x, VarRef):
                if k in _SP_ROW_POS[key]:
                    roles.append("row")
                elif x.vid == cur:
                    return None      # the chain value in a weight position (e.g. x^T-shaped use): not row-local
                else:
                    roles.append("param")
            elif k in _SP_ROW_POS[key]:
                return None          # the row operand is not a graph value
            else:
                roles.append("const")
            continue
        # elementwise / activation: row-aligned iff same rank as the chain value with the row count leading
        if isinstance(x, VarRef):
            xs = prog.vars[x.vid].shape
            if x.vid == cur or (len(xs) == nd and nd > 0 and xs[0] == rows):
                roles.append("row")
            elif len(xs) < nd or (len(xs) == nd and xs[0] == 1):
                roles.append("param")   # broadcast along the rows
            else:
                return None
        elif isinstance(x, torch.Tensor) and x.dim() == nd and nd > 0 and x.shape[0] == rows and x.shape[0] != 1:
            return None              # a full-length constant would need its own split
        else:
            roles.append("const")
    if key in _SP_ROW_POS and not any(isinstance(x, VarRef) and x.vid == cur for k, x in enumerate(e.args)
                                      if k in _SP_ROW_POS[key]):
        return None
    return roles


def sequence_parallel_optimization_pass(dmp):
    """Megatron sequence parallelism on the plan (reference python/paddle/distributed/passes/
    auto_parallel_sequence_parallel_optimization.py:33): a partial sum that is all-reduced, then run through
    row-local ops (residual add, activation, norm, a linear with replicated weights), then split on the sequence
    (dim 0) over the same mesh dim is rewritten as ONE reduce-scatter onto the sequence shards followed by the same
    ops on the shard — the all-reduce's second half and the redundant full-length ops disappear.  Per-row
    activation operands of the moved ops are split to the shard (their gradient all-gathers back); a replicated
    parameter operand gets a gradient all-reduce over the mesh dim (it now sees only the local rows).
    -> number of rewritten chains."""
    from ....static.graph import Op, VarRef
    from ..placement import Partial, Replicate, Shard
    from .resharder import _comm_fn, _grad_allreduce_fn, comm_kinds

    prog = dmp.program
    uses = _consumers(prog)
    n_done = 0
    i = 0
    while i < len(prog.ops):
        a = prog.ops[i]
        fa = a.fn
        if not (a.kind == "torch" and getattr(fa, "comm", False) and fa.__name__ in ("c_allreduce_sum", "c_allreduce_avg")
                and hasattr(fa, "src")):
            i += 1
            continue
        dims = [d for d, (s_, t_) in enumerate(zip(fa.src, fa.dst)) if isinstance(s_, Partial) and isinstance(t_, Replicate)]
        # follow the single-consumer chain
        chain, cur, b = [], a.outs[0], None
        while True:
            us = uses.get(cur, [])
            if len(us) != 1:
                break
            e = prog.ops[us[0]]
            fe = e.fn
            if e.kind == "torch" and getattr(fe, "comm", False) and fe.__name__ == "c_split" and hasattr(fe, "dst"):
                sd = [d for d, (s_, t_) in enumerate(zip(fe.src, fe.dst)) if isinstance(s_, Replicate) and isinstance(t_, Shard)]
                if sd == dims and all(fe.dst[d].dim == 0 for d in sd):
                    b = (us[0], e)
                break
            if e.kind not in ("torch", "native") or op_key(e) not in _ROW_LOCAL or len(e.outs) != 1:
                break
            roles = _sp_operand_roles(prog, e, cur)
            if roles is None:
                break
            chain.append((us[0], e, roles))
            cur = e.outs[0]
        if b is None or not dims:
            i += 1
            continue
        mesh = fa.mesh
        nsh = 1
        for d in dims:
            nsh *= mesh.size(d)
        rows = prog.vars[a.outs[0]].shape[0]
        # the all-reduce becomes the reduce-scatter onto the sequence shards
        dst = list(fa.src)
        for d in dims:
            dst[d] = Shard(0)
        a.fn = _comm_fn(comm_kinds(fa.src, tuple(dst)), mesh, fa.src, tuple(dst))
        old_out = a.outs[0]
        ov = prog.vars[old_out]
        nv = _new_var(prog, [ov.shape[0] // nsh] + list(ov.shape[1:]), ov.dtype)
        a.outs = [nv._vid]
        rename = {old_out: nv._vid}
        inserts = []   # (before op index, Op)
        for idx, e, roles in chain:
            new_args = []
            for x, role in zip(e.args, roles):
                if isinstance(x, VarRef) and x.vid in rename:
                    new_args.append(VarRef(rename[x.vid]))
                elif isinstance(x, VarRef) and role == "row":
                    # a per-row activation operand: split it onto the shard too (backward: all-gather)
                    xv = prog.vars[x.vid]
                    sv = _new_var(prog, [rows // nsh] + list(xv.shape[1:]), xv.dtype)
                    srcp = tuple(Replicate() for _ in fa.src)
                    inserts.append((idx, Op("torch", _comm_fn(["c_split"], mesh, srcp, tuple(dst)), (x,), {},
                                            [sv._vid])))
                    new_args.append(VarRef(sv._vid))
                elif (isinstance(x, torch.Tensor) and x.requires_grad) or (isinstance(x, VarRef) and role == "param"):
                    # a replicated parameter now applied to the local rows only: its gradient is summed over dims
                    xm = prog.vars[x.vid] if isinstance(x, VarRef) else x
                    pv = _new_var(prog, list(xm.shape), xm.dtype)
                    inserts.append((idx, Op("torch", _grad_allreduce_fn(mesh, tuple(dims)), (x,), {}, [pv._vid])))
                    new_args.append(VarRef(pv._vid))
                else:
                    new_args.append(x)
            e.args = tuple(new_args)
            old = e.outs[0]
            evr = prog.vars[old]
            ev = _new_var(prog, [evr.shape[0] // nsh] + list(evr.shape[1:]), evr.dtype)
            e.outs = [ev._vid]
            rename[old] = ev._vid
        bidx, bop = b
        bop.args = tuple(VarRef(rename[x.vid]) if isinstance(x, VarRef) and x.vid in rename else x for x in bop.args)
        bop.fn = _named(lambda x: x, "identity")   # the split is already done
        for idx, op in sorted(inserts, key=lambda t: -t[0]):
            prog.ops.insert(idx, op)
        uses = _consumers(prog)
        n_done += 1
        i += 1
    return n_done


# ------------------------------------------------------------------------------------------------ comm / compute overlap
class _OverlapLinear(torch.autograd.Function):
    """y = x @ w (+ b) whose input gradient is all-reduced over mesh dims: the all-reduce of dX is issued
    asynchronously right after dX and waited for only after dW / db — the column-parallel pattern of
    allreduce_matmul_grad_overlapping.py:37."""

    @staticmethod
    def forward(ctx, x, w, b, mesh, dims):
        ctx.save_for_backward(x, w)
        ctx.mesh, ctx.dims, ctx.has_b = mesh, dims, b is not None
        return torch.addmm(b, x, w) if b is not None else x @ w

    @staticmethod
    def backward(ctx, g):
        from ..reshard import COMM_LOG, _group

        x, w = ctx.saved_tensors
        dx = (g @ w.t()).contiguous()
        works = []
        for d in ctx.dims:
            works.append(dist.all_reduce(dx, op=dist.ReduceOp.SUM, group=_group(ctx.mesh, d), async_op=True))
            COMM_LOG.append(("grad_all_reduce_overlap", d))
            if len(ctx.dims) > 1:   # several dims: each sum must finish before the next starts
                works.pop().wait()
        dw = x.t() @ g
        db = g.sum(0) if ctx.has_b else None
        for wk in works:
            wk.wait()
        return dx, dw, db, None, None


def allreduce_matmul_grad_overlap_pass(dmp):
    """(reference python/paddle/distributed/passes/allreduce_matmul_grad_overlapping.py:37) a ``c_identity`` on a
    linear's activation input (its backward all-reduces dX over the mesh: the column-parallel input) followed by
    that linear (``addmm`` / ``mm`` / ``matmul``, the activation as the row operand) becomes one op whose backward
    overlaps the dX all-reduce with the dW / db GEMMs instead of running it after them.  -> fused pairs."""
    from ....static.graph import Op, VarRef

    prog = dmp.program
    uses = _consumers(prog)
    n = 0
    for i, op in enumerate(prog.ops):
        f = op.fn
        if not (op.kind == "torch" and getattr(f, "comm", False) and f.__name__ == "c_identity"
                and isinstance(op.args[0], VarRef) and hasattr(f, "mesh")):
            continue
        us = uses.get(op.outs[0], [])
        if len(us) != 1:
            continue
        mm = prog.ops[us[0]]
        key = op_key(mm) if mm.kind in ("torch", "native") else ""
        if key == "addmm" and len(mm.args) == 3 and isinstance(mm.args[1], VarRef) and mm.args[1].vid == op.outs[0] \
                and not mm.kwargs:
            b, w = mm.args[0], mm.args[2]
        elif key in ("mm", "matmul") and len(mm.args) == 2 and isinstance(mm.args[0], VarRef) and \
                mm.args[0].vid == op.outs[0] and not mm.kwargs:
            b, w = None, mm.args[1]
        else:
            continue
        if not (isinstance(w, (torch.Tensor, VarRef))) or (isinstance(w, torch.Tensor) and w.dim() != 2):
            continue
        mesh, dims = f.mesh, tuple(f.dims)

        def fused(x, w_, b_=None, mesh=mesh, dims=dims):
            return _OverlapLinear.apply(x, w_, b_, mesh, dims)

        mm.fn = _named(fused, "linear_overlap_dx_allreduce", comm=True)
        mm.args = (op.args[0], w) + ((b,) if b is not None else ())
        op.fn = _named(lambda x: x, "identity")   # its all-reduce moved into the fused backward
        op.fn.comm = False
        n += 1
    return n
