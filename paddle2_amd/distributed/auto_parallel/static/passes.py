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
def sharding_pass(dmp, mesh_dim=0):
    """Stage 1: the optimizer state sharded over ``mesh_dim``.  Parameters are assigned to owners greedily by size;
    each rank steps its own and broadcasts them (one coalesced broadcast per owner).  -> {param name: owner}."""
    from ....static.graph import Op

    prog = dmp.program
    mesh = dmp._dm
    group = mesh.get_group(mesh_dim)
    n = mesh.size(mesh_dim)
    me = mesh.get_local_rank(mesh_dim)
    ranks = mesh.mesh.movedim(mesh_dim, -1).reshape(-1, n)
    row = next(r for r in ranks.tolist() if dist.get_rank() in r)
    owners = {}
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

        def step(env, opt=opt, mine=mine):
            full = opt._parameter_list
            with torch.no_grad():
                opt._parameter_list, opt._mt_cache = mine, None
                try:
                    opt.step()
                finally:
                    opt._parameter_list, opt._mt_cache = full, None
                for o in range(n):
                    ps = [p._t for p in full if owners[p.name] == o]
                    if not ps:
                        continue
                    flat = torch.cat([t.reshape(-1) for t in ps])
                    dist.broadcast(flat, src=row[o], group=group)
                    off = 0
                    for t in ps:
                        t.copy_(flat[off:off + t.numel()].view_as(t))
                        off += t.numel()
            opt.clear_grad(set_to_zero=False)

        prog.ops[i] = Op("call", None, (), {}, [], {"fn": step, "name": "sharding_stage1_step", "optimizer": opt})
    return owners
