"""Static auto-parallel: the Resharder — materialise a completed, partitioned Program as this rank's
``dist_main_program`` with explicit communication ops (reference python/paddle/distributed/auto_parallel/static/
reshard.py ``Resharder.reshard`` — inserts c_allgather / c_allreduce_sum / c_reducescatter / alltoall / slice ops —
and partitioner.py ``Partitioner.partition`` — local variables and parameters).

Where ``DistributedProgram.run`` moves tensors on the fly while it interprets the serial program, ``build`` writes
every movement into a NEW static Program:

* parameters become their local shards (leaf tensors; a sharded Parameter's storage is replaced by its shard so
  the user's optimizer steps it), variables get local shapes from their completed dims_mapping;
* in front of an op whose SPMD rule needs an input in another distribution, a communication op named after the
  collectives it runs (``c_allgather``, ``c_allreduce_sum`` / ``_avg``, ``c_reducescatter``, ``alltoall``,
  ``c_split`` (local slice), ``c_partial`` (replicated -> partial)) is inserted; each is differentiable — its
  backward is the conjugate movement;
* a replicated input of an op that computes different data per mesh coordinate gets a ``c_identity`` op whose
  backward all-reduces the gradient (Megatron's column-parallel input / the data-parallel weight gradient);
* local attribute rewrites (reshape targets) are applied to the copied op, and a bias added to a partial
  product goes through a ``c_partial`` op (kept on mesh coordinate 0) so the partial sum counts it once;
* fetch targets are resharded to replicated at the end; ``backward`` / ``param_grad`` / ``optimize`` instructions
  are carried over, ``backward`` starting from the replicated loss.

The result is an ordinary Program: it prints, and the framework's static ``Executor`` (PIR passes + the native
interpreter plan) runs it — forward, the autograd backward through the communication ops, the optimizer step.
"""
from __future__ import annotations

import torch
import torch.utils._pytree as pytree

from ..placement import Partial, Replicate, Shard
from .completion import DistAttr, tensor_key
from .partitioner import _GradAllReduce, _LocalReshard


def comm_kinds(src, dst):
    """The collectives ``reshard.reshard_local`` runs for src -> dst placements (same order)."""
    cur = list(src)
    out = []
    nd = len(cur)
    for d in range(nd):
        s, t = cur[d], dst[d]
        if isinstance(s, Partial) and not isinstance(t, Partial):
            if isinstance(t, Shard) and not any(isinstance(c, Shard) and c.dim == t.dim for c in cur):
                out.append("c_reducescatter")
                cur[d] = t
            else:
                out.append("c_allreduce_" + s.reduce_op)
                cur[d] = Replicate()
    for d in reversed(range(nd)):
        s, t = cur[d], dst[d]
        if isinstance(s, Shard) and s != t:
            if isinstance(t, Shard) and not any(isinstance(c, Shard) and c.dim == t.dim
                                                for i, c in enumerate(cur) if i != d):
                out.append("alltoall")
                cur[d] = t
            else:
                out.append("c_allgather")
                cur[d] = Replicate()
    for d in range(nd):
        s, t = cur[d], dst[d]
        if isinstance(s, Replicate) and isinstance(t, Shard):
            out.append("c_split")
        elif isinstance(s, Replicate) and isinstance(t, Partial):
            out.append("c_partial")
    return out


def _comm_fn(kinds, mesh, src, dst):
    def fn(x):
        return _LocalReshard.apply(x, mesh, src, dst)

    fn.__name__ = fn.__qualname__ = "+".join(kinds) or "identity"
    fn.comm = True
    fn.mesh, fn.src, fn.dst = mesh, tuple(src), tuple(dst)   # what passes (sequence_parallel_optimization) rewrite
    return fn


def _partial_term_fn(mesh, dims):
    """Replicated -> partial-sum term: the value on mesh coordinate 0 of ``dims``, zeros elsewhere (the product with
    zero carries the matching zero gradient)."""
    root = all(mesh.get_local_rank(d) == 0 for d in dims)

    def fn(x):
        return x if root else x * 0

    fn.__name__ = fn.__qualname__ = "c_partial"
    fn.comm = True
    return fn


def _grad_allreduce_fn(mesh, dims):
    def fn(x):
        return _GradAllReduce.apply(x, mesh, dims)

    fn.__name__ = fn.__qualname__ = "c_identity"
    fn.comm = True
    fn.dims = tuple(dims)
    fn.mesh = mesh
    return fn


class DistMainProgram:
    """This rank's program + how to feed it (global feeds are sliced to the feed annotations)."""

    def __init__(self, program, feed_attrs, fetch_map, mesh_groups, nd):
        self.program = program
        self._feed_attrs = feed_attrs      # feed name -> DistAttr
        self._fetch = fetch_map            # serial vid -> dist vid
        self._dm, self._nd = mesh_groups, nd

    def local_feed(self, feed):
        from ..reshard import reshard_local

        out = {}
        for name, v in feed.items():
            t = v._t if hasattr(v, "_t") else torch.as_tensor(v)
            attr = self._feed_attrs.get(name) or DistAttr([-1] * t.dim())
            out[name] = reshard_local(t, self._dm, DistAttr([-1] * t.dim()).placements(self._nd),
                                      attr.placements(self._nd))
        return out

    def fetch(self, var):
        """The dist program's variable for a serial fetch target."""
        t = var._t if hasattr(var, "_t") else var
        return self.program.vars[self._fetch[t._vid]]

    def comm_ops(self):
        return [op.name for op in self.program.ops if getattr(op.fn, "comm", False)]


class Resharder:
    def __init__(self, dist_program):
        self.dp = dist_program
        self.ctx = dist_program.ctx
        self.mesh = dist_program.mesh
        self.dm = dist_program.dm
        self.nd = dist_program.nd

    def _local_shape(self, shape, attr):
        return [s // self.mesh.shape[d] if d != -1 and s > 0 else s for s, d in zip(shape, attr.dims_mapping)]

    def build(self, fetch_list=()):
        from ....static.graph import Op, Program, VarRef

        src, ctx = self.dp.program, self.ctx
        prog = Program()
        env = {}        # serial key -> (VarRef or leaf tensor, DistAttr)
        feed_attrs = {}
        for name, sym in src.feeds.items():
            key = ("v", sym._vid)
            attr = ctx.attrs.get(key) or DistAttr([-1] * sym.dim())
            meta = torch.empty(self._local_shape(list(sym.shape), attr), dtype=sym.dtype, device="meta")
            v = prog.new_var(meta, name=name)
            prog.feeds[name] = v
            env[key] = (VarRef(v._vid), attr)
            feed_attrs[name] = attr

        def move(val, cur, req, dtype, gshape):
            if cur.same(req):
                return val, cur
            s, d = cur.placements(self.nd), req.placements(self.nd)
            meta = torch.empty(self._local_shape(gshape, req), dtype=dtype, device="meta")
            v = prog.new_var(meta)
            prog.ops.append(Op("torch", _comm_fn(comm_kinds(s, d), self.dm, s, d), (val,), {}, [v._vid]))
            return VarRef(v._vid), req

        for op, plan in zip(src.ops, ctx.plans):
            if op.kind not in ("torch", "native"):
                attrs = dict(op.attrs)
                if "loss" in attrs and ("v", attrs["loss"]) in env:
                    # backward starts from the REPLICATED loss (a partial-avg loss gives each rank grad / n)
                    val, cur = env[("v", attrs["loss"])]
                    lv = src.vars[attrs["loss"]]
                    val, _ = move(val, cur, DistAttr([-1] * lv.dim()), lv.dtype, list(lv.shape))
                    attrs["loss"] = val.vid
                if op.kind == "param_grad" and "out" in attrs:
                    gv = src.vars.get(attrs["out"])
                    if gv is not None:
                        nv = prog.new_var(torch.empty_like(attrs["param"]._t, device="meta"), name=gv._name)
                        env[("v", attrs["out"])] = (VarRef(nv._vid), DistAttr([-1] * gv.dim()))
                        attrs["out"] = nv._vid
                prog.ops.append(Op(op.kind, op.fn, op.args, op.kwargs, list(op.outs), attrs))
                continue
            leaves, spec = pytree.tree_flatten((op.args, op.kwargs))
            new, ti = [], 0
            for x in leaves:
                is_t = isinstance(x, VarRef) or (isinstance(x, torch.Tensor) and x.dim() > 0)
                if not is_t:
                    new.append(x)
                    continue
                key = tensor_key(x)
                if key in env:
                    val, cur = env[key]
                elif key in self.dp._local_params:
                    val, cur = self.dp._local_params[key], ctx.attrs.get(key) or DistAttr([-1] * x.dim())
                else:
                    val, cur = x, DistAttr([-1] * x.dim())
                gshape = list(src.vars[x.vid].shape) if isinstance(x, VarRef) else list(x.shape)
                dtype = src.vars[x.vid].dtype if isinstance(x, VarRef) else x.dtype
                req = plan.in_attrs[ti]
                val, cur = move(val, cur, req, dtype, gshape)
                grad_dims = tuple(sorted(d for d in plan.split_dims if d not in req.dims_mapping and d not in req.partial))
                if grad_dims and dtype.is_floating_point:
                    meta = torch.empty(self._local_shape(gshape, req), dtype=dtype, device="meta")
                    v = prog.new_var(meta)
                    prog.ops.append(Op("torch", _grad_allreduce_fn(self.dm, grad_dims), (val,), {}, [v._vid]))
                    val = VarRef(v._vid)
                new.append(val)
                ti += 1
            args, kwargs = pytree.tree_unflatten(new, spec)
            args = self._local_attrs(op, plan, list(args))
            if plan.key in ("addmm", "linear") and plan.out_attrs[0].partial:
                # a bias added to a partial product: a partial term itself (kept on coordinate 0 only)
                bi = 0 if plan.key == "addmm" else 2
                if len(args) > bi and args[bi] is not None:
                    b = args[bi]
                    bshape, bdt = (list(prog.vars[b.vid].shape), prog.vars[b.vid].dtype) if isinstance(b, VarRef) \
                        else (None, None)
                    if bshape is None and isinstance(b, torch.Tensor):
                        bshape, bdt = list(b.shape), b.dtype
                    if bshape is not None:
                        part = tuple(sorted(plan.out_attrs[0].partial))
                        v = prog.new_var(torch.empty(bshape, dtype=bdt, device="meta"))
                        prog.ops.append(Op("torch", _partial_term_fn(self.dm, part), (b,), {}, [v._vid]))
                        args[bi] = VarRef(v._vid)
            outs = []
            for i, vid in enumerate(op.outs):
                if vid is None:
                    outs.append(None)
                    continue
                sv = src.vars[vid]
                meta = torch.empty(self._local_shape(list(sv.shape), plan.out_attrs[i]), dtype=sv.dtype,
                                   device="meta")
                nv = prog.new_var(meta)
                outs.append(nv._vid)
                env[("v", vid)] = (VarRef(nv._vid), plan.out_attrs[i])
            prog.ops.append(Op(op.kind, op.fn, tuple(args), kwargs, outs, dict(op.attrs)))
        fetch_map = {}
        for f in fetch_list:
            t = f._t if hasattr(f, "_t") else f
            val, cur = env[("v", t._vid)]
            sv = src.vars[t._vid]
            val, _ = move(val, cur, DistAttr([-1] * sv.dim()), sv.dtype, list(sv.shape))
            fetch_map[t._vid] = val.vid
        return DistMainProgram(prog, feed_attrs, fetch_map, self.dm, self.nd)

    def _local_attrs(self, op, plan, args):
        """Reshape / view targets divided by the sharded mesh sizes (as DistributedProgram._local_attrs)."""
        if plan.key in ("reshape", "view") and len(args) >= 2:
            out = plan.out_attrs[0]
            shape = list(args[1]) if isinstance(args[1], (list, tuple, torch.Size)) else list(args[1:])
            return [args[0], [s // self.mesh.shape[d] if d != -1 and s > 0 else s
                              for s, d in zip(shape, out.dims_mapping)]]
        return args


def build_dist_main_program(dist_program, fetch_list=(), adopt_params=True):
    """-> DistMainProgram; with ``adopt_params`` every sharded Parameter's storage becomes its local shard (the
    replicated ones keep theirs), so a ``minimize``'d serial program's optimizer steps the shards."""
    if adopt_params:
        for key, leaf in list(dist_program._local_params.items()):
            p = dist_program._param_objs[key]
            if tuple(p._t.shape) != tuple(leaf.shape):
                p._t = leaf
            else:
                dist_program._local_params[key] = p._t
    return Resharder(dist_program).build(fetch_list)
