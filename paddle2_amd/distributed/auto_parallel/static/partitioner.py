"""Static auto-parallel: partitioner + reshard insertion (reference python/paddle/distributed/auto_parallel/static/
partitioner.py ``Partitioner.partition`` and reshard.py ``Resharder``) — turn a completed serial Program into this
rank's SPMD program and execute it.

``DistributedProgram(program, ctx)``:

* every parameter is replaced by its LOCAL shard (a fresh leaf tensor; ``parameters()`` are what the optimizer
  steps), cut from the serial value by its completed dims_mapping;
* op by op, each tensor input is moved from the attribute its producer left it in to the attribute the op's
  SPMD rule requires, through the framework's reshard engine (``auto_parallel/reshard.py``: p->r all-reduce,
  p->s reduce-scatter, s->s all-to-all, s->r all-gather, r->s slice), wrapped differentiably here so the
  backward runs the conjugate movement (all-gather <-> slice, reduce-scatter -> all-gather, a partial AVG
  source receives grad / n);
* a replicated input of an op that computes different data per mesh coordinate (the op's ``split_dims``) gets
  a gradient all-reduce over those dims in backward — the column-parallel input / data-parallel weight
  gradient reduction, derived from the plan instead of hand-placed;
* local-shape attributes are rewritten: ``reshape`` / ``view`` targets are divided by the sharded mesh sizes;
  a bias added to a PARTIAL matmul output is added on mesh coordinate 0 only (so the partial sum counts it
  once);
* fetches are resharded to replicated.

The program runs under autograd, so ``loss.backward()`` + any optimizer over ``parameters()`` trains it.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.utils._pytree as pytree

from ..reshard import COMM_LOG, _group, reshard_local
from .completion import DistAttr, tensor_key


class _LocalReshard(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mesh, src, dst):
        ctx.mesh, ctx.src, ctx.dst = mesh, src, dst
        return reshard_local(x, mesh, src, dst)

    @staticmethod
    def backward(ctx, g):
        from ..placement import Partial as TP
        from ..placement import Replicate as TR

        tgt = tuple(TR() if isinstance(p, TP) else p for p in ctx.src)
        gsrc = tuple(TR() if isinstance(p, TP) else p for p in ctx.dst)
        out = reshard_local(g.contiguous(), ctx.mesh, gsrc, tgt, backward=True)
        for d, p in enumerate(ctx.src):
            if isinstance(p, TP) and p.reduce_op == "avg":
                out = out / ctx.mesh.size(d)
        return out, None, None, None


class _GradAllReduce(torch.autograd.Function):
    """Identity forward; backward sums the gradient over the given mesh dims."""

    @staticmethod
    def forward(ctx, x, mesh, dims):
        ctx.mesh, ctx.dims = mesh, dims
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        for d in ctx.dims:
            grp = _group(ctx.mesh, d)
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=grp)
            COMM_LOG.append(("grad_all_reduce", d))
        return g, None, None


class DistributedProgram:
    def __init__(self, program, ctx):
        self.program, self.ctx = program, ctx
        self.mesh = ctx.mesh
        self.dm = ctx.mesh._device_mesh()
        self.nd = self.mesh.ndim
        self._local_params = {}   # key -> local leaf tensor
        self._param_objs = {}
        from ....framework.tensor import Tensor

        for op in program.ops:
            for x in pytree.tree_leaves((op.args, op.kwargs)):
                if isinstance(x, torch.Tensor) and getattr(x, "_pd_param", None) is not None:
                    key = tensor_key(x)
                    if key in self._local_params:
                        continue
                    attr = ctx.attrs.get(key) or DistAttr([-1] * x.dim())
                    full = x.detach()
                    local = reshard_local(full, self.dm, DistAttr([-1] * x.dim()).placements(self.nd),
                                             attr.placements(self.nd))
                    leaf = local.clone().requires_grad_(not x._pd_param.stop_gradient)
                    self._local_params[key] = leaf
                    self._param_objs[key] = x._pd_param
        self._Tensor = Tensor

    def parameters(self):
        return list(self._local_params.values())

    def local_param(self, param):
        t = param._t if hasattr(param, "_t") else param
        return self._local_params[tensor_key(t)]

    def _coord0(self, dims):
        return all(self.dm.get_local_rank(d) == 0 for d in dims)

    def _move(self, x, src, dst):
        if src.same(dst):
            return x
        return _LocalReshard.apply(x, self.dm, src.placements(self.nd), dst.placements(self.nd))

    def run(self, feed, fetch_list):
        """feed: name -> FULL (serial) value (sliced here to the feed's annotation); fetch_list: symbolic vars."""
        from ....static.graph import VarRef

        T = self._Tensor
        prog, ctx = self.program, self.ctx
        env = {}   # key -> (local tensor, DistAttr)
        for name, sym in prog.feeds.items():
            if name not in feed:
                continue
            v = feed[name]
            v = v._t if isinstance(v, T) else torch.as_tensor(v)
            key = ("v", sym._vid)
            attr = ctx.attrs.get(key) or DistAttr([-1] * v.dim())
            local = reshard_local(v, self.dm, DistAttr([-1] * v.dim()).placements(self.nd),
                                     attr.placements(self.nd))
            env[key] = (local, attr)
        for op, plan in zip(prog.ops, ctx.plans):
            if plan is None:
                continue
            leaves, spec = pytree.tree_flatten((op.args, op.kwargs))
            ti = 0
            new = []
            for x in leaves:
                is_t = isinstance(x, VarRef) or (isinstance(x, torch.Tensor) and x.dim() > 0)
                if not is_t:
                    new.append(x)
                    continue
                key = tensor_key(x)
                if key in env:
                    val, cur = env[key]
                elif key in self._local_params:
                    val, cur = self._local_params[key], ctx.attrs.get(key) or DistAttr([-1] * x.dim())
                else:  # a constant tensor: replicated
                    val, cur = x, DistAttr([-1] * x.dim())
                req = plan.in_attrs[ti]
                val = self._move(val, cur, req)
                grad_dims = sorted(d for d in plan.split_dims
                                   if d not in req.dims_mapping and d not in req.partial)
                if grad_dims and val.requires_grad:
                    val = _GradAllReduce.apply(val, self.dm, tuple(grad_dims))
                new.append(val)
                ti += 1
            args, kwargs = pytree.tree_unflatten(new, spec)
            args = self._local_attrs(op, plan, list(args))
            out = op.fn(*args, **kwargs)
            outs = pytree.tree_leaves(out)
            for i, v in enumerate(op.outs):
                if v is not None:
                    env[("v", v)] = (outs[i], plan.out_attrs[i])
        res = []
        for f in fetch_list:
            t = f._t if isinstance(f, T) else f
            val, cur = env[("v", t._vid)]
            res.append(T._wrap(self._move(val, cur, DistAttr([-1] * val.dim()))))
        return res

    def _local_attrs(self, op, plan, args):
        """Local-shape rewrites of non-tensor attributes."""
        key = plan.key
        if key in ("reshape", "view") and len(args) >= 2:
            out = plan.out_attrs[0]
            shape = list(args[1]) if isinstance(args[1], (list, tuple, torch.Size)) else list(args[1:])
            local = [s // self.mesh.shape[d] if d != -1 and s > 0 else s
                     for s, d in zip(shape, out.dims_mapping)]
            return [args[0], local]
        if key in ("addmm", "linear") and plan.out_attrs[0].partial:
            bi = 0 if key == "addmm" else 2
            if len(args) > bi and isinstance(args[bi], torch.Tensor) and not self._coord0(plan.out_attrs[0].partial):
                args[bi] = args[bi] * 0
        return args


def parallelize_program(program, mesh, annotations):
    """Complete + partition: -> DistributedProgram for this rank."""
    from .completion import Completer

    ctx = Completer(mesh).complete(program, annotations)
    return DistributedProgram(program, ctx)
