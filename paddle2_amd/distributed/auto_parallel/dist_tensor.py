"""DistTensor: the framework's own distributed tensor (reference: paddle/phi/core/distributed/auto_parallel/
dist_tensor.h — a local DenseTensor + global dims + TensorDistAttr; the generated dist branch of every phi API —
InferSpmd, reshard the inputs, run the local kernel, set the outputs' dist attrs).

A ``DistTensor`` is a torch wrapper tensor of the GLOBAL shape that owns this rank's local shard, a ``MeshGroups``
(the ProcessMesh's communicators) and one placement per mesh dimension.  Autograd sees it as an ordinary tensor;
every aten op that reaches it (forward and backward) comes to ``__torch_dispatch__``, which

  1. infers the op's input / output placements from its SPMD rule (matmul, elementwise with broadcasting and
     partial-sum algebra, reductions, softmax, layer norm, views, embedding, ... below);
  2. reshards every input to the placements the rule asks for with the framework's reshard engine
     (``reshard.reshard_local``: all-gather / all-reduce / reduce-scatter / all-to-all over the mesh dim's group);
  3. runs the op on the local shards;
  4. wraps the local results with the rule's output placements.

Ops without a rule run replicated (inputs gathered, outputs replicated) — always correct, never silent.  The
framework's fused ops (linear, norms, RoPE, flash attention, SwiGLU, embedding) dispatch one level higher, at op
entry (``dist_ops.py``), so their native HIP kernels run on the local shards.
"""
from __future__ import annotations

import math

import torch
from torch.utils import _pytree as pytree

from .placement import Partial, Replicate, Shard, local_shape_and_offset

aten = torch.ops.aten
TRACE = []   # (aten op name, input placements, output placements) for the tests


def _contig_stride(shape):
    st, acc = [], 1
    for s in reversed(list(shape)):
        st.append(acc)
        acc *= max(int(s), 1)
    return tuple(reversed(st))


class DistTensor(torch.Tensor):
    _local_tensor: torch.Tensor

    @staticmethod
    def __new__(cls, local, mesh, placements, shape, requires_grad=False):
        shape = tuple(int(s) for s in shape)
        r = torch.Tensor._make_wrapper_subclass(cls, shape, strides=_contig_stride(shape), dtype=local.dtype,
                                                device=local.device, requires_grad=requires_grad)
        r._local_tensor = local
        r._mesh = mesh
        r._placements = tuple(placements)
        return r

    __torch_function__ = torch._C._disabled_torch_function_impl

    # ---------------------------------------------------------------- metadata
    @property
    def device_mesh(self):
        return self._mesh

    @property
    def placements(self):
        return self._placements

    def __repr__(self):
        return (f"DistTensor(shape={list(self.shape)}, dtype={self.dtype}, placements={list(self._placements)}, "
                f"mesh={self._mesh}, local={self._local_tensor})")

    # ---------------------------------------------------------------- conversions (differentiable)
    def to_local(self, grad_placements=None):
        return _ToLocal.apply(self, grad_placements)

    @staticmethod
    def from_local(local, mesh, placements, run_check=False, shape=None, stride=None):
        placements = tuple(placements) + (Replicate(),) * (mesh.ndim - len(placements))
        if shape is None:
            shape = list(local.shape)
            for d, p in enumerate(placements):
                if isinstance(p, Shard):
                    shape[p.dim % len(shape)] *= mesh.size(d)
        return _FromLocal.apply(local, mesh, placements, tuple(shape))

    def full_tensor(self):
        from .reshard import reshard

        return reshard(self, (Replicate(),) * self._mesh.ndim).to_local()

    def redistribute(self, mesh=None, placements=None):
        from .reshard import reshard

        return reshard(self, tuple(placements))

    # ---------------------------------------------------------------- dispatch
    @classmethod
    def __torch_dispatch__(cls, func, types, args=(), kwargs=None):
        return _dispatch(func, args, kwargs or {})


class _ToLocal(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dt, grad_placements):
        ctx.mesh, ctx.shape = dt._mesh, tuple(dt.shape)
        ctx.gpl = tuple(grad_placements) if grad_placements is not None else dt._placements
        return dt._local_tensor.view_as(dt._local_tensor)

    @staticmethod
    def backward(ctx, g):
        return DistTensor(g.contiguous(), ctx.mesh, ctx.gpl, ctx.shape), None


class _FromLocal(torch.autograd.Function):
    @staticmethod
    def forward(ctx, local, mesh, placements, shape):
        ctx.mesh, ctx.pl = mesh, placements
        return DistTensor(local.view_as(local), mesh, placements, shape)

    @staticmethod
    def backward(ctx, g):
        from .reshard import reshard_local

        if isinstance(g, DistTensor):
            # the gradient's piece under the forward placements (a replicated gradient of a partial input stays
            # replicated: see reshard_local's backward mode)
            return reshard_local(g._local_tensor, ctx.mesh, g._placements, ctx.pl, backward=True), None, None, None
        # a plain (replicated, full) gradient: this rank's piece of it
        local = reshard_local(g, ctx.mesh, (Replicate(),) * ctx.mesh.ndim, ctx.pl, backward=True)
        return local, None, None, None


def distribute_tensor(t, mesh, placements):
    """A full tensor, identical on every rank -> DistTensor with ``placements`` (slicing only, no communication)."""
    from .reshard import reshard_local

    placements = tuple(placements) + (Replicate(),) * (mesh.ndim - len(placements))
    local = reshard_local(t.detach(), mesh, (Replicate(),) * mesh.ndim, placements)
    return DistTensor(local, mesh, placements, tuple(t.shape), requires_grad=t.requires_grad)


# =============================================================================================== SPMD dispatch
def _axis_of(p, nd):
    return p.dim % nd if isinstance(p, Shard) and nd > 0 else None


def _replicated(n):
    return (Replicate(),) * n


class _Plan:
    """A rule's verdict: required placements per DistTensor-position input, output placements per output."""

    def __init__(self, ins, outs, local_fn=None):
        self.ins, self.outs, self.local_fn = ins, outs, local_fn


def _reshard_to(x, pl):
    from .reshard import reshard_local

    if not isinstance(x, DistTensor):
        return x
    pl = tuple(pl)
    if pl == x._placements:
        return x._local_tensor
    return reshard_local(x._local_tensor, x._mesh, x._placements, pl)


def _shape_of(x):
    return tuple(x.shape) if isinstance(x, torch.Tensor) else ()


def _out_shape(func, args, kwargs):
    """Global output shapes from meta tensors of the global shapes."""
    def to_meta(a):
        if isinstance(a, torch.Tensor):
            return torch.empty(a.shape, dtype=a.dtype, device="meta")
        return a

    margs, mkwargs = pytree.tree_map(to_meta, (args, kwargs))
    try:
        out = func(*margs, **mkwargs)
    except Exception:   # noqa: BLE001 - ops without a meta kernel: derived from the local result instead
        return None
    return out


# --------------------------------------------------------------------------- rules
def _pointwise_rule(func, args, kwargs, dts, nd_mesh):
    """Elementwise with numpy broadcasting.  Per mesh dim: a shard of an output axis is kept if the first input
    that carries it has the full axis; partial inputs stay partial through linear combinations (add / sub of
    partials, scaling by a non-partial operand), everything else is reduced first."""
    out_nd = max(x.dim() for x in dts)
    tensors = [a for a in pytree.tree_leaves((args, kwargs)) if isinstance(a, torch.Tensor)]
    name = func.overloadpacket.__name__
    ins = {id(x): list(x._placements) for x in dts}
    outp = []
    for d in range(nd_mesh):
        # shard candidate from the first dist input sharded on d
        cand = None
        for x in dts:
            p = x._placements[d]
            if isinstance(p, Shard):
                a = _axis_of(p, x.dim()) + out_nd - x.dim()
                cand = a
                break
        partial_in = [x for x in dts if isinstance(x._placements[d], Partial)]
        keep_partial = False
        if partial_in and cand is None:
            red = {x._placements[d].reduce_op for x in partial_in}
            if red == {"sum"}:
                if name in ("add", "sub", "add_", "sub_") and len(partial_in) == len(tensors):
                    keep_partial = True
                elif name in ("mul", "mul_", "neg", "neg_", "clone", "_to_copy", "alias", "detach", "view_as",
                              "div", "div_", "copy_") and len(partial_in) == 1:
                    px = partial_in[0]
                    keep_partial = not (name in ("div", "div_") and len(tensors) > 1 and tensors[0] is not px)
        for x in dts:
            p = x._placements[d]
            if cand is not None:
                xa = cand - (out_nd - x.dim())
                if xa >= 0 and x.shape[xa] == (max(t.shape[cand - (out_nd - t.dim())] for t in dts
                                                   if cand - (out_nd - t.dim()) >= 0)) and x.shape[xa] != 1:
                    ins[id(x)][d] = Shard(xa)
                else:
                    ins[id(x)][d] = Replicate()
            elif isinstance(p, Partial):
                ins[id(x)][d] = p if keep_partial else Replicate()
            else:
                ins[id(x)][d] = Replicate()
        if cand is not None:
            outp.append(Shard(cand))
        elif keep_partial:
            outp.append(partial_in[0]._placements[d])
        else:
            outp.append(Replicate())
    return _Plan(ins, [tuple(outp)])


def _mm_rule(a, b, batch=False):
    """a [.., m, k] . b [.., k, n]; per mesh dim: m / n / batch shards pass through, a k shard on both operands
    makes the output partial, a partial operand stays partial against a replicated one."""
    nd_mesh = a._mesh.ndim if isinstance(a, DistTensor) else b._mesh.ndim
    off = 1 if batch else 0
    pa = list(a._placements) if isinstance(a, DistTensor) else [Replicate()] * nd_mesh
    pb = list(b._placements) if isinstance(b, DistTensor) else [Replicate()] * nd_mesh
    ia, ib, out = [], [], []
    for d in range(nd_mesh):
        x, y = pa[d], pb[d]
        xa = x.dim if isinstance(x, Shard) else None
        ya = y.dim if isinstance(y, Shard) else None
        if batch and xa == 0 and ya in (0, None):
            ia.append(Shard(0)); ib.append(Shard(0)); out.append(Shard(0))
        elif xa == off + 1 or ya == off + 0:           # a contraction shard: both sides on k -> partial
            ia.append(Shard(off + 1)); ib.append(Shard(off + 0)); out.append(Partial())
        elif xa == off + 0:                             # rows of a
            ia.append(Shard(off + 0)); ib.append(Replicate()); out.append(Shard(off + 0))
        elif ya == off + 1:                             # columns of b
            ia.append(Replicate()); ib.append(Shard(off + 1)); out.append(Shard(off + 1))
        elif isinstance(x, Partial) and not isinstance(y, Partial):
            ia.append(x); ib.append(Replicate()); out.append(x)
        elif isinstance(y, Partial) and not isinstance(x, Partial):
            ia.append(Replicate()); ib.append(y); out.append(y)
        else:
            ia.append(Replicate()); ib.append(Replicate()); out.append(Replicate())
    return ia, ib, out


def _view_rule(x, out_shape):
    """Shards survive a view when the sharded axis starts a merge / split group at the same flat offset in the
    output and the output axis splits evenly; otherwise that axis is gathered first."""
    in_shape = list(x.shape)
    ins, outp = [], []
    for d, p in enumerate(x._placements):
        if isinstance(p, Shard):
            a = p.dim % len(in_shape)
            pre = math.prod(in_shape[:a])
            j, acc = 0, 1
            while j < len(out_shape) and acc < pre:
                acc *= out_shape[j]
                j += 1
            n = x._mesh.size(d)
            ok = acc == pre and j < len(out_shape)
            if ok:
                # the sharded block must be the outermost factor of its group on both sides
                ok = out_shape[j] % n == 0 and in_shape[a] % n == 0 and (
                    out_shape[j] % in_shape[a] == 0 or in_shape[a] % out_shape[j] == 0)
            if ok:
                ins.append(p)
                outp.append(Shard(j))
                continue
            ins.append(Replicate())
            outp.append(Replicate())
        else:
            ins.append(p)
            outp.append(p)
    return ins, outp


def _local_view_shape(out_shape, outp, mesh):
    s = list(out_shape)
    for d, p in enumerate(outp):
        if isinstance(p, Shard):
            s[p.dim] //= mesh.size(d)
    return s


def _reduce_rule(x, dims, keepdim, mean=False):
    nd = x.dim()
    dims = sorted(set(dd % nd for dd in dims)) if dims else list(range(nd))
    ins, outp = [], []
    for p in x._placements:
        if isinstance(p, Shard):
            a = p.dim % nd
            if a in dims:
                ins.append(p)
                outp.append(Partial("avg" if mean else "sum"))
            else:
                ins.append(p)
                outp.append(Shard(a if keepdim else a - sum(1 for r in dims if r < a)))
        elif isinstance(p, Partial) and p.reduce_op == "sum":
            ins.append(p)
            outp.append(p)   # sum / mean of a partial sum is a partial sum
        else:
            ins.append(Replicate() if isinstance(p, Partial) else p)
            outp.append(Replicate() if isinstance(p, Partial) else p)
    return ins, outp


def _keep_axes_replicated(x, axes):
    """Placements of x with every shard of ``axes`` (and any partial) gathered."""
    nd = x.dim()
    out = []
    for p in x._placements:
        if isinstance(p, Shard) and p.dim % nd in axes:
            out.append(Replicate())
        elif isinstance(p, Partial):
            out.append(Replicate())
        else:
            out.append(p)
    return out


_POINTWISE_EXTRA = {"clone", "detach", "alias", "_to_copy", "copy_", "fill_", "zero_", "view_as", "where",
                    "masked_fill", "gelu_backward", "silu_backward", "threshold_backward", "sigmoid_backward",
                    "tanh_backward", "_softmax_backward_data_", "lerp", "addcmul", "addcdiv", "clamp", "clamp_"}
_LIKE = {"zeros_like", "ones_like", "empty_like", "full_like", "rand_like", "randn_like"}


def _dispatch(func, args, kwargs):
    name = func.overloadpacket.__name__
    mesh = next(a for a in pytree.tree_leaves((args, kwargs)) if isinstance(a, DistTensor))._mesh
    nd_mesh = mesh.ndim
    # plain tensors (not 0-d scalars) join replicated
    args, kwargs = pytree.tree_map_only(
        torch.Tensor, lambda t: t if isinstance(t, DistTensor) or t.dim() == 0 else
        DistTensor(t, mesh, _replicated(nd_mesh), t.shape), (args, kwargs))
    dts = [a for a in pytree.tree_leaves((args, kwargs)) if isinstance(a, DistTensor)]
    if name in ("new_zeros", "new_empty", "new_ones", "new_full", "new_empty_strided"):
        loc = func(args[0]._local_tensor, *args[1:], **kwargs)
        return DistTensor(loc, mesh, _replicated(nd_mesh), loc.shape)
    if func in (aten._local_scalar_dense.default, aten.equal.default, aten.is_same_size.default):
        full = pytree.tree_map_only(DistTensor, lambda t: _reshard_to(t, _replicated(nd_mesh)), (args, kwargs))
        return func(*full[0], **full[1])
    if func in (aten.detach.default, aten.alias.default, aten.clone.default, aten._to_copy.default) or name in _LIKE:
        x = args[0]
        loc = func(x._local_tensor, *args[1:], **kwargs)
        pl = tuple(Replicate() if (name in _LIKE and isinstance(p, Partial)) else p for p in x._placements)
        return DistTensor(loc, mesh, pl, x.shape, requires_grad=False)

    plan_in, outp, local_args, local_kwargs = None, None, None, None
    try:
        r = _rule(func, name, args, kwargs, dts, nd_mesh, mesh)
    except _Fallback:
        r = None
    if r is None:
        # no rule: run replicated
        local_args, local_kwargs = pytree.tree_map_only(DistTensor, lambda t: _reshard_to(t, _replicated(nd_mesh)),
                                                         (args, kwargs))
        out = func(*local_args, **local_kwargs)
        TRACE.append((name, "replicated-fallback"))
        return pytree.tree_map_only(torch.Tensor, lambda o: DistTensor(o, mesh, _replicated(nd_mesh), o.shape), out)
    local_args, local_kwargs, outp, shapes = r
    out = func(*local_args, **local_kwargs)
    TRACE.append((name, [list(x._placements) for x in dts], outp))
    if func._schema.is_mutable or name.endswith("_"):
        # in place: the first argument is the result; its placements were kept
        return args[0]
    flat, spec = pytree.tree_flatten(out)
    res, k = [], 0
    for o in flat:
        if isinstance(o, torch.Tensor):
            pl = outp[k] if k < len(outp) else outp[-1]
            shp = shapes[k] if shapes is not None and k < len(shapes) else None
            if shp is None:
                shp = list(o.shape)
                for d, p in enumerate(pl):
                    if isinstance(p, Shard):
                        shp[p.dim] *= mesh.size(d)
            res.append(DistTensor(o, mesh, tuple(pl), shp))
            k += 1
        else:
            res.append(o)
    return pytree.tree_unflatten(res, spec)


class _Fallback(Exception):
    pass


def _global_out_shapes(func, args, kwargs):
    m = _out_shape(func, args, kwargs)
    if m is None:
        return None
    return [tuple(t.shape) for t in pytree.tree_leaves(m) if isinstance(t, torch.Tensor)]


def _apply(args, kwargs, want):
    """Reshard every DistTensor argument to want[id(t)] (or keep it) and replace it by its local tensor."""
    def f(t):
        pl = want.get(id(t))
        return _reshard_to(t, pl if pl is not None else t._placements)
    return pytree.tree_map_only(DistTensor, f, (args, kwargs))


def _rule(func, name, args, kwargs, dts, nd_mesh, mesh):
    """-> (local args, local kwargs, output placements per tensor output, global output shapes) or None."""
    shapes = _global_out_shapes(func, args, kwargs)
    if name in ("mm", "bmm"):
        a, b = args[0], args[1]
        ia, ib, out = _mm_rule(a, b, batch=(name == "bmm"))
        la, lk = _apply(args, kwargs, {id(a): ia, id(b): ib})
        return la, lk, [tuple(out)], shapes
    if name in ("addmm",):
        bias, a, b = args[0], args[1], args[2]
        ia, ib, out = _mm_rule(a, b)
        la, lk = _apply(args, kwargs, {id(a): ia, id(b): ib})
        # bias [n] follows the output: sliced where the output's columns are sharded, added once where partial
        lb = la[1] if not isinstance(bias, DistTensor) else _reshard_to(bias, _replicated(nd_mesh))
        for d, p in enumerate(out):
            if isinstance(p, Shard) and p.dim == 1:
                lb = lb.chunk(mesh.size(d), dim=-1)[mesh.get_local_rank(d)]
            elif isinstance(p, Partial) and mesh.get_local_rank(d) != 0:
                lb = torch.zeros_like(lb)
        la = (lb,) + tuple(la[1:])
        return la, lk, [tuple(out)], shapes
    if name in ("t", "transpose", "permute"):
        x = args[0]
        nd = x.dim()
        if name == "t":
            perm = list(range(nd))[::-1]
        elif name == "transpose":
            perm = list(range(nd))
            i, j = args[1] % nd, args[2] % nd
            perm[i], perm[j] = perm[j], perm[i]
        else:
            perm = [p % nd for p in args[1]]
        outp = [Shard(perm.index(p.dim % nd)) if isinstance(p, Shard) else p for p in x._placements]
        la, lk = _apply(args, kwargs, {})
        return la, lk, [tuple(outp)], shapes
    if name in ("view", "_unsafe_view", "reshape"):
        x = args[0]
        out_shape = list(shapes[0]) if shapes else list(args[1])
        ins, outp = _view_rule(x, out_shape)
        lx = _reshard_to(x, ins)
        if not lx.is_contiguous():   # the global view is of a contiguous tensor; the local shard may be strided
            lx = lx.contiguous()
        return (lx, _local_view_shape(out_shape, outp, mesh)) + tuple(args[2:]), kwargs, [tuple(outp)], shapes
    if name in ("unsqueeze", "squeeze", "expand", "slice", "select", "split", "split_with_sizes", "unbind", "cat",
                "stack", "index_select", "gather", "scatter_add", "index_add", "index_put", "nonzero", "sort",
                "topk", "argmax", "argmin", "max", "min", "cumsum", "flip", "roll", "repeat", "pad",
                "constant_pad_nd", "embedding_dense_backward", "nll_loss_forward", "nll_loss_backward",
                "native_dropout", "native_dropout_backward"):
        return _unsqueeze_like(func, name, args, kwargs, dts, nd_mesh, mesh, shapes)
    if name in ("sum", "mean"):
        x = args[0]
        dims = args[1] if len(args) > 1 else kwargs.get("dim")
        keepdim = args[2] if len(args) > 2 else kwargs.get("keepdim", False)
        if dims is None or (isinstance(dims, (list, tuple)) and len(dims) == 0):
            dims = list(range(x.dim()))
        dims = [dims] if isinstance(dims, int) else list(dims)
        ins, outp = _reduce_rule(x, dims, keepdim, mean=(name == "mean"))
        la, lk = _apply(args, kwargs, {id(x): ins})
        return la, lk, [tuple(outp)], shapes
    if name in ("_softmax", "_log_softmax"):
        x = args[0]
        ins = _keep_axes_replicated(x, {args[1] % x.dim()})
        la, lk = _apply(args, kwargs, {id(x): ins})
        return la, lk, [tuple(ins)], shapes
    if name in ("_softmax_backward_data", "_log_softmax_backward_data"):
        g, y = args[0], args[1]
        axis = args[2] % y.dim()
        pl = _keep_axes_replicated(y, {axis})
        la, lk = _apply(args, kwargs, {id(g): pl, id(y): pl})
        return la, lk, [tuple(pl)], shapes
    if name == "native_layer_norm":
        x, normalized = args[0], args[1]
        axes = set(range(x.dim() - len(normalized), x.dim()))
        pl = _keep_axes_replicated(x, axes)
        want = {id(x): pl}
        for w in args[2:4]:
            if isinstance(w, DistTensor):
                want[id(w)] = _replicated(nd_mesh)
        la, lk = _apply(args, kwargs, want)
        return la, lk, [tuple(pl)] * 3, shapes
    if name == "native_layer_norm_backward":
        g, x, normalized, mean, rstd, w, b = args[:7]
        axes = set(range(x.dim() - len(normalized), x.dim()))
        pl = _keep_axes_replicated(x, axes)
        want = {id(g): pl, id(x): pl, id(mean): pl, id(rstd): pl}
        for t in (w, b):
            if isinstance(t, DistTensor):
                want[id(t)] = _replicated(nd_mesh)
        la, lk = _apply(args, kwargs, want)
        wpl = tuple(Partial() if isinstance(p, Shard) else Replicate() for p in pl)
        return la, lk, [tuple(pl), wpl, wpl], shapes
    if name == "embedding":
        w, ids = args[0], args[1]
        wpl = list(w._placements) if isinstance(w, DistTensor) else list(_replicated(nd_mesh))
        ipl = list(ids._placements) if isinstance(ids, DistTensor) else list(_replicated(nd_mesh))
        outp, wn, idn = [], [], []
        for d in range(nd_mesh):
            pw, pi = wpl[d], ipl[d]
            if isinstance(pw, Shard) and pw.dim == 1 and not isinstance(pi, Shard):
                wn.append(pw); idn.append(Replicate()); outp.append(Shard(ids.dim()))
            elif isinstance(pi, Shard):
                wn.append(Replicate()); idn.append(pi); outp.append(Shard(pi.dim))
            else:
                wn.append(Replicate()); idn.append(Replicate()); outp.append(Replicate())
        la, lk = _apply(args, kwargs, {id(w): wn, id(ids): idn})
        return la, lk, [tuple(outp)], shapes
    if torch.Tag.pointwise in func.tags or name in _POINTWISE_EXTRA:
        plan = _pointwise_rule(func, args, kwargs, dts, nd_mesh)
        if func._schema.is_mutable or name.endswith("_"):
            self_ = args[0]
            # in place: self keeps its placements; the rest follow self
            want = {id(x): _follow(x, self_, name) for x in dts}
            want[id(self_)] = self_._placements
            la, lk = _apply(args, kwargs, want)
            return la, lk, [self_._placements], shapes
        la, lk = _apply(args, kwargs, plan.ins)
        return la, lk, plan.outs, shapes
    return None


def _follow(x, self_, name):
    """Placements of operand x of an in-place op on ``self_`` (broadcast-aligned shards follow self).  Into a partial
    self an add / sub operand goes as a partial term (a replicated value is kept on one rank only, so it is counted
    once); a scaling operand goes replicated."""
    out = []
    off = self_.dim() - x.dim()
    for p in self_._placements:
        if isinstance(p, Shard):
            a = p.dim - off
            out.append(Shard(a) if a >= 0 and x.shape[a] == self_.shape[p.dim] and x.shape[a] != 1 else Replicate())
        elif isinstance(p, Partial):
            out.append(p if name in ("add_", "sub_", "copy_") else Replicate())
        else:
            out.append(Replicate())
    return out


def _unsqueeze_like(func, name, args, kwargs, dts, nd_mesh, mesh, shapes):
    """Shape ops that touch given axes: shards on untouched leading axes survive, touched ones are gathered."""
    x = args[0] if isinstance(args[0], DistTensor) else None
    if name in ("unsqueeze", "squeeze") and x is not None:
        nd = x.dim()
        if name == "unsqueeze":
            ax = args[1] % (nd + 1)
            outp = [Shard(p.dim + (1 if p.dim >= ax else 0)) if isinstance(p, Shard) else p for p in x._placements]
            la, lk = _apply(args, kwargs, {})
            return la, lk, [tuple(outp)], shapes
        dims = args[1] if len(args) > 1 else list(range(nd))
        dims = [dims] if isinstance(dims, int) else list(dims)
        dims = [d % nd for d in dims if x.shape[d % nd] == 1]
        outp = [Shard(p.dim - sum(1 for d in dims if d < p.dim)) if isinstance(p, Shard) else p
                for p in x._placements]
        la, lk = _apply(args, kwargs, {})
        return la, lk, [tuple(outp)], shapes
    if name == "expand" and x is not None:
        size = list(args[1])
        off = len(size) - x.dim()
        ins, outp, loc = [], [], list(size)
        for d, p in enumerate(x._placements):
            if isinstance(p, Shard) and x.shape[p.dim] == size[p.dim + off]:
                ins.append(p); outp.append(Shard(p.dim + off))
                loc[p.dim + off] //= mesh.size(d)
            elif isinstance(p, Partial):
                ins.append(p); outp.append(p)
            else:
                ins.append(Replicate()); outp.append(Replicate())
        lx = _reshard_to(x, ins)
        return (lx, loc) + tuple(args[2:]), kwargs, [tuple(outp)], shapes
    if name == "embedding_dense_backward":
        g, ids = args[0], args[1]
        gpl = list(g._placements)
        ins_g, ins_i, outp = [], [], []
        ipl = list(ids._placements) if isinstance(ids, DistTensor) else list(_replicated(nd_mesh))
        for d in range(nd_mesh):
            pg, pi = gpl[d], ipl[d]
            if isinstance(pi, Shard) and isinstance(pg, Shard) and pg.dim == pi.dim:
                ins_g.append(pg); ins_i.append(pi); outp.append(Partial())
            elif isinstance(pg, Shard) and pg.dim == g.dim() - 1 and not isinstance(pi, Shard):
                ins_g.append(pg); ins_i.append(Replicate()); outp.append(Shard(1))
            elif isinstance(pg, Partial) and not isinstance(pi, Shard):
                ins_g.append(pg); ins_i.append(Replicate()); outp.append(pg)
            else:
                ins_g.append(Replicate()); ins_i.append(Replicate()); outp.append(Replicate())
        la, lk = _apply(args, kwargs, {id(g): ins_g, id(ids): ins_i})
        return la, lk, [tuple(outp)], shapes
    if name in ("slice", "select", "split", "split_with_sizes", "unbind", "flip", "roll", "cumsum") \
            and x is not None:
        nd = x.dim()
        if name in ("slice", "select", "cumsum"):
            axis = args[1] if len(args) > 1 else kwargs.get("dim", 0)
        elif name in ("split", "split_with_sizes"):   # (self, split_size(s), dim=0)
            axis = args[2] if len(args) > 2 else kwargs.get("dim", 0)
        elif name == "unbind":
            axis = args[1] if len(args) > 1 else kwargs.get("dim", 0)
        elif name == "flip":
            axis = list(args[1])
        else:   # roll(x, shifts, dims)
            axis = list(args[2]) if len(args) > 2 and args[2] else list(range(nd))
        axes = {a % nd for a in (axis if isinstance(axis, (list, tuple)) else [axis])}
        ins = []
        for p in x._placements:
            ins.append(Replicate() if (isinstance(p, Shard) and p.dim % nd in axes) else p)
        if name in ("select", "unbind"):
            a = next(iter(axes))
            outp = [Shard(p.dim - (1 if p.dim > a else 0)) if isinstance(p, Shard) else p for p in ins]
        else:
            outp = ins
        la, lk = _apply(args, kwargs, {id(x): ins})
        return la, lk, [tuple(outp)], shapes
    if name in ("cat", "stack"):
        ts = [t for t in args[0]]
        dim = args[1] if len(args) > 1 else kwargs.get("dim", 0)
        ref = next(t for t in ts if isinstance(t, DistTensor))
        nd = ref.dim()
        a = dim % (nd + (1 if name == "stack" else 0))
        base = [Replicate() if (isinstance(p, Shard) and p.dim == a and name == "cat") or isinstance(p, Partial)
                else p for p in ref._placements]
        want = {id(t): base for t in ts if isinstance(t, DistTensor)}
        la, lk = _apply(args, kwargs, want)
        outp = base if name == "cat" else [Shard(p.dim + (1 if p.dim >= a else 0)) if isinstance(p, Shard) else p
                                           for p in base]
        return la, lk, [tuple(outp)], shapes
    raise _Fallback()
