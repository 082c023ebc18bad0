"""Static auto-parallel: completion (reference python/paddle/distributed/auto_parallel/static/completion.py,
``Completer.complete_forward_annotation``) — propagate distributed attributes through a recorded Program.

Input: a ``static.Program`` (the framework's recorded op list: every op is a torch / native callable over
``VarRef`` symbolic inputs and concrete parameter tensors) plus user annotations for some tensors (feeds by
name, parameters by object).  Output: a ``DistContext`` holding, for every tensor, its ``TensorDistAttr``
(dims_mapping + partial mesh dims + the partial reduction) and, for every op, the attributes its inputs must be
resharded to and the attributes of its outputs.  The per-op decision is the SPMD rule of that op
(``auto_parallel/spmd_rules.py`` — the same rules the dynamic DistTensor path uses); ops without a rule run
replicated.
"""
from __future__ import annotations

import torch
import torch.utils._pytree as pytree

from .. import spmd_rules as R
from ..api import Partial, ProcessMesh, Replicate, Shard

ELEMENTWISE = {"add", "sub", "mul", "div", "true_divide", "gelu", "relu", "silu", "tanh", "sigmoid", "exp", "neg",
               "pow", "rsqrt", "sqrt", "maximum", "minimum", "abs", "square", "clone", "contiguous", "to",
               "type_as", "float", "bfloat16", "half", "dropout", "log", "erf", "scale", "swish", "relu6",
               "leaky_relu", "elu", "softplus", "mish", "hardswish", "hardsigmoid", "rsub", "add_", "mul_"}
LINEAR_PARTIAL = {"add", "sub"}  # partial + partial stays partial


def op_key(op):
    """Short op name: ``_VariableFunctionsClass.addmm`` -> ``addmm``, ``TensorBase.add`` -> ``add``."""
    return op.name.rsplit(".", 1)[-1].lower()


class DistAttr:
    """dims_mapping (tensor axis -> mesh dim, -1 replicated) + partial mesh dims with their reduction."""

    __slots__ = ("dims_mapping", "partial", "reduce")

    def __init__(self, dims_mapping, partial=(), reduce="sum"):
        self.dims_mapping = list(dims_mapping)
        self.partial = set(partial)
        self.reduce = reduce

    def placements(self, ndim_mesh):
        """placements per mesh dim (for the reshard engine)."""
        from ..placement import Partial as TP
        from ..placement import Replicate as TR
        from ..placement import Shard as TS

        out = []
        for d in range(ndim_mesh):
            if d in self.partial:
                out.append(TP(self.reduce))
            elif d in self.dims_mapping:
                out.append(TS(self.dims_mapping.index(d)))
            else:
                out.append(TR())
        return tuple(out)

    def same(self, o):
        return (self.dims_mapping == o.dims_mapping and self.partial == o.partial
                and (not self.partial or self.reduce == o.reduce))

    def __repr__(self):
        p = f", partial={sorted(self.partial)}({self.reduce})" if self.partial else ""
        return f"DistAttr({self.dims_mapping}{p})"


def attr_from_placements(placements, ndim):
    dm = [-1] * ndim
    partial, red = set(), "sum"
    for d, p in enumerate(placements):
        if isinstance(p, Shard):
            dm[p.get_dim() if hasattr(p, "get_dim") else p.dim] = d
        elif isinstance(p, Partial):
            partial.add(d)
            red = p.reduce_op
    return DistAttr(dm, partial, red)


class OpPlan:
    __slots__ = ("key", "in_attrs", "out_attrs", "split_dims")

    def __init__(self, key, in_attrs, out_attrs):
        self.key, self.in_attrs, self.out_attrs = key, in_attrs, out_attrs
        # mesh dims on which this op computes different data per coordinate: a replicated input's gradient is
        # PARTIAL over them (the conjugate all-reduce of Megatron's column-parallel input)
        dims = set()
        for a in list(in_attrs) + list(out_attrs):
            if a is None:
                continue
            dims |= {d for d in a.dims_mapping if d != -1} | a.partial
        self.split_dims = dims


class DistContext:
    def __init__(self, program, mesh):
        self.program, self.mesh = program, mesh
        self.attrs = {}      # tensor key -> DistAttr (as produced / stored)
        self.plans = []      # per op: OpPlan

    def attr(self, key):
        return self.attrs.get(key)


def tensor_key(x):
    from ....static.graph import VarRef

    if isinstance(x, VarRef):
        return ("v", x.vid)
    return ("p", id(x))


def _is_tensor_leaf(x):
    from ....static.graph import VarRef

    return isinstance(x, VarRef) or (isinstance(x, torch.Tensor) and x.dim() > 0)


class Completer:
    """Forward completion over one Program (reference Completer)."""

    def __init__(self, mesh: ProcessMesh):
        self.mesh = mesh

    def _shape(self, prog, x):
        from ....static.graph import VarRef

        return list(prog.vars[x.vid].shape) if isinstance(x, VarRef) else list(x.shape)

    def _spec(self, shape, attr):
        return R.DistTensorSpec(shape, R.TensorDistAttr(attr.dims_mapping, self.mesh, attr.partial))

    def _rule(self, key, op, specs, attrs):
        """-> (required input DistAttrs, output DistAttrs) for the op's tensor leaves / outputs."""
        n = len(specs)

        def conv(ta, reduce="sum"):
            return DistAttr(ta.dims_mapping, ta._partial_dims(), reduce)

        args = op.args
        if key in ("addmm",) and n == 3:
            ins, outs = R.matmul_forward(specs[1], specs[2])
            o = outs[0]
            bias = DistAttr([o.dims_mapping[-1]] if len(specs[0].shape) == 1 else o.dims_mapping)
            return [bias, conv(ins[0]), conv(ins[1])], [conv(o)]
        if key in ("mm", "matmul", "bmm") and n == 2:
            ins, outs = R.matmul_forward(specs[0], specs[1])
            return [conv(a) for a in ins], [conv(outs[0])]
        if key == "linear" and n >= 2:
            ins, outs = R.matmul_forward(specs[0], specs[1], trans_y=True)
            o = outs[0]
            res = [conv(ins[0]), conv(ins[1])]
            if n == 3:
                res.append(DistAttr([o.dims_mapping[-1]]))
            return res, [conv(o)]
        if key in ("softmax", "log_softmax", "_softmax"):
            axis = args[1] if len(args) > 1 and isinstance(args[1], int) else op.kwargs.get("dim", -1)
            ins, outs = R.softmax_forward(specs[0], axis)
            return [conv(ins[0])] + [DistAttr([-1] * len(s.shape)) for s in specs[1:]], [conv(outs[0])]
        if key in ("sum", "mean") and n == 1:
            axis = args[1] if len(args) > 1 and isinstance(args[1], (int, list, tuple)) else op.kwargs.get("dim")
            keep = bool(args[2]) if len(args) > 2 and isinstance(args[2], bool) else bool(op.kwargs.get("keepdim",
                                                                                                         False))
            if isinstance(axis, tuple):
                axis = list(axis)
            ins, outs = R.reduction_forward(specs[0], axis, keep, key)
            return [conv(ins[0])], [conv(outs[0], "avg" if key == "mean" else "sum")]
        if key in ("layer_norm", "rms_norm") and n >= 1:
            x = specs[0]
            if key == "layer_norm":
                ins, outs = R.layer_norm_forward(x, specs[1] if n > 1 else None, specs[2] if n > 2 else None,
                                                 begin_norm_axis=len(x.shape) - 1)
            else:
                ins, outs = R.rms_norm_forward(x, specs[1] if n > 1 else None)
            req = [conv(ins[0])] + [DistAttr([-1] * len(s.shape)) for s in specs[1:]]
            return req, [conv(outs[0])] + [DistAttr([-1])] * (len(op.outs) - 1)
        if key in ("transpose", "permute") and n == 1:
            nd = len(specs[0].shape)
            if key == "transpose":
                a, b = args[1] % nd, args[2] % nd
                perm = list(range(nd))
                perm[a], perm[b] = perm[b], perm[a]
            else:
                perm = [p % nd for p in (args[1] if isinstance(args[1], (list, tuple)) else args[1:])]
            ins, outs = R.transpose_forward(specs[0], perm)
            return [conv(ins[0])], [conv(outs[0])]
        if key in ("reshape", "view") and n == 1:
            shape = list(args[1]) if isinstance(args[1], (list, tuple, torch.Size)) else list(args[1:])
            ins, outs = R.reshape_forward(specs[0], shape)
            return [conv(ins[0])], [conv(outs[0])]
        if key in ELEMENTWISE and n >= 1:
            if key in LINEAR_PARTIAL and n == 2 and all(a.partial for a in attrs) and \
                    attrs[0].same(attrs[1]) and list(specs[0].shape) == list(specs[1].shape):
                return [attrs[0], attrs[1]], [DistAttr(attrs[0].dims_mapping, attrs[0].partial, attrs[0].reduce)]
            ins, outs = R.elementwise_forward(*specs)
            return [conv(a) for a in ins], [conv(outs[0])]
        return ([DistAttr([-1] * len(s.shape)) for s in specs],
                [DistAttr([-1] * len(self._out_meta(op, i).shape)) for i in range(len(op.outs))])

    def _out_meta(self, op, i):
        v = op.outs[i]
        return self._prog.vars[v] if v is not None else torch.empty(())

    def complete(self, program, annotations=None):
        """annotations: {feed name | Parameter / Tensor | vid: placements list or DistAttr}."""
        from ....framework.tensor import Tensor

        self._prog = program
        ctx = DistContext(program, self.mesh)
        for k, v in (annotations or {}).items():
            if isinstance(k, str):
                key = ("v", program.feeds[k]._vid)
                nd = program.feeds[k].dim()
            elif isinstance(k, int):
                key, nd = ("v", k), program.vars[k].dim()
            else:
                t = k._t if isinstance(k, Tensor) else k
                key, nd = ("p", id(t)), t.dim()
            ctx.attrs[key] = v if isinstance(v, DistAttr) else attr_from_placements(v, nd)
        for op in program.ops:
            if op.kind not in ("torch", "native"):
                ctx.plans.append(None)
                continue
            leaves = [x for x in pytree.tree_leaves((op.args, op.kwargs)) if _is_tensor_leaf(x)]
            shapes = [self._shape(program, x) for x in leaves]
            attrs = []
            for x, s in zip(leaves, shapes):
                a = ctx.attrs.get(tensor_key(x))
                if a is None:
                    a = DistAttr([-1] * len(s))
                    ctx.attrs[tensor_key(x)] = a
                attrs.append(a)
            specs = [self._spec(s, a) for s, a in zip(shapes, attrs)]
            key = op_key(op)
            try:
                ins, outs = self._rule(key, op, specs, attrs)
            except Exception:  # noqa: BLE001 — a rule that cannot handle this call: run the op replicated
                ins = [DistAttr([-1] * len(s)) for s in shapes]
                outs = [DistAttr([-1] * len(self._out_meta(op, i).shape)) for i in range(len(op.outs))]
            outs = list(outs) + [DistAttr([-1] * len(self._out_meta(op, i).shape))
                                 for i in range(len(outs), len(op.outs))]
            for i, v in enumerate(op.outs):
                if v is not None:
                    ctx.attrs[("v", v)] = outs[i]
            ctx.plans.append(OpPlan(key, ins, outs))
        return ctx
