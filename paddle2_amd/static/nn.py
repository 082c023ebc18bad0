"""paddle.static.nn: layer helpers that create parameters and record ops (reference: static/nn/common.py)."""
from __future__ import annotations

from .. import nn as _nn
from ..nn import functional as F


def fc(x, size, num_flatten_dims=1, weight_attr=None, bias_attr=None, activation=None, name=None):
    in_dim = 1
    for d in x.shape[num_flatten_dims:]:
        in_dim *= d
    lin = _nn.Linear(in_dim, size, weight_attr=weight_attr, bias_attr=bias_attr)
    h = x.reshape(list(x.shape[:num_flatten_dims]) + [in_dim]) if len(x.shape) > num_flatten_dims + 1 else x
    y = lin(h)
    if activation:
        y = getattr(F, activation)(y)
    return y


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None, param_attr=None, dtype="float32"):
    return _nn.Embedding(size[0], size[1], padding_idx=padding_idx, weight_attr=param_attr)(input)


def conv2d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=1, param_attr=None,
           bias_attr=None, act=None, name=None, data_format="NCHW"):
    c = _nn.Conv2D(input.shape[1], num_filters, filter_size, stride, padding, dilation, groups,
                   weight_attr=param_attr, bias_attr=bias_attr, data_format=data_format)
    y = c(input)
    return getattr(F, act)(y) if act else y


def batch_norm(input, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None, bias_attr=None,
               data_layout="NCHW", name=None, **kw):
    bn = _nn.BatchNorm2D(input.shape[1], momentum=momentum, epsilon=epsilon, weight_attr=param_attr,
                         bias_attr=bias_attr, data_format=data_layout)
    if is_test:
        bn.eval()
    y = bn(input)
    return getattr(F, act)(y) if act else y


def layer_norm(input, scale=True, shift=True, begin_norm_axis=1, epsilon=1e-05, param_attr=None, bias_attr=None,
               act=None, name=None):
    shp = list(input.shape[begin_norm_axis:])
    ln = _nn.LayerNorm(shp, epsilon=epsilon, weight_attr=param_attr if scale else False,
                       bias_attr=bias_attr if shift else False)
    y = ln(input)
    return getattr(F, act)(y) if act else y


# ------------------------------------------------------------------------------------------ control flow
def _is_sym(t):
    from .graph import SymTensor

    tt = t._t if hasattr(t, "_t") else t
    return isinstance(tt, SymTensor)


def _flat(out):
    import torch.utils._pytree as pytree

    return pytree.tree_flatten(out)


def cond(pred, true_fn=None, false_fn=None, name=None, return_names=None):
    """paddle.static.nn.cond (reference static/nn/control_flow.py cond).  Eager / Python predicate: runs the
    chosen branch.  Symbolic predicate (inside a recorded Program): BOTH branches are recorded and every
    output is selected with ``where(pred, true_out, false_out)`` — exact for side-effect-free branches (the
    dy2static contract), static shapes, and no sub-block machinery in the executor."""
    import torch

    from ..framework.tensor import Tensor

    if not _is_sym(pred):
        p = pred
        if isinstance(p, Tensor):
            p = bool(p._t.reshape(-1)[0]) if p._t.numel() else False
        return (true_fn() if true_fn is not None else None) if p else (false_fn() if false_fn is not None else None)
    t_out = true_fn() if true_fn is not None else None
    f_out = false_fn() if false_fn is not None else None
    tl, tspec = _flat(t_out)
    fl, fspec = _flat(f_out)
    if tspec != fspec:
        raise ValueError(f"cond: true_fn and false_fn must return the same structure ({tspec} vs {fspec})")
    import torch.utils._pytree as pytree

    pt = pred._t
    outs = []
    for a, b in zip(tl, fl):
        if isinstance(a, Tensor) or isinstance(b, Tensor):
            at = a._t if isinstance(a, Tensor) else torch.as_tensor(a)
            bt = b._t if isinstance(b, Tensor) else torch.as_tensor(b)
            outs.append(Tensor._wrap(torch.where(pt.reshape([]) if pt.dim() else pt, at, bt)))
        else:
            if a != b:
                raise ValueError("cond: non-tensor outputs of the two branches differ under a symbolic predicate")
            outs.append(a)
    return pytree.tree_unflatten(outs, tspec)


class _WhileRunner:
    """Executes a recorded while-loop: ``cond_prog`` / ``body_prog`` are sub-Programs over placeholder loop
    variables; the loop runs them (through the Executor's replay) until the predicate is false."""

    def __init__(self, cond_prog, body_prog, in_vids, cond_out, body_outs, free_vids):
        self.cond_prog, self.body_prog = cond_prog, body_prog
        self.in_vids, self.cond_out, self.body_outs = in_vids, cond_out, body_outs
        self.free_vids = free_vids  # outer-program values the loop reads (loop invariants)
        self.__qualname__ = self.__name__ = "while_loop"

    def __call__(self, *vals):
        n = len(self.in_vids)
        loop, free = list(vals[:n]), list(vals[n:])
        if loop and loop[0].device.type == "meta":  # shape inference while recording: loop vars keep their metas
            return tuple(v.clone() for v in loop)
        import torch

        from .executor import Executor

        exe = Executor.__new__(Executor)
        inv = dict(zip(self.free_vids, free))
        grad = torch.is_grad_enabled()  # a training replay differentiates through every iteration
        while True:
            env = exe._replay(self.cond_prog, {**inv, **dict(zip(self.in_vids, loop))})
            if not bool(env[self.cond_out].reshape(-1)[0]):
                return tuple(loop)
            env = exe._replay(self.body_prog, {**inv, **dict(zip(self.in_vids, loop))}, grad=grad)
            loop = [env[v] for v in self.body_outs]


def while_loop(cond, body, loop_vars, is_test=False, name=None):
    """paddle.static.nn.while_loop (reference static/nn/control_flow.py while_loop): eager -> a Python loop;
    symbolic loop variables -> ONE recorded op whose sub-programs (cond, body) the executor iterates."""
    from ..framework.tensor import Tensor
    from .graph import Program, default_main_program, program_guard

    loop_vars = list(loop_vars)
    if not any(_is_sym(v) for v in loop_vars):
        while True:
            c = cond(*loop_vars)
            if _is_sym(c):  # concrete initial state, symbolic predicate (reads a feed): record the loop
                break
            if isinstance(c, Tensor):
                c = bool(c._t.reshape(-1)[0])
            if not c:
                return loop_vars
            out = body(*loop_vars)
            loop_vars = list(out) if isinstance(out, (list, tuple)) else [out]
    outer = default_main_program()

    def sub(fn):
        p = Program()
        with program_guard(p, Program()):
            ph = []
            for i, v in enumerate(loop_vars):
                m = v._t
                s = p.new_var(m.new_empty(m.shape, device="meta") if m.device.type != "meta" else m.clone(),
                              name=f"loop_var_{i}")
                ph.append(Tensor._wrap(s))
            out = fn(*ph)
        return p, [t._t._vid for t in ph], out

    import torch.utils._pytree as pytree

    from .graph import VarRef

    cp, cvids, c_out = sub(cond)
    bp, bvids, b_out = sub(body)
    b_out = list(b_out) if isinstance(b_out, (list, tuple)) else [b_out]
    # both sub-programs were traced with their own placeholders: map body placeholders onto the cond ones
    remap = dict(zip(bvids, cvids))
    for op in bp.ops:
        fix = lambda x: VarRef(remap.get(x.vid, x.vid)) if isinstance(x, VarRef) else x  # noqa: E731
        op.args = pytree.tree_map(fix, op.args)
        op.kwargs = pytree.tree_map(fix, op.kwargs)
    body_outs = [remap.get(o._t._vid, o._t._vid) for o in b_out]
    # loop invariants: values of the OUTER program the sub-programs read (closures in cond / body)
    free = []
    for p in (cp, bp):
        produced = {v for op in p.ops for v in op.outs if v is not None}
        for op in p.ops:
            for x in pytree.tree_leaves((op.args, op.kwargs)):
                if isinstance(x, VarRef) and x.vid not in produced and x.vid not in cvids and x.vid not in free:
                    free.append(x.vid)
    runner = _WhileRunner(cp, bp, cvids, c_out._t._vid, body_outs, free)
    args = tuple(v._t for v in loop_vars) + tuple(outer.vars[v] for v in free)
    res = outer._record(runner, args, {}, kind="native")
    return [Tensor._wrap(r) for r in res]
