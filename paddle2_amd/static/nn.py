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


def _act(y, act):
    return getattr(F, act)(y) if act else y


def conv2d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,
                     groups=1, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
                     data_format="NCHW"):
    if filter_size is None:
        if output_size is None:
            raise ValueError("conv2d_transpose: filter_size or output_size is required")
        # reference: filter = out - (in - 1) * stride + 2 * padding (per spatial dim, dilation 1)
        osz = [output_size] * 2 if isinstance(output_size, int) else list(output_size)
        st = [stride] * 2 if isinstance(stride, int) else list(stride)
        pd = [padding] * 2 if isinstance(padding, int) else list(padding)[:2]
        hw = input.shape[2:4] if data_format == "NCHW" else input.shape[1:3]
        filter_size = [osz[i] - (hw[i] - 1) * st[i] + 2 * pd[i] for i in range(2)]
    cin = input.shape[1] if data_format == "NCHW" else input.shape[-1]
    c = _nn.Conv2DTranspose(cin, num_filters, filter_size, stride, padding, dilation=dilation, groups=groups,
                            weight_attr=param_attr, bias_attr=bias_attr, data_format=data_format)
    return _act(c(input, output_size=output_size) if output_size is not None else c(input), act)


def conv3d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=1, param_attr=None,
           bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCDHW"):
    cin = input.shape[1] if data_format == "NCDHW" else input.shape[-1]
    c = _nn.Conv3D(cin, num_filters, filter_size, stride, padding, dilation, groups, weight_attr=param_attr,
                   bias_attr=bias_attr, data_format=data_format)
    return _act(c(input), act)


def conv3d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,
                     groups=1, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
                     data_format="NCDHW"):
    if filter_size is None:
        raise ValueError("conv3d_transpose: filter_size is required")
    cin = input.shape[1] if data_format == "NCDHW" else input.shape[-1]
    c = _nn.Conv3DTranspose(cin, num_filters, filter_size, stride, padding, dilation=dilation, groups=groups,
                            weight_attr=param_attr, bias_attr=bias_attr, data_format=data_format)
    return _act(c(input, output_size=output_size) if output_size is not None else c(input), act)


def group_norm(input, groups, epsilon=1e-05, param_attr=None, bias_attr=None, act=None, data_layout="NCHW",
               name=None):
    cin = input.shape[1] if data_layout == "NCHW" else input.shape[-1]
    gn = _nn.GroupNorm(groups, cin, epsilon=epsilon, weight_attr=param_attr, bias_attr=bias_attr,
                       data_format=data_layout)
    return _act(gn(input), act)


def instance_norm(input, epsilon=1e-05, param_attr=None, bias_attr=None, name=None):
    cls = {3: _nn.InstanceNorm1D, 4: _nn.InstanceNorm2D, 5: _nn.InstanceNorm3D}[len(input.shape)]
    return cls(input.shape[1], epsilon=epsilon, weight_attr=param_attr, bias_attr=bias_attr)(input)


def data_norm(input, act=None, epsilon=1e-05, param_attr=None, data_layout="NCHW", in_place=False, name=None,
              moving_mean_name=None, moving_variance_name=None, do_model_average_for_mean_and_var=True,
              slot_dim=-1, sync_stats=False, summary_decay_rate=0.9999999, enable_scale_and_shift=False):
    """Reference static/nn/common.py data_norm: normalise by accumulated batch statistics — parameters
    batch_size (init 1e4), batch_sum (0), batch_square_sum (1e4): mean = sum / size,
    scale = sqrt(size / square_sum); y = (x - mean) * scale (optionally * scale_w + bias)."""
    from ..framework.param import create_parameter
    from ..nn import initializer as I

    c = input.shape[-1]
    size = create_parameter([c], "float32", default_initializer=I.Constant(1e4))
    bsum = create_parameter([c], "float32", default_initializer=I.Constant(0.0))
    sq = create_parameter([c], "float32", default_initializer=I.Constant(1e4))
    for t in (size, bsum, sq):
        t.stop_gradient = True
    mean = bsum / size
    scale = (size / sq).sqrt()
    y = (input - mean) * scale
    if enable_scale_and_shift:
        w = create_parameter([c], "float32", default_initializer=I.Constant(1.0))
        b = create_parameter([c], "float32", default_initializer=I.Constant(0.0))
        y = y * w + b
    return _act(y, act)


def prelu(x, mode, param_attr=None, data_format="NCHW", name=None):
    if mode == "all":
        n = 1
    elif mode == "channel":
        n = x.shape[1] if data_format == "NCHW" else x.shape[-1]
    elif mode == "element":
        n = 1
        for d in x.shape[1:]:
            n *= d
    else:
        raise ValueError(f"prelu: unknown mode {mode!r}")
    if mode == "element":
        from ..framework.param import create_parameter
        from ..nn import initializer as I

        alpha = create_parameter(list(x.shape[1:]), "float32", attr=param_attr, default_initializer=I.Constant(0.25))
        return F.relu(x) - alpha * F.relu(-x)
    return _nn.PReLU(n, weight_attr=param_attr, data_format=data_format)(x)


def bilinear_tensor_product(x, y, size, act=None, name=None, param_attr=None, bias_attr=None):
    b = _nn.Bilinear(x.shape[-1], y.shape[-1], size, weight_attr=param_attr, bias_attr=bias_attr)
    return _act(b(x, y), act)


def spectral_norm(weight, dim=0, power_iters=1, eps=1e-12, name=None):
    return _nn.SpectralNorm(list(weight.shape), dim=dim, power_iters=power_iters, eps=eps)(weight)


def deform_conv2d(x, offset, mask, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=1,
                  deformable_groups=1, im2col_step=1, weight_attr=None, bias_attr=None, name=None):
    from ..framework.param import create_parameter
    from ..vision import ops as vops

    ks = [filter_size] * 2 if isinstance(filter_size, int) else list(filter_size)
    w = create_parameter([num_filters, x.shape[1] // groups] + ks, "float32", attr=weight_attr)
    b = None if bias_attr is False else create_parameter([num_filters], "float32", attr=bias_attr, is_bias=True)
    return vops.deform_conv2d(x, offset, w, bias=b, stride=stride, padding=padding, dilation=dilation,
                              deformable_groups=deformable_groups, groups=groups, mask=mask)


def row_conv(input, future_context_size, param_attr=None, act=None):
    """Lookahead (row) convolution over the time axis of [B, T, D] (reference row_conv_op):
    out[t] = sum_{i=0..k} w[i] * x[t + i] (zero past the end), w [k + 1, D]."""
    from ..framework.param import create_parameter

    k = future_context_size
    d = input.shape[-1]
    w = create_parameter([k + 1, d], "float32", attr=param_attr)
    from .. import tensor as _T

    T = input.shape[1]
    xp = _T.concat([input, _T.zeros([input.shape[0], k, d], dtype=input.dtype)], axis=1) if k else input
    out = None
    for i in range(k + 1):
        term = xp[:, i:i + T, :] * w[i]
        out = term if out is None else out + term
    return _act(out, act)


def sparse_embedding(input, size, padding_idx=None, is_test=False, entry=None, table_class="MemorySparseTable",
                     param_attr=None, dtype="float32", slot=None):
    """Reference: the parameter-server sparse table lookup.  Single-node form: an Embedding whose gradient is
    a SelectedRows (only the touched rows are updated)."""
    return _nn.Embedding(size[0], size[1], padding_idx=padding_idx, sparse=True, weight_attr=param_attr)(input)


def nce(input, label, num_total_classes, sample_weight=None, param_attr=None, bias_attr=None, num_neg_samples=None,
        name=None, sampler="uniform", custom_dist=None, seed=0, is_sparse=False):
    """Noise-contrastive estimation loss (reference static/nn/loss.py nce): per row, the true class and
    ``num_neg_samples`` sampled classes are scored with a logistic classifier; with a uniform sampler the
    noise probability of every class is 1/N: loss = -log sigma(s_t - log(k q)) - sum_j log(1 - sigma(s_j - log(k q)))."""
    import math

    import torch

    from ..framework.param import create_parameter
    from ..framework.tensor import Tensor

    k = num_neg_samples or 10
    dim = input.shape[-1]
    w = create_parameter([num_total_classes, dim], "float32", attr=param_attr)
    b = create_parameter([num_total_classes], "float32", attr=bias_attr, is_bias=True)
    gen = torch.Generator().manual_seed(seed)
    n = input.shape[0]
    if sampler == "uniform":
        neg = torch.randint(0, num_total_classes, (n, k), generator=gen)
        logq = torch.full((n, k), math.log(k / num_total_classes))
        logq_t = math.log(k / num_total_classes)
    elif sampler == "custom_dist":
        dist = torch.as_tensor(custom_dist, dtype=torch.float64)
        neg = torch.multinomial(dist, n * k, replacement=True, generator=gen).reshape(n, k)
        logq = torch.log(k * dist[neg]).float()
        logq_t = None
    else:
        raise ValueError(f"nce: unsupported sampler {sampler!r}")
    lab = label.reshape([-1])
    s_t = (input * w[lab]).sum(-1) + b[lab]
    negt = Tensor._wrap(neg.to(input._t.device if hasattr(input, "_t") else "cpu"))
    s_n = (input.unsqueeze(1) * w[negt]).sum(-1) + b[negt]
    if logq_t is None:
        dl = Tensor._wrap(torch.log(k * torch.as_tensor(custom_dist, dtype=torch.float32))).to(s_t.place if hasattr(s_t, "place") else None)
        lq_t = dl[lab]
    else:
        lq_t = logq_t
    lq_n = Tensor._wrap(logq.to(negt._t.device))
    loss = -F.log_sigmoid(s_t - lq_t) - F.log_sigmoid(-(s_n - lq_n)).sum(-1)
    if sample_weight is not None:
        loss = loss * sample_weight.reshape([-1])
    return loss.reshape([-1, 1])


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    """Run a Python function as an op (reference static/nn/common.py py_func): ``func`` maps the input
    tensors to outputs shaped like ``out``; with ``backward_func`` the op is differentiable
    (grads = backward_func(*inputs, *outputs, *output_grads), minus ``skip_vars_in_backward_input``)."""
    from ..autograd import PyLayer

    xs = list(x) if isinstance(x, (list, tuple)) else [x]
    single = not isinstance(out, (list, tuple))

    def _call(*args):
        r = func(*args)
        return r if isinstance(r, (list, tuple)) else (r,)

    if backward_func is None:
        res = _call(*xs)
        return res[0] if single else list(res)
    skip = {id(v) for v in (skip_vars_in_backward_input or [])}

    class _PyFunc(PyLayer):
        @staticmethod
        def forward(ctx, *ins):
            outs = _call(*ins)
            ctx.save_for_backward(*ins, *outs)
            ctx.n_in = len(ins)
            return outs[0] if single else tuple(outs)

        @staticmethod
        def backward(ctx, *grads):
            saved = list(ctx.saved_tensor())
            ins, outs = saved[:ctx.n_in], saved[ctx.n_in:]
            args = [v for v in ins if id(v) not in skip] + [v for v in outs if id(v) not in skip] + list(grads)
            g = backward_func(*args)
            return g if isinstance(g, (list, tuple)) else g

    res = _PyFunc.apply(*xs)
    return res if single else list(res)


def static_pylayer(forward_fn, inputs, backward_fn=None, name=None):
    """Reference static/nn/static_pylayer.py: a forward sub-graph with a user backward sub-graph."""
    if backward_fn is None:
        return forward_fn(*inputs)
    from ..autograd import PyLayer

    class _SPL(PyLayer):
        @staticmethod
        def forward(ctx, *ins):
            return forward_fn(*ins)

        @staticmethod
        def backward(ctx, *grads):
            return backward_fn(*grads)

    return _SPL.apply(*inputs)


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


def case(pred_fn_pairs, default=None, name=None):
    """Reference static/nn/control_flow.py case: the first pair whose predicate holds runs (nested cond)."""
    pairs = list(pred_fn_pairs)
    if not pairs:
        raise ValueError("case: pred_fn_pairs is empty")
    if default is None:
        pairs, (_, default) = pairs[:-1], pairs[-1]
    if not pairs:
        return default()
    (pred, fn), rest = pairs[0], pairs[1:]
    return cond(pred, fn, lambda: case(rest, default) if rest else default())


def switch_case(branch_index, branch_fns, default=None, name=None):
    """Reference static/nn/control_flow.py switch_case: branch_fns is a list of fns or (index, fn) pairs /
    a dict; the branch whose index equals ``branch_index`` runs, else ``default`` (or the last branch)."""
    if isinstance(branch_fns, dict):
        items = sorted(branch_fns.items())
    elif branch_fns and isinstance(branch_fns[0], (list, tuple)):
        items = sorted((int(i), f) for i, f in branch_fns)
    else:
        items = list(enumerate(branch_fns))
    if default is None:
        items, (_, default) = items[:-1], items[-1]
    pairs = [(branch_index == i, f) for i, f in items]
    return case(pairs, default) if pairs else default()


from .sequence import (lod_reset, sequence_conv, sequence_expand, sequence_first_step,  # noqa: E402,F401
                       sequence_last_step, sequence_pool, sequence_softmax)
