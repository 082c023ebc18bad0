"""Primitive decomposition breadth (decomposition/rules.py) and reverse mode over primitives (decomposition/vjp.py).

Each composite op is put into a one-op PIR program, decomposed, run by the PIR interpreter and compared with a
torch reference of the same op (reference: paddle/fluid/primitive/composite/composite.h rules,
test/prim/pir_prim/ checks decomposed vs original numerics).  The VJP tests differentiate decomposed programs with
``append_backward`` and compare every gradient with torch autograd.
"""
import math

import pytest
import torch
import torch.nn.functional as F

import paddle2_amd as paddle
from paddle2_amd import decomposition, pir
from paddle2_amd.decomposition import vjp


def _program(name, inputs, attrs=None, out_shape=None, out_dtype=torch.float32, n_results=1):
    p = pir.Program()
    vals = []
    for i, t in enumerate(inputs):
        d = p.block.append(pir.Operation("pd_op.data", [], [(list(t.shape), t.dtype)], {"name": f"x{i}", "col": i}))
        vals.append(d.result(0))
    rt = [(out_shape, out_dtype)] + [(None, torch.float32)] * (n_results - 1)
    op = p.block.append(pir.Operation(name, vals, rt, attrs or {}))
    p.block.append(pir.Operation("pd_op.fetch", [op.result(0)], [(out_shape, out_dtype)], {"name": "out", "col": 0}))
    return p


def _check(name, inputs, ref, attrs=None, out_shape=None, out_dtype=torch.float32, atol=1e-5, n_results=1):
    p = _program(name, inputs, attrs, out_shape, out_dtype, n_results)
    assert decomposition.decompose(p) == 1, f"{name} was not decomposed"
    left = {o.name() for o in p.block.ops} - {"pd_op.data", "pd_op.fetch"}
    assert left <= decomposition.PRIMITIVES, left - decomposition.PRIMITIVES
    got = pir.run(p, inputs)[0]
    exp = ref(*inputs)
    assert tuple(got.shape) == tuple(exp.shape), (name, got.shape, exp.shape)
    if exp.dtype == torch.bool or not exp.is_floating_point():
        assert torch.equal(got.to(exp.dtype), exp)
    else:
        torch.testing.assert_close(got.to(exp.dtype), exp, atol=atol, rtol=1e-5)


g = torch.Generator().manual_seed(0)


def _r(*shape, lo=-2.0, hi=2.0):
    return torch.rand(*shape, generator=g) * (hi - lo) + lo


X = _r(3, 5)
POS = _r(3, 5, lo=0.05, hi=2.0)
PROB = _r(3, 5, lo=0.02, hi=0.98)
LAB = _r(3, 5, lo=0.0, hi=1.0)

ACTIVATIONS = [
    ("pd_op.tanh_shrink", {}, lambda x: x - torch.tanh(x)),
    ("pd_op.hardtanh", {"t_min": -0.5, "t_max": 1.2}, lambda x: F.hardtanh(x, -0.5, 1.2)),
    ("pd_op.selu", {}, F.selu),
    ("pd_op.celu", {"alpha": 1.5}, lambda x: F.celu(x, 1.5)),
    ("pd_op.thresholded_relu", {"threshold": 0.3}, lambda x: F.threshold(x, 0.3, 0.0)),
    ("pd_op.logsigmoid", {}, F.logsigmoid),
    ("pd_op.softshrink", {"threshold": 0.4}, lambda x: F.softshrink(x, 0.4)),
    ("pd_op.hardshrink", {"threshold": 0.4}, lambda x: F.hardshrink(x, 0.4)),
    ("pd_op.softsign", {}, F.softsign),
    ("pd_op.expm1", {}, torch.expm1),
    ("pd_op.stanh", {"scale_a": 0.67, "scale_b": 1.7159}, lambda x: 1.7159 * torch.tanh(0.67 * x)),
    ("pd_op.clip", {"min": -0.5, "max": 0.7}, lambda x: x.clamp(-0.5, 0.7)),
]


@pytest.mark.parametrize("name,attrs,ref", ACTIVATIONS, ids=[a[0] for a in ACTIVATIONS])
def test_activation_rules(name, attrs, ref):
    _check(name, [X], ref, attrs, [3, 5])


@pytest.mark.parametrize("name,ref", [("pd_op.log2", torch.log2), ("pd_op.log10", torch.log10),
                                      ("pd_op.log1p", torch.log1p)])
def test_log_rules(name, ref):
    _check(name, [POS], ref, {}, [3, 5])


@pytest.mark.parametrize("p", [0.0, 1.0, 2.0, 3.0, math.inf, -math.inf])
@pytest.mark.parametrize("keep", [False, True])
def test_p_norm(p, keep):
    shape = [3, 1] if keep else [3]
    _check("pd_op.p_norm", [X], lambda x: torch.linalg.vector_norm(x, p, dim=1, keepdim=keep),
           {"porder": p, "axis": 1, "keepdim": keep}, shape, atol=1e-4)


@pytest.mark.parametrize("y,ref", [(2.0, lambda x: x * x), (3.0, lambda x: x ** 3), (0.5, torch.sqrt),
                                   (-1.0, torch.reciprocal)])
def test_pow(y, ref):
    _check("pd_op.pow", [POS], ref, {"y": y}, [3, 5])


def test_reductions_and_norms():
    b = torch.rand(3, 5, generator=g) > 0.5
    _check("pd_op.any", [b], lambda x: torch.any(x, dim=1), {"axis": [1], "keepdim": False}, [3], torch.bool)
    _check("pd_op.mean_all", [X], lambda x: x.mean(), {}, [])
    _check("pd_op.squared_l2_norm", [X], lambda x: (x * x).sum().reshape(1), {}, [1])
    _check("pd_op.numel", [X], lambda x: torch.tensor(15), {}, [], torch.int64)


def test_losses():
    _check("pd_op.huber_loss", [X, LAB], lambda x, l: F.huber_loss(x, l, reduction="none", delta=0.6),
           {"delta": 0.6}, [3, 5], n_results=2)
    _check("pd_op.bce_loss", [PROB, LAB], lambda x, l: F.binary_cross_entropy(x, l, reduction="none"), {}, [3, 5])
    _check("pd_op.sigmoid_cross_entropy_with_logits", [X, LAB],
           lambda x, l: F.binary_cross_entropy_with_logits(x, l, reduction="none"), {}, [3, 5])
    _check("pd_op.log_loss", [PROB, LAB],
           lambda x, l: -l * torch.log(x + 1e-4) - (1 - l) * torch.log(1 - x + 1e-4), {"epsilon": 1e-4}, [3, 5])
    logp = torch.log_softmax(X, -1)
    for red, shape in (("none", [3, 5]), ("sum", []), ("mean", []), ("batchmean", [])):
        _check("pd_op.kldiv_loss", [logp, LAB], lambda x, l: F.kl_div(x, l, reduction=red), {"reduction": red}, shape)


def test_shape_ops():
    a, b2, c = _r(2, 3), _r(2, 3), _r(2, 3)
    _check("pd_op.stack", [a, b2, c], lambda *t: torch.stack(t, 1), {"axis": 1}, [2, 3, 3])
    _check("pd_op.add_n", [a, b2, c], lambda *t: t[0] + t[1] + t[2], {}, [2, 3])
    _check("pd_op.squeeze", [_r(2, 1, 3)], lambda x: x.squeeze(1), {"axis": [1]}, [2, 3])
    _check("pd_op.unsqueeze", [a], lambda x: x.unsqueeze(0), {"axis": [0]}, [1, 2, 3])
    _check("pd_op.flatten", [_r(2, 3, 4)], lambda x: x.flatten(1), {"start_axis": 1, "stop_axis": 2}, [2, 12])
    _check("pd_op.full_like", [a], lambda x: torch.full_like(x, 3.5), {"value": 3.5}, [2, 3])
    _check("pd_op.bmm", [_r(2, 3, 4), _r(2, 4, 5)], torch.bmm, {}, [2, 3, 5])


def _check_multi(name, inputs, attrs, out_shapes, refs):
    """Multi-output composite (unbind / unstack / meshgrid): every result fetched and compared."""
    p = pir.Program()
    vals = [p.block.append(pir.Operation("pd_op.data", [], [(list(t.shape), t.dtype)],
                                         {"name": f"x{i}", "col": i})).result(0) for i, t in enumerate(inputs)]
    op = p.block.append(pir.Operation(name, vals, [(s, torch.float32) for s in out_shapes], attrs))
    for i, s in enumerate(out_shapes):
        p.block.append(pir.Operation("pd_op.fetch", [op.result(i)], [(s, torch.float32)], {"name": f"o{i}", "col": i}))
    assert decomposition.decompose(p) == 1, f"{name} was not decomposed"
    left = {o.name() for o in p.block.ops} - {"pd_op.data", "pd_op.fetch"}
    assert left <= decomposition.PRIMITIVES, left - decomposition.PRIMITIVES
    got = pir.run(p, inputs)
    assert len(got) == len(refs)
    for a, b in zip(got, refs):
        torch.testing.assert_close(a, b)


def test_multi_output_ops():
    x = _r(2, 3, 4)
    _check_multi("pd_op.unbind", [x], {"axis": 1}, [[2, 4]] * 3, list(torch.unbind(x, 1)))
    _check_multi("pd_op.unstack", [x], {"axis": -1}, [[2, 3]] * 4, list(torch.unbind(x, -1)))
    u, v = _r(3), _r(5)
    _check_multi("pd_op.meshgrid", [u, v], {}, [[3, 5], [3, 5]], list(torch.meshgrid(u, v, indexing="ij")))


def test_indexing_ops():
    x = _r(4, 6)
    idx = torch.tensor([3, 0, 3, 1])
    _check("pd_op.index_select", [x, idx], lambda t, i: torch.index_select(t, 1, i), {"axis": 1}, [4, 4])
    si = torch.randint(0, 6, (4, 2), generator=g)
    _check("pd_op.index_sample", [x, si], lambda t, i: torch.gather(t, 1, i), {}, [4, 2])
    ids = torch.tensor([[1, 0, 3], [2, 2, 0]])
    w = _r(5, 4)

    def emb(i, t):
        out = F.embedding(i, t)
        return torch.where((i == 0).unsqueeze(-1), torch.zeros_like(out), out)

    _check("pd_op.embedding", [ids, w], emb, {"padding_idx": 0}, [2, 3, 4])
    oh = torch.tensor([0, 4, 2, 2, 6])
    _check("pd_op.one_hot", [oh], lambda t: F.one_hot(t, 7).float(), {"num_classes": 7}, [5, 7])


def test_elementwise_ternary():
    x, y, w = _r(3, 5), _r(3, 5), _r(3, 5, lo=0.0, hi=1.0)
    _check("pd_op.lerp", [x, y, w], torch.lerp, {}, [3, 5])
    xz = x.clone()
    xz[0, :2] = 0.0
    _check("pd_op.heaviside", [xz, y], torch.heaviside, {}, [3, 5])


def test_norm_layers():
    x = _r(2, 4, 3, 3)
    m, v = _r(4), _r(4, lo=0.5, hi=2.0)
    s, b = _r(4), _r(4)
    _check("pd_op.batch_norm", [x, m, v, s, b], lambda x_, m_, v_, s_, b_: F.batch_norm(x_, m_, v_, s_, b_, False,
                                                                                         eps=1e-5),
           {"is_test": True, "epsilon": 1e-5, "data_format": "NCHW"}, [2, 4, 3, 3], atol=1e-4, n_results=6)
    _check("pd_op.batch_norm", [x, m, v, s, b], lambda x_, m_, v_, s_, b_: F.batch_norm(x_, None, None, s_, b_, True,
                                                                                         eps=1e-5),
           {"is_test": False, "epsilon": 1e-5, "data_format": "NCHW"}, [2, 4, 3, 3], atol=1e-4, n_results=6)
    _check("pd_op.instance_norm", [x, s, b], lambda x_, s_, b_: F.instance_norm(x_, weight=s_, bias=b_, eps=1e-5),
           {"epsilon": 1e-5}, [2, 4, 3, 3], atol=1e-4, n_results=3)
    _check("pd_op.group_norm", [x, s, b], lambda x_, s_, b_: F.group_norm(x_, 2, s_, b_, eps=1e-5),
           {"epsilon": 1e-5, "groups": 2, "data_format": "NCHW"}, [2, 4, 3, 3], atol=1e-4, n_results=3)


def test_dropout():
    x = _r(64, 64, lo=0.5, hi=1.5)
    _check("pd_op.dropout", [x], lambda t: t, {"p": 0.3, "is_test": True, "mode": "upscale_in_train"}, [64, 64],
           n_results=2)
    _check("pd_op.dropout", [x], lambda t: t * 0.7, {"p": 0.3, "is_test": True, "mode": "downgrade_in_infer"},
           [64, 64], n_results=2)
    p = _program("pd_op.dropout", [x], {"p": 0.3, "is_test": False, "mode": "upscale_in_train", "seed": 7},
                 [64, 64], n_results=2)
    assert decomposition.decompose(p) == 1
    y = pir.run(p, [x])[0]
    kept = y != 0
    assert 0.6 < float(kept.float().mean()) < 0.8
    torch.testing.assert_close(y[kept], x[kept] / 0.7)


def test_side_output_in_use_is_left_alone():
    x = _r(2, 4, 3, 3)
    p = _program("pd_op.instance_norm", [x, _r(4), _r(4)], {"epsilon": 1e-5}, [2, 4, 3, 3], n_results=3)
    op = next(o for o in p.block.ops if o.name() == "pd_op.instance_norm")
    p.block.append(pir.Operation("pd_op.fetch", [op.result(1)], [(None, torch.float32)], {"name": "m", "col": 1}))
    assert decomposition.decompose(p) == 0


def test_rule_count_covers_reference_composites():
    ref = ["any", "mean", "p_norm", "pow", "huber_loss", "one_hot", "squared_l2_norm", "reciprocal", "bce_loss", "bmm",
           "batch_norm", "softmax", "log_softmax", "stack", "silu", "swiglu", "relu", "relu6", "squeeze", "unsqueeze",
           "add_n", "layer_norm", "full_like", "dropout", "gelu", "hardsigmoid", "hardswish", "heaviside",
           "leaky_relu", "instance_norm", "flatten", "clip", "index_select", "group_norm", "square",
           "sigmoid_cross_entropy_with_logits", "mean_all", "embedding", "index_sample", "elu", "lerp", "log_loss",
           "kldiv_loss", "softsign", "numel", "swish"]
    missing = [n for n in ref if not decomposition.has_rule("pd_op." + n)]
    assert not missing, missing


# ------------------------------------------------------------------------------------------------- reverse mode
def _grad_check(build, inputs, torch_fn, atol=1e-4):
    """build(b, vals) -> out Value over data values; compares append_backward grads with torch autograd."""
    p = pir.Program()
    vals = []
    for i, t in enumerate(inputs):
        d = p.block.append(pir.Operation("pd_op.data", [], [(list(t.shape), t.dtype)], {"name": f"x{i}", "col": i}))
        vals.append(d.result(0))
    b = vjp._B(p, None)
    out = build(b, vals)
    p.block.append(pir.Operation("pd_op.fetch", [out], [(out.shape, out.dtype)], {"name": "out", "col": 0}))
    gw = torch.randn(*out.shape, generator=g)
    gop = pir.Operation("pd_op.data", [], [(list(gw.shape), gw.dtype)], {"name": "gout", "col": len(inputs)})
    p.block.insert_before(p.block.ops[0], gop)
    gv = gop.result(0)
    grads = vjp.append_backward(p, out, vals, out_grad=gv)
    vjp.add_fetch(p, [gr for gr in grads if gr is not None])
    res = pir.run(p, list(inputs) + [gw])
    ts = [t.clone().requires_grad_(t.is_floating_point()) for t in inputs]
    y = torch_fn(*ts)
    torch.testing.assert_close(res[0], y.detach(), atol=atol, rtol=1e-4)
    y.backward(gw)
    k = 1
    for t, gr in zip(ts, grads):
        if gr is None:
            continue
        torch.testing.assert_close(res[k], t.grad, atol=atol, rtol=1e-4)
        k += 1


def test_vjp_elementwise_and_reductions():
    from paddle2_amd.decomposition import rules as R

    def build(b, v):
        x, y = v
        z = R.div(b, R.mul(b, R.un(b, "pd_op.tanh", x), R.un(b, "pd_op.exp", y)), R.sc(b, R.un(b, "pd_op.abs", y), 1, 1))
        z = R.sub(b, z, b.reduce("pd_op.max", z, [1]))
        z = R.add(b, z, R.un(b, "pd_op.sqrt", R.sc(b, R.mul(b, x, x), 1.0, 1.0)))
        z = b.op("pd_op.maximum", [z, R.sc(b, y, 0.5)], z)
        return b.reduce("pd_op.sum", R.mul(b, z, R.un(b, "pd_op.sigmoid", x)), [0])

    def ref(x, y):
        z = torch.tanh(x) * torch.exp(y) / (y.abs() + 1)
        z = z - z.amax(1, keepdim=True)
        z = z + torch.sqrt(x * x + 1)
        z = torch.maximum(z, 0.5 * y)
        return (z * torch.sigmoid(x)).sum(0, keepdim=True)

    _grad_check(build, [_r(4, 6), _r(4, 6)], ref)


@pytest.mark.parametrize("tx,ty", [(False, False), (True, False), (False, True), (True, True)])
def test_vjp_matmul_broadcast_bias(tx, ty):
    from paddle2_amd.decomposition import rules as R

    x = _r(5, 3) if tx else _r(3, 5)
    w = _r(4, 5) if ty else _r(5, 4)
    bias = _r(4)

    def build(b, v):
        m = b.op2("pd_op.matmul", [v[0], v[1]], [3, 4], torch.float32, transpose_x=tx, transpose_y=ty)
        return R.add(b, m, v[2])

    def ref(x_, w_, b_):
        return (x_.t() if tx else x_) @ (w_.t() if ty else w_) + b_

    _grad_check(build, [x, w, bias], ref)


def test_vjp_shape_and_index_ops():
    from paddle2_amd.decomposition import rules as R

    idx = torch.tensor([2, 0, 2])

    def build(b, v):
        x, y, i = v
        c = b.op2("pd_op.concat", [x, y], [3, 7], torch.float32, axis=1)
        s = b.op2("pd_op.slice", [c], [3, 4], torch.float32, axis=1, start=2, end=6)
        gth = b.op2("pd_op.gather", [s, i], [3, 4], torch.float32, axis=0)
        t = b.op2("pd_op.transpose", [gth], [4, 3], torch.float32, perm=[1, 0])
        r = R.reshape(b, t, [2, 6])
        return b.op("pd_op.pow", [R.sc(b, r, 1.0, 3.0)], r, y=1.5)

    def ref(x, y, i):
        c = torch.cat([x, y], 1)[:, 2:6]
        return (torch.index_select(c, 0, i).t().reshape(2, 6) + 3.0) ** 1.5

    _grad_check(build, [_r(3, 3), _r(3, 4), idx], ref)


def test_vjp_through_decomposed_mlp():
    """Record an MLP, translate to PIR, decompose its composites, append the backward of sum(out), and compare
    every parameter and input gradient with torch autograd on the eager net."""
    from paddle2_amd.jit import StaticFunction, _spec_tensors
    from paddle2_amd.static import InputSpec

    paddle.seed(3)
    net = paddle.nn.Sequential(paddle.nn.Linear(6, 16), paddle.nn.GELU(), paddle.nn.LayerNorm(16),
                               paddle.nn.Linear(16, 8), paddle.nn.Silu(), paddle.nn.Linear(8, 4), paddle.nn.Softmax())
    net.eval()
    spec = [InputSpec([3, 6], "float32", name="x")]
    sf = StaticFunction(lambda *a: net(*a), spec)
    prog, feeds, outs, _ = sf._record(_spec_tensors(spec))
    pp = pir.translate_to_pir(prog, [paddle.Tensor._wrap(prog.feeds[n]) for n in feeds], outs)
    decomposition.decompose(pp)
    out = next(o for o in pp.block.ops if o.name() == "pd_op.fetch").operand_source(0)
    params = [o.result(0) for o in pp.block.ops if o.name() == "builtin.parameter"]
    data = [o.result(0) for o in pp.block.ops if o.name() == "pd_op.data"]
    grads = vjp.append_backward(pp, out, params + data)
    assert all(gr is not None for gr in grads)
    vjp.add_fetch(pp, grads)
    x = torch.randn(3, 6, generator=g)
    res = pir.run(pp, [x])
    # eager reference
    xt = paddle.to_tensor(x, stop_gradient=False)
    for prm in net.parameters():
        prm.clear_gradient() if prm.grad is not None else None
    y = net(xt)
    y.sum().backward()
    torch.testing.assert_close(res[0], y._t.detach(), atol=1e-5, rtol=1e-5)
    eager = {prm.name: prm.grad._t for prm in net.parameters()}
    for v, gres in zip(params, res[1:1 + len(params)]):
        name = v.get_defining_op().attrs()["parameter_name"]
        torch.testing.assert_close(gres, eager[name], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(res[-1], xt.grad._t, atol=1e-4, rtol=1e-4)
