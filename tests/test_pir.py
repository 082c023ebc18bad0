"""PIR (paddle2_amd/pir): translation of recorded static programs to SSA, interpretation, passes (DCE, CSE,
constant folding, fused_gemm_epilogue) and primitive decomposition — every rewritten program must compute
what the eager model computes (reference: paddle/pir, fluid/pir/transforms, primitive composite rules)."""
import numpy as np
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd import decomposition, pir
from paddle2_amd.jit import StaticFunction, _spec_tensors
from paddle2_amd.pir import passes
from paddle2_amd.static import InputSpec


def _record(net, shape):
    net.eval()
    spec = [InputSpec(shape, "float32", name="x")]
    sf = StaticFunction(lambda *a: net(*a), spec)
    prog, feeds, outs, _ = sf._record(_spec_tensors(spec))
    feed_vars = [paddle.Tensor._wrap(prog.feeds[n]) for n in feeds]
    return pir.translate_to_pir(prog, feed_vars, outs)


def _mlp():
    paddle.seed(4)
    return paddle.nn.Sequential(paddle.nn.Linear(6, 16), paddle.nn.GELU(), paddle.nn.LayerNorm(16),
                                paddle.nn.Linear(16, 8), paddle.nn.ReLU(), paddle.nn.Linear(8, 4), paddle.nn.Softmax())


def test_translate_print_and_run():
    net = _mlp()
    x = torch.randn(3, 6)
    prog = _record(net, [3, 6])
    text = str(prog)
    assert '"pd_op.matmul"' in text and '"pd_op.layer_norm"' in text and "tensor<3x16xf32>" in text
    assert prog.op_names()[-1] == "pd_op.fetch" and "pd_op.data" in prog.op_names()
    out = pir.run(prog, [x])[0]
    torch.testing.assert_close(out, net(paddle.to_tensor(x))._t, rtol=1e-5, atol=1e-6)


def test_fused_gemm_epilogue_dce_cse_constant_folding():
    net = _mlp()
    x = torch.randn(3, 6)
    ref = net(paddle.to_tensor(x))._t
    prog = _record(net, [3, 6])
    stats = passes.apply(prog, ["fused_gemm_epilogue_pass", "common_subexpression_elimination_pass",
                                "dead_code_elimination_pass", "constant_folding_pass"])
    names = prog.op_names()
    assert stats["fused_gemm_epilogue_pass"] == 3 and names.count("pd_op.fused_gemm_epilogue") == 3
    assert "pd_op.matmul" not in names and "pd_op.relu" not in names
    fused = [o for o in prog.global_block().ops if o.name() == "pd_op.fused_gemm_epilogue"]
    assert {o.attrs()["activation"] for o in fused} == {"gelu", "identity", "relu"}
    torch.testing.assert_close(pir.run(prog, [x])[0], ref, rtol=1e-5, atol=1e-6)


def test_cse_and_dce_on_duplicates():
    class Dup(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.fc = paddle.nn.Linear(4, 4)

        def forward(self, x):
            a = paddle.exp(x)
            b = paddle.exp(x)          # same op, same operand -> CSE
            _unused = paddle.tanh(x)   # dead -> DCE (pruned already by the fetch-driven lowering)
            return self.fc(a + b)

    prog = _record(Dup(), [2, 4])
    x = torch.randn(2, 4)
    before = pir.run(prog, [x])[0]
    n = passes.common_subexpression_elimination_pass(prog)
    assert n == 1 and prog.op_names().count("pd_op.exp") == 1
    torch.testing.assert_close(pir.run(prog, [x])[0], before)


def test_decomposition_to_primitives():
    net = _mlp()
    x = torch.randn(3, 6)
    ref = net(paddle.to_tensor(x))._t
    prog = _record(net, [3, 6])
    n = decomposition.decompose(prog)
    names = set(prog.op_names())
    assert n == 4 and not names & {"pd_op.softmax", "pd_op.gelu", "pd_op.layer_norm", "pd_op.relu"}
    assert {"pd_op.erf", "pd_op.rsqrt", "pd_op.exp"} <= names
    torch.testing.assert_close(pir.run(prog, [x])[0], ref, rtol=1e-5, atol=1e-5)
    # whitelist restricts the rules applied
    prog2 = _record(net, [3, 6])
    assert decomposition.decompose(prog2, whitelist={"pd_op.softmax"}) == 1
    assert "pd_op.gelu" in prog2.op_names()
    np.testing.assert_allclose(pir.run(prog2, [x])[0].detach().numpy(), ref.detach().numpy(), rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------ dialect registry / verifier, DRR, serialization
def test_verify_registered_program_and_catches_breakage():
    prog = _record(_mlp(), [3, 6])
    assert pir.verify(prog) == prog.num_ops()
    info = pir.IrContext.instance().op_info("pd_op.matmul")
    assert info.has_trait("Pure") and pir.dialect.has_trait(prog.global_block().ops[-1], "SideEffect")
    # an operand used before its definition
    ops = prog.global_block().ops
    i = next(k for k, o in enumerate(ops) if o.name() == "pd_op.matmul")
    ops.insert(0, ops.pop(i))
    try:
        pir.verify(prog)
        raise AssertionError("verify accepted a use before definition")
    except pir.VerifyError as e:
        assert "before its definition" in str(e)


def test_verify_rejects_bad_arity_attrs_and_unknown_dialect():
    p = pir.Program()
    d = p.global_block().append(pir.Operation("pd_op.data", [], [([4, 4], torch.float32)], {"name": "x", "col": 0}))
    x = d.result(0)
    p.global_block().append(pir.Operation("pd_op.matmul", [x], [([4, 4], torch.float32)]))
    with pytest.raises(pir.VerifyError, match="operands"):
        pir.verify(p)
    p2 = pir.Program()
    d2 = p2.global_block().append(pir.Operation("pd_op.data", [], [([4, 4], torch.float32)], {"name": "x", "col": 0}))
    p2.global_block().append(pir.Operation("pd_op.softmax", [d2.result(0)], [([4, 4], torch.float32)], {"axis": "1"}))
    with pytest.raises(pir.VerifyError, match="attribute 'axis'"):
        pir.verify(p2)
    p3 = pir.Program()
    p3.global_block().append(pir.Operation("mydialect.op", [], [([1], torch.float32)]))
    with pytest.raises(pir.VerifyError, match="dialect"):
        pir.verify(p3)


def test_drr_rewrites_match_the_handwritten_fusion_pass():
    net = _mlp()
    x = torch.randn(3, 6)
    ref = net(paddle.to_tensor(x))._t
    a, b = _record(net, [3, 6]), _record(net, [3, 6])
    passes.apply(a, ["fused_gemm_epilogue_pass"])
    stats = passes.apply(b, ["drr_rewrite_pass"])
    assert stats["drr_rewrite_pass"] == 3
    assert sorted(a.op_names()) == sorted(b.op_names())
    acts = sorted(o.attrs()["activation"] for o in b.global_block().ops if o.name() == "pd_op.fused_gemm_epilogue")
    assert acts == ["gelu", "identity", "relu"]
    pir.verify(b)
    torch.testing.assert_close(pir.run(b, [x])[0], ref, rtol=1e-5, atol=1e-6)


def _chain_program():
    from paddle2_amd.pir import drr  # noqa: F401

    p = pir.Program()
    blk = p.global_block()
    x = blk.append(pir.Operation("pd_op.data", [], [([2, 3, 4], torch.float32)], {"name": "x", "col": 0})).result(0)
    s1 = blk.append(pir.Operation("pd_op.scale", [x], [([2, 3, 4], torch.float32)],
                                  {"scale": 2.0, "bias": 1.0, "bias_after_scale": True})).result(0)
    s2 = blk.append(pir.Operation("pd_op.scale", [s1], [([2, 3, 4], torch.float32)],
                                  {"scale": 3.0, "bias": -0.5, "bias_after_scale": True})).result(0)
    t1 = blk.append(pir.Operation("pd_op.transpose", [s2], [([3, 4, 2], torch.float32)], {"axis": [1, 2, 0]})).result(0)
    t2 = blk.append(pir.Operation("pd_op.transpose", [t1], [([2, 3, 4], torch.float32)], {"axis": [2, 0, 1]})).result(0)
    blk.append(pir.Operation("pd_op.fetch", [t2], [([2, 3, 4], torch.float32)], {"name": "y", "col": 0}))
    return p


def test_drr_cancels_inverse_transposes_and_folds_scales():
    from paddle2_amd.pir import drr

    x = torch.randn(2, 3, 4)
    p = _chain_program()
    stats = drr.apply_patterns_greedily(p, drr.default_patterns())
    assert stats["cancel_transpose_pair"] == 1 and stats["fold_scale_pair"] == 1
    assert p.op_names() == ["pd_op.data", "pd_op.scale", "pd_op.fetch"]
    sc = p.global_block().ops[1].attrs()
    assert sc["scale"] == 6.0 and sc["bias"] == 2.5
    pir.verify(p)
    torch.testing.assert_close(pir.run(p, [x])[0], (x * 2 + 1) * 3 - 0.5)


def test_serialize_round_trip(tmp_path):
    net = _mlp()
    x = torch.randn(3, 6)
    prog = _record(net, [3, 6])
    passes.apply(prog, ["drr_rewrite_pass"])
    path = str(tmp_path / "m.pir.json")
    pir.save(prog, path)
    back = pir.load(path)
    assert back.op_names() == prog.op_names()
    for a, b in zip(prog.global_block().ops, back.global_block().ops):
        assert a.attrs() == b.attrs() and [r.shape for r in a.results()] == [r.shape for r in b.results()]
    pir.verify(back)
    torch.testing.assert_close(pir.run(back, [x])[0], pir.run(prog, [x])[0])


def _unary_program(name, shape, attrs=None, extra=None):
    p = pir.Program()
    blk = p.global_block()
    x = blk.append(pir.Operation("pd_op.data", [], [(shape, torch.float32)], {"name": "x", "col": 0})).result(0)
    operands = [x]
    if extra is not None:
        operands.append(blk.append(pir.Operation("pd_op.data", [], [(extra, torch.float32)],
                                                 {"name": "y", "col": 1})).result(0))
    y = blk.append(pir.Operation(name, operands, [(shape, torch.float32)], attrs or {})).result(0)
    blk.append(pir.Operation("pd_op.fetch", [y], [(shape, torch.float32)], {"name": "out", "col": 0}))
    return p


@pytest.mark.parametrize("name,attrs,ref", [
    ("pd_op.relu", {}, torch.relu),
    ("pd_op.relu6", {"threshold": 6.0}, lambda x: torch.clamp(x, 0, 6)),
    ("pd_op.leaky_relu", {"alpha": 0.1}, lambda x: torch.nn.functional.leaky_relu(x, 0.1)),
    ("pd_op.elu", {"alpha": 0.7}, lambda x: torch.nn.functional.elu(x, 0.7)),
    ("pd_op.softplus", {"beta": 1.0}, torch.nn.functional.softplus),
    ("pd_op.mish", {}, torch.nn.functional.mish),
    ("pd_op.hardswish", {}, torch.nn.functional.hardswish),
    ("pd_op.hardsigmoid", {"slope": 1.0 / 6, "offset": 0.5}, torch.nn.functional.hardsigmoid),
    ("pd_op.square", {}, torch.square),
    ("pd_op.reciprocal", {}, torch.reciprocal),
    ("pd_op.log_softmax", {"axis": -1}, lambda x: torch.log_softmax(x, -1)),
    ("pd_op.swish", {}, torch.nn.functional.silu),
    ("pd_op.mean", {"dim": [1], "keep_dim": True}, lambda x: x.mean(1, keepdim=True)),
    ("pd_op.logsumexp", {"axis": [1], "keepdim": True}, lambda x: torch.logsumexp(x, 1, keepdim=True)),
])
def test_decomposition_rules_match_reference(name, attrs, ref):
    x = torch.randn(5, 7) * 4
    p = _unary_program(name, [5, 7], attrs)
    assert decomposition.decompose(p) == 1
    names = set(p.op_names()) - {"pd_op.data", "pd_op.fetch"}
    assert names <= decomposition.PRIMITIVES, names - decomposition.PRIMITIVES
    torch.testing.assert_close(pir.run(p, [x])[0], ref(x), rtol=1e-5, atol=1e-5)


def test_decomposition_swiglu_and_rms_norm():
    x, y = torch.randn(4, 8), torch.randn(4, 8)
    p = _unary_program("pd_op.swiglu", [4, 8], {}, extra=[4, 8])
    assert decomposition.decompose(p) == 1
    torch.testing.assert_close(pir.run(p, [x, y])[0], torch.nn.functional.silu(x) * y)
    p2 = _unary_program("pd_op.rms_norm", [4, 8], {"epsilon": 1e-6})
    assert decomposition.decompose(p2) == 1
    torch.testing.assert_close(pir.run(p2, [x])[0], x * torch.rsqrt((x * x).mean(-1, keepdim=True) + 1e-6))
