"""PIR (paddle2_amd/pir): translation of recorded static programs to SSA, interpretation, passes (DCE, CSE,
constant folding, fused_gemm_epilogue) and primitive decomposition — every rewritten program must compute
what the eager model computes (reference: paddle/pir, fluid/pir/transforms, primitive composite rules)."""
import numpy as np
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
    assert n == 3 and not names & {"pd_op.softmax", "pd_op.gelu", "pd_op.layer_norm"}
    assert {"pd_op.erf", "pd_op.rsqrt", "pd_op.exp"} <= names
    torch.testing.assert_close(pir.run(prog, [x])[0], ref, rtol=1e-5, atol=1e-5)
    # whitelist restricts the rules applied
    prog2 = _record(net, [3, 6])
    assert decomposition.decompose(prog2, whitelist={"pd_op.softmax"}) == 1
    assert "pd_op.gelu" in prog2.op_names()
    np.testing.assert_allclose(pir.run(prog2, [x])[0].detach().numpy(), ref.detach().numpy(), rtol=1e-5, atol=1e-5)
