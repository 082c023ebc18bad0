"""Op table over the reference op inventory: coverage, schema records, InferMeta on meta tensors, alias
semantics, reference-signature optimizer ops vs the optimizer classes, fake-quant ops (reference tests:
test/legacy_test/test_sgd_op.py, test_momentum_op.py, test_adam_op.py, test_adagrad_op.py, test_rmsprop_op.py,
test_adamax_op.py, test_lamb_op.py, test_adadelta_op.py, test_fake_quantize_op.py)."""
import numpy as np
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.ops import op_schema as S
from paddle2_amd.ops import registry as R


def test_reference_inventory_coverage():
    cov = S.coverage()
    assert cov["reference_ops"] >= 560
    assert cov["implemented"] / cov["reference_ops"] >= 0.8, cov["missing"]
    names = R.list_ops()
    for core in ("matmul", "softmax", "layer_norm", "rms_norm", "flash_attn", "adamw_", "c_allreduce_sum",
                 "bilinear_interp", "yolo_box", "roi_align", "fused_rotary_position_embedding", "swiglu"):
        assert core in names


def test_schema_records_and_kernel_info():
    sch = S.op_schema("bilinear_interp")
    assert sch["op"] == "bilinear_interp" and any(a["name"] == "size" for a in sch["args"])
    info = R.kernel_info("rms_norm")
    assert info["native_kernel"] == "norm_fwd"
    assert R.kernel_info("fused_moe")["native_kernel"] == "gemm_grouped"
    for name in R.list_ops()[:400:7]:
        rec = S.op_schema(name)
        assert rec["op"] == name and isinstance(rec["args"], list)


@pytest.mark.parametrize("name,args,kw", [
    ("matmul", ([3, 4], [4, 5]), {}),
    ("add", ([2, 3], [1, 3]), {}),
    ("softmax", ([2, 7],), {"axis": -1}),
    ("transpose", ([2, 3, 4],), {"perm": [2, 0, 1]}),
    ("sum", ([2, 3, 4],), {"axis": 1}),
    ("layer_norm", ([4, 8], None, None), {"epsilon": 1e-5, "begin_norm_axis": 1}),
])
def test_infer_meta_matches_execution(name, args, kw):
    xs = [paddle.ones(s) if s is not None else None for s in args]
    meta = S.infer_meta(name, *xs, **kw)
    real = R.select(name).fn(*xs, **kw)
    if isinstance(real, tuple):   # multi-output ops: one MetaTensor per output
        assert [m.shape for m in meta] == [list(r.shape) for r in real]
        return
    assert meta.shape == list(real.shape) and meta.dtype == real._t.dtype


def test_aliases_match_public_api():
    x = paddle.to_tensor(np.random.RandomState(0).randn(1, 2, 4, 5).astype("float32"))
    a = paddle._C_ops.bilinear_interp(x, size=[8, 10])
    b = paddle.nn.functional.interpolate(x, size=[8, 10], mode="bilinear")
    np.testing.assert_allclose(a.numpy(), b.numpy())
    np.testing.assert_allclose(paddle._C_ops.reverse(x, [3]).numpy(), x.numpy()[..., ::-1])
    np.testing.assert_allclose(paddle._C_ops.p_norm(x).numpy(), np.linalg.norm(x.numpy().ravel()), rtol=1e-5)
    out = paddle._C_ops.pool2d(x, [2, 2], [2, 2], 0, pooling_type="avg")
    np.testing.assert_allclose(out.numpy(), paddle.nn.functional.avg_pool2d(x, 2, 2).numpy())
    np.testing.assert_allclose(paddle._C_ops.squared_l2_norm(x).numpy(), [(x.numpy() ** 2).sum()], rtol=1e-5)
    ra = paddle._C_ops.reduce_as(paddle.ones([2, 3, 4]), paddle.ones([3, 1]))
    assert list(ra.shape) == [3, 1] and float(ra.numpy()[0, 0]) == 8.0


def _setup(shape=(6,), seed=0):
    rs = np.random.RandomState(seed)
    return rs.randn(*shape).astype("float32"), rs.randn(*shape).astype("float32")


def _class_step(cls, p0, g, **kw):
    lin = paddle.create_parameter(list(p0.shape), "float32")
    lin._t.data.copy_(torch.tensor(p0))
    opt = cls(parameters=[lin], **kw)
    lin._t.grad = torch.tensor(g)
    opt.step()
    return lin.numpy()


def test_optimizer_ops_match_optimizer_classes():
    p0, g = _setup()
    lr = paddle.to_tensor([0.1])
    # sgd
    p = paddle.to_tensor(p0.copy())
    paddle._C_ops.sgd_(p, lr, paddle.to_tensor(g))
    np.testing.assert_allclose(p.numpy(), _class_step(paddle.optimizer.SGD, p0, g, learning_rate=0.1), rtol=1e-6)
    # momentum (one step)
    p, v = paddle.to_tensor(p0.copy()), paddle.zeros([6])
    paddle._C_ops.momentum_(p, paddle.to_tensor(g), v, lr, None, 0.9)
    np.testing.assert_allclose(p.numpy(), _class_step(paddle.optimizer.Momentum, p0, g, learning_rate=0.1,
                                                      momentum=0.9), rtol=1e-6)
    # adam (two steps through the beta-pow accumulators)
    p, m1, m2 = paddle.to_tensor(p0.copy()), paddle.zeros([6]), paddle.zeros([6])
    b1p, b2p = paddle.to_tensor([0.9]), paddle.to_tensor([0.999])
    for _ in range(2):
        paddle._C_ops.adam_(p, paddle.to_tensor(g), lr, m1, m2, b1p, b2p, None, None)
    lin = paddle.create_parameter([6], "float32")
    lin._t.data.copy_(torch.tensor(p0))
    opt = paddle.optimizer.Adam(0.1, parameters=[lin])
    for _ in range(2):
        lin._t.grad = torch.tensor(g)
        opt.step()
    np.testing.assert_allclose(p.numpy(), lin.numpy(), rtol=1e-5, atol=1e-6)
    assert abs(float(b1p.numpy()[0]) - 0.9 ** 3) < 1e-6
    # adagrad
    p, mom = paddle.to_tensor(p0.copy()), paddle.zeros([6])
    paddle._C_ops.adagrad_(p, paddle.to_tensor(g), mom, lr, None, 1e-6)
    np.testing.assert_allclose(p.numpy(), _class_step(paddle.optimizer.Adagrad, p0, g, learning_rate=0.1,
                                                      epsilon=1e-6), rtol=1e-5)
    # rmsprop
    p, ms, mom, mg = paddle.to_tensor(p0.copy()), paddle.zeros([6]), paddle.zeros([6]), paddle.zeros([6])
    paddle._C_ops.rmsprop_(p, ms, paddle.to_tensor(g), mom, lr, mg, None, 1e-6, 0.95, 0.0, False)
    np.testing.assert_allclose(p.numpy(), _class_step(paddle.optimizer.RMSProp, p0, g, learning_rate=0.1, rho=0.95,
                                                      epsilon=1e-6), rtol=1e-5)
    # adadelta: first step moves by -sqrt(eps / (0.05 g^2 + eps)) * g * lr
    p, asg, asu = paddle.to_tensor(p0.copy()), paddle.zeros([6]), paddle.zeros([6])
    paddle._C_ops.adadelta_(p, paddle.to_tensor(g), asg, asu, paddle.to_tensor([1.0]), None, 0.95, 1e-6)
    exp = p0 - np.sqrt(1e-6 / (0.05 * g * g + 1e-6)) * g
    np.testing.assert_allclose(p.numpy(), exp, rtol=1e-5)
    # lamb: trust-ratio-scaled adam direction
    p, m1, m2 = paddle.to_tensor(p0.copy()), paddle.zeros([6]), paddle.zeros([6])
    paddle._C_ops.lamb_(p, paddle.to_tensor(g), lr, m1, m2, paddle.to_tensor([1.0]), paddle.to_tensor([1.0]), None,
                        None, 0.01)
    r = (0.1 * g / 0.1) / (np.sqrt(0.001 * g * g / 0.001) + 1e-6) + 0.01 * p0
    exp = p0 - 0.1 * np.linalg.norm(p0) / np.linalg.norm(r) * r
    np.testing.assert_allclose(p.numpy(), exp, rtol=1e-4)


def test_fake_quant_ops():
    x = paddle.to_tensor(np.random.RandomState(3).randn(4, 16).astype("float32"))
    q, scale = paddle._C_ops.fake_quantize_abs_max(x, 8, 1)
    assert float(np.abs(q.numpy()).max()) <= 127 and np.allclose(q.numpy(), np.round(q.numpy()))
    dq, _ = paddle._C_ops.fake_quantize_dequantize_abs_max(x, 8, 1)
    assert np.abs(dq.numpy() - x.numpy()).max() <= float(scale.numpy()[0]) / 127 / 2 + 1e-6
    qc, sc = paddle._C_ops.fake_channel_wise_quantize_abs_max(x, 8, 1, 0)
    assert list(sc.shape) == [4]
    back = paddle._C_ops.fake_channel_wise_dequantize_max_abs(qc, [sc], [8], 0)
    np.testing.assert_allclose(back.numpy(), x.numpy(), atol=float(sc.numpy().max()) / 127)


def test_schema_backward_and_inplace_records():
    """Per-op backward kind (reference backward.yaml <op>_grad) and inplace pairing."""
    assert S.op_schema("exp")["backward"] == {"kind": "prim_vjp", "grad_op": "exp_grad"}
    assert S.op_schema("softmax")["backward"]["kind"] == "composite"
    assert S.op_schema("argmax")["backward"]["kind"] == "none"
    assert S.op_schema("equal")["backward"]["grad_op"] is None
    assert S.op_schema("flash_attn")["backward"]["kind"] in ("autograd", "composite")
    rec = S.op_schema("relu")
    assert rec["inplace_variant"] in (None, "relu_")
    if R.has_op("relu_"):
        assert S.op_schema("relu_")["inplace_of"] == "relu"
    kinds = {S.op_schema(n)["backward"]["kind"] for n in R.list_ops()[:600:5]}
    assert {"none", "autograd"} <= kinds
