"""nn layers, losses, optimizers and LR schedulers vs NumPy / closed-form references
(reference test strategy: test/legacy_test/test_adamw_op.py, test_lr_scheduler.py, test_layers.py)."""
import math

import numpy as np
import pytest
import torch

import paddle2_amd as paddle
import paddle2_amd.nn.functional as F


def test_linear_layout_and_state_dict_roundtrip(tmp_path):
    paddle.seed(0)
    lin = paddle.nn.Linear(4, 3)
    assert lin.weight.shape == [4, 3] and lin.bias.shape == [3]
    x = paddle.randn([2, 4])
    ref = x.numpy() @ lin.weight.numpy() + lin.bias.numpy()
    np.testing.assert_allclose(lin(x).numpy(), ref, rtol=1e-5)
    path = str(tmp_path / "m.pdparams")
    paddle.save(lin.state_dict(), path)
    lin2 = paddle.nn.Linear(4, 3)
    lin2.set_state_dict(paddle.load(path))
    np.testing.assert_array_equal(lin2.weight.numpy(), lin.weight.numpy())


def test_layer_containers_and_hooks():
    seq = paddle.nn.Sequential(paddle.nn.Linear(4, 8), paddle.nn.ReLU(), paddle.nn.Linear(8, 2))
    names = [n for n, _ in seq.named_parameters()]
    assert names == ["0.weight", "0.bias", "2.weight", "2.bias"]
    seen = []
    h = seq[0].register_forward_post_hook(lambda l, i, o: seen.append(o.shape))
    seq(paddle.randn([3, 4]))
    h.remove()
    seq(paddle.randn([3, 4]))
    assert seen == [[3, 8]]
    ll = paddle.nn.LayerList([paddle.nn.Linear(2, 2) for _ in range(3)])
    assert len(ll) == 3 and len(list(ll.parameters())) == 6
    seq.eval()
    assert not seq.training
    seq.train()
    assert seq[1].training


def test_norm_layers_vs_numpy():
    x = np.random.randn(4, 6).astype("float32")
    ln = paddle.nn.LayerNorm(6)
    mu, var = x.mean(-1, keepdims=True), x.var(-1, keepdims=True)
    np.testing.assert_allclose(ln(paddle.to_tensor(x)).numpy(), (x - mu) / np.sqrt(var + 1e-5), rtol=1e-4, atol=1e-5)
    rms = paddle.nn.RMSNorm(6) if hasattr(paddle.nn, "RMSNorm") else None
    if rms is not None:
        ref = x / np.sqrt((x ** 2).mean(-1, keepdims=True) + 1e-6)
        np.testing.assert_allclose(rms(paddle.to_tensor(x)).numpy(), ref, rtol=1e-3, atol=1e-4)
    bn = paddle.nn.BatchNorm1D(6)
    y = bn(paddle.to_tensor(x)).numpy()
    np.testing.assert_allclose(y.mean(0), np.zeros(6), atol=1e-5)


def test_conv_pool_shapes():
    x = paddle.randn([2, 3, 16, 16])
    conv = paddle.nn.Conv2D(3, 8, 3, stride=2, padding=1)
    assert conv.weight.shape == [8, 3, 3, 3]
    y = conv(x)
    assert y.shape == [2, 8, 8, 8]
    assert paddle.nn.MaxPool2D(2, 2)(y).shape == [2, 8, 4, 4]
    assert paddle.nn.AdaptiveAvgPool2D(1)(y).shape == [2, 8, 1, 1]
    assert F.interpolate(y, scale_factor=2, mode="nearest").shape == [2, 8, 16, 16]


def test_losses_vs_numpy():
    logits = np.random.randn(5, 7).astype("float32")
    lab = np.random.randint(0, 7, (5,))
    lse = np.log(np.exp(logits).sum(1))
    ref = (lse - logits[np.arange(5), lab]).mean()
    out = F.cross_entropy(paddle.to_tensor(logits), paddle.to_tensor(lab))
    assert float(out) == pytest.approx(ref, rel=1e-5)
    # soft label + ignore_index
    lab2 = lab.copy()
    lab2[0] = -100
    out2 = F.cross_entropy(paddle.to_tensor(logits), paddle.to_tensor(lab2), ignore_index=-100)
    ref2 = (lse - logits[np.arange(5), np.where(lab2 < 0, 0, lab2)])[1:].mean()
    assert float(out2) == pytest.approx(ref2, rel=1e-5)
    a, b = np.random.rand(4, 3).astype("float32"), np.random.rand(4, 3).astype("float32")
    assert float(F.mse_loss(paddle.to_tensor(a), paddle.to_tensor(b))) == pytest.approx(((a - b) ** 2).mean(), rel=1e-5)
    assert float(F.l1_loss(paddle.to_tensor(a), paddle.to_tensor(b))) == pytest.approx(np.abs(a - b).mean(), rel=1e-5)
    p = 1 / (1 + np.exp(-a))
    bce = -(b * np.log(p) + (1 - b) * np.log(1 - p)).mean()
    assert float(F.binary_cross_entropy_with_logits(paddle.to_tensor(a), paddle.to_tensor(b))) == pytest.approx(
        bce, rel=1e-5)


def test_activations():
    a = np.linspace(-3, 3, 13).astype("float32")
    x = paddle.to_tensor(a)
    np.testing.assert_allclose(F.relu(x).numpy(), np.maximum(a, 0))
    np.testing.assert_allclose(F.sigmoid(x).numpy(), 1 / (1 + np.exp(-a)), rtol=1e-5)
    np.testing.assert_allclose(F.silu(x).numpy(), a / (1 + np.exp(-a)), rtol=1e-5)
    np.testing.assert_allclose(F.softmax(x).numpy(), np.exp(a) / np.exp(a).sum(), rtol=1e-5)
    g = F.gelu(x).numpy()
    ref = 0.5 * a * (1 + np.vectorize(math.erf)(a / np.sqrt(2)))
    np.testing.assert_allclose(g, ref, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(F.leaky_relu(x, 0.1).numpy(), np.where(a > 0, a, 0.1 * a), rtol=1e-6)


def _np_adamw(p, g, m, v, t, lr, b1, b2, eps, wd):
    p = p * (1 - lr * wd)
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    mh = m / (1 - b1 ** t)
    vh = v / (1 - b2 ** t)
    return p - lr * mh / (np.sqrt(vh) + eps), m, v


def test_adamw_matches_numpy():
    w0 = np.random.randn(5, 3).astype("float32")
    lin = paddle.nn.Linear(5, 3, bias_attr=False)
    lin.weight.set_value(w0)
    opt = paddle.optimizer.AdamW(learning_rate=0.01, parameters=lin.parameters(), weight_decay=0.1)
    x = np.random.randn(4, 5).astype("float32")
    p, m, v = w0.astype("float64"), np.zeros_like(w0, dtype="float64"), np.zeros_like(w0, dtype="float64")
    for t in range(1, 4):
        loss = (lin(paddle.to_tensor(x)) ** 2).sum()
        loss.backward()
        g = lin.weight.grad.numpy().astype("float64")
        opt.step()
        opt.clear_grad()
        p, m, v = _np_adamw(p, g, m, v, t, 0.01, 0.9, 0.999, 1e-8, 0.1)
        np.testing.assert_allclose(lin.weight.numpy(), p, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("name", ["SGD", "Momentum", "Adam", "Adamax", "Adagrad", "RMSProp", "Adadelta", "Lamb",
                                  "NAdam", "RAdam"])
def test_optimizers_decrease_quadratic(name):
    paddle.seed(0)
    w = paddle.create_parameter([8], "float32", default_initializer=paddle.nn.initializer.Constant(2.0))
    cls = getattr(paddle.optimizer, name)
    lr = 1.0 if name == "Adadelta" else 0.05
    opt = cls(learning_rate=lr, parameters=[w])
    first = None
    for _ in range(30):
        loss = (w * w).sum()
        if first is None:
            first = float(loss)
        loss.backward()
        opt.step()
        opt.clear_grad()
    assert float((w * w).sum()) < first


def test_optimizer_state_dict_names():
    lin = paddle.nn.Linear(2, 2)
    opt = paddle.optimizer.Adam(0.1, parameters=lin.parameters())
    lin(paddle.randn([1, 2])).sum().backward()
    opt.step()
    sd = opt.state_dict()
    keys = [k for k in sd if k.endswith("_moment1_0")]
    assert len(keys) == 2
    opt2 = paddle.optimizer.Adam(0.1, parameters=lin.parameters())
    opt2.set_state_dict(sd)


def test_lr_schedulers():
    s = paddle.optimizer.lr.StepDecay(1.0, step_size=2, gamma=0.5)
    vals = []
    for _ in range(5):
        vals.append(s())
        s.step()
    assert vals == [1.0, 1.0, 0.5, 0.5, 0.25]
    c = paddle.optimizer.lr.CosineAnnealingDecay(1.0, T_max=10)
    for _ in range(10):
        c.step()
    assert c() == pytest.approx(0.0, abs=1e-6)
    w = paddle.optimizer.lr.LinearWarmup(0.5, warmup_steps=4, start_lr=0.0, end_lr=0.5)
    got = []
    for _ in range(6):
        got.append(w())
        w.step()
    assert got[:5] == pytest.approx([0.0, 0.125, 0.25, 0.375, 0.5])
    n = paddle.optimizer.lr.NoamDecay(d_model=512, warmup_steps=4000)
    n.step()
    assert n() > 0
    pw = paddle.optimizer.lr.PiecewiseDecay([2, 4], [1.0, 0.5, 0.1])
    out = []
    for _ in range(6):
        out.append(pw())
        pw.step()
    assert out == [1.0, 1.0, 0.5, 0.5, 0.1, 0.1]


def test_grad_clip_global_norm_cpu():
    w = paddle.create_parameter([4], "float32", default_initializer=paddle.nn.initializer.Constant(1.0))
    opt = paddle.optimizer.SGD(1.0, parameters=[w], grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    (w * paddle.to_tensor([3.0, 4.0, 0.0, 0.0])).sum().backward()
    opt.step()
    np.testing.assert_allclose(w.numpy(), [1 - 0.6, 1 - 0.8, 1, 1], rtol=1e-5)


def test_multi_precision_master_weights_cpu():
    lin = paddle.nn.Linear(4, 4)
    lin.to(dtype="bfloat16")
    opt = paddle.optimizer.AdamW(1e-3, parameters=lin.parameters(), multi_precision=True)
    lin(paddle.randn([2, 4]).astype("bfloat16")).astype("float32").sum().backward()
    opt.step()
    sd = opt.state_dict()
    assert "master_weights" in sd and len(sd["master_weights"]) == 2
    assert all(v.dtype == paddle.float32 for v in sd["master_weights"].values())


def test_auto_cast_custom_lists_are_honoured():
    """custom_white_list / custom_black_list (reference amp/auto_cast.py:1029) override the defaults at this
    framework's op entry points: a black-listed matmul runs in fp32, a white-listed softmax in the AMP
    dtype; an op in both lists is an error."""
    import pytest
    import torch

    import paddle2_amd as paddle

    x = paddle.to_tensor(torch.randn(4, 8))
    w = paddle.to_tensor(torch.randn(8, 3))
    with paddle.amp.auto_cast(custom_black_list={"matmul"}, dtype="bfloat16"):
        y = paddle.matmul(x, w)
        s = paddle.nn.functional.softmax(x)
    assert y._t.dtype == torch.float32 and s._t.dtype == torch.float32
    with paddle.amp.auto_cast(custom_white_list={"softmax"}, dtype="bfloat16"):
        s = paddle.nn.functional.softmax(x)
        m = paddle.mean(x)
    assert s._t.dtype == torch.bfloat16 and m._t.dtype == torch.float32
    with pytest.raises(ValueError):
        with paddle.amp.auto_cast(custom_white_list={"exp"}, custom_black_list={"exp"}):
            pass
