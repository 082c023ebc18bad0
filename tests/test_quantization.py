"""paddle.quantization / paddle.nn.quant (reference tests: test/quantization/test_qat.py, test_ptq.py,
test/legacy_test/test_weight_only_linear.py, test_weight_quantize_op.py, test_llm_int8_linear.py,
test_imperative_qat.py).  Weight-only GPU kernel numerics vs a PyTorch fp32 reference."""
import numpy as np
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.nn import quant as Q
from paddle2_amd.quantization import PTQ, QAT, QuantConfig
from paddle2_amd.quantization.observers import AbsmaxObserver
from paddle2_amd.quantization.quanters import FakeQuanterWithAbsMaxObserver


@pytest.mark.parametrize("algo,group", [("weight_only_int8", -1), ("weight_only_int8", 64), ("weight_only_int4", -1),
                                        ("weight_only_int4", 128), ("llm.int8", -1)])
def test_weight_quantize_roundtrip(algo, group):
    torch.manual_seed(0)
    w = paddle.Tensor._wrap(torch.randn(256, 128))
    q, s = Q.weight_quantize(w, algo=algo, group_size=group)
    bits = 4 if algo == "weight_only_int4" else 8
    assert q.dtype == paddle.int8
    assert q.shape == ([128 // 2, 256] if bits == 4 else [128, 256])
    assert s.shape == ([128] if group == -1 else [256 // group, 128])
    wd = Q.weight_dequantize(q, s, algo=algo, out_dtype="float32", group_size=group)
    assert wd.shape == [256, 128]
    step = (w._t.abs().amax(0) / (2 ** (bits - 1) - 1)).max()
    assert float((wd._t - w._t).abs().max()) <= float(step) * 0.5 + 1e-6


def test_weight_only_linear_and_llm_int8_cpu():
    torch.manual_seed(1)
    x = paddle.Tensor._wrap(torch.randn(3, 5, 256))
    w = torch.randn(256, 128) * 0.05
    q, s = Q.weight_quantize(paddle.Tensor._wrap(w))
    b = paddle.Tensor._wrap(torch.randn(128))
    y = Q.weight_only_linear(x, q, b, s)
    ref = x._t @ Q.weight_dequantize(q, s, out_dtype="float32")._t + b._t
    torch.testing.assert_close(y._t, ref, atol=1e-4, rtol=1e-4)
    q8, s8 = Q.weight_quantize(paddle.Tensor._wrap(w), algo="llm.int8")
    y8 = Q.llm_int8_linear(x, q8, None, s8, threshold=6.0)
    torch.testing.assert_close(y8._t, x._t @ w, atol=0.05, rtol=0.05)
    xo = x._t.clone()
    xo[..., 7] = 20.0  # outlier feature runs in floating point
    y8o = Q.llm_int8_linear(paddle.Tensor._wrap(xo), q8, None, s8, threshold=6.0)
    torch.testing.assert_close(y8o._t, xo @ w, atol=0.1, rtol=0.05)


def test_fake_quant_layers_ste():
    x = paddle.Tensor._wrap(torch.linspace(-1, 1, 11).requires_grad_())
    for layer in (Q.FakeQuantAbsMax(quant_bits=4), Q.FakeQuantMovingAverageAbsMax(quant_bits=4)):
        y = layer(x)
        lv = set(np.round(y.numpy() * 7, 4))
        assert len(lv) <= 15
        y.sum().backward()
        np.testing.assert_allclose(x.grad.numpy(), np.ones(11))
        x.clear_gradient()
    cw = Q.FakeQuantChannelWiseAbsMax(channel_num=3, quant_axis=0)
    out = cw(paddle.randn([3, 8]))
    assert out.shape == [3, 8]
    fp8 = Q.fake_fp8_dequant(Q.fake_fp8_quant(paddle.to_tensor([0.5, -1.0]), paddle.to_tensor(1.0)),
                             paddle.to_tensor(1.0))
    np.testing.assert_allclose(fp8.numpy(), [0.5, -1.0], rtol=1e-2)


def _mlp():
    paddle.seed(2)
    return paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.ReLU(), paddle.nn.Linear(16, 4))


def test_qat_train_convert_matches():
    m = _mlp()
    q = FakeQuanterWithAbsMaxObserver(moving_rate=0.9)
    qat = QAT(QuantConfig(activation=q, weight=q))
    qm = qat.quantize(m)
    assert type(qm[0]).__name__ == "QuantedLinear" and type(m[0]).__name__ == "Linear"
    opt = paddle.optimizer.SGD(learning_rate=0.01, parameters=qm.parameters())
    for _ in range(3):
        loss = qm(paddle.randn([16, 8])).square().mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
    qm.eval()
    x = paddle.randn([4, 8])
    ref = qm(x)
    cm = qat.convert(qm)
    w = cm[0].weight.numpy()
    assert np.allclose(w, np.round(w)) and np.abs(w).max() <= 127
    torch.testing.assert_close(cm(x)._t, ref._t, atol=1e-5, rtol=1e-5)


def test_ptq_observers_and_layer_config():
    m = _mlp()
    cfg = QuantConfig(activation=None, weight=None)
    cfg.add_layer_config([m[0]], activation=AbsmaxObserver(), weight=AbsmaxObserver())
    pm = PTQ(cfg).quantize(m)
    assert type(pm[0]).__name__ == "QuantedLinear" and type(pm[2]).__name__ == "Linear"
    x = paddle.randn([32, 8])
    pm(x)
    assert abs(float(pm[0].activation_quanter.scales()) - float(x.abs().max())) < 1e-6
    cm = PTQ(cfg).convert(pm)
    assert cm[0].converted


def test_imperative_qat_and_ptq(tmp_path):
    from paddle2_amd.quantization import (AbsmaxQuantizer, HistQuantizer, ImperativePTQ, ImperativeQuantAware,
                                          KLQuantizer, PerChannelAbsmaxQuantizer, PTQConfig)

    m = ImperativeQuantAware(weight_quantize_type="channel_wise_abs_max").quantize(_mlp())
    assert type(m[0]).__name__ == "QuantizedLinear"
    y = m(paddle.randn([4, 8]))
    y.sum().backward()
    for act in (AbsmaxQuantizer(), HistQuantizer(), KLQuantizer()):
        ptq = ImperativePTQ(PTQConfig(act, PerChannelAbsmaxQuantizer()))
        pm = ptq.quantize(_mlp())
        for _ in range(3):
            pm(paddle.randn([64, 8]))
        ptq._calc(pm)
        th = pm[0]._quant_config.out_act_quantizer.thresholds[0]
        assert 0 < th <= pm[0]._quant_config.out_act_quantizer.abs_max_vals[0] + 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("wd", ["int8", "int4"])
@pytest.mark.parametrize("group", [-1, 64, 128])
@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (5, 256, 512), (16, 11008, 4096), (33, 512, 1024),
                                   (64, 128, 8192), (8, 4096, 11008)])
def test_weight_only_kernel_matches_fp32(wd, group, M, N, K):
    from paddle2_amd.ops import weight_only as WO

    torch.manual_seed(0)
    w = torch.randn(K, N, device="cuda") * 0.02
    q, s = Q.weight_quantize(paddle.Tensor._wrap(w), algo=f"weight_only_{wd}", group_size=group)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    assert WO._native_ok(x, q._t, wd, group)
    y = WO.weight_only_matmul(x, q._t, s._t, wd, group)
    ref = x.float() @ WO.dequantize(q._t, s._t, wd, group, torch.float32).t()
    torch.testing.assert_close(y.float(), ref, atol=2e-2 * ref.abs().max().item() ** 0.5 + 1e-3, rtol=2e-2)


@pytest.mark.gpu
def test_weight_only_linear_bias_gpu():
    torch.manual_seed(3)
    w = torch.randn(1024, 512, device="cuda") * 0.03
    q, s = Q.weight_quantize(paddle.Tensor._wrap(w), algo="weight_only_int8")
    x = paddle.Tensor._wrap(torch.randn(2, 3, 1024, device="cuda").to(torch.bfloat16))
    b = paddle.Tensor._wrap(torch.randn(512, device="cuda").to(torch.bfloat16))
    y = Q.weight_only_linear(x, q, b, s)
    ref = x._t.float() @ Q.weight_dequantize(q, s, out_dtype="float32")._t + b._t.float()
    assert y.shape == [2, 3, 512] and y.dtype == paddle.bfloat16
    torch.testing.assert_close(y._t.float(), ref, atol=3e-2, rtol=2e-2)
