"""Fused channels-last BatchNorm(+add+ReLU) HIP kernel vs a PyTorch fp32 reference
(reference tests: test/legacy_test/test_batch_norm_op.py, test_fused_bn_add_act.py)."""
import pytest
import torch
import torch.nn.functional as F

import paddle2_amd as paddle
from paddle2_amd.ops.torch_ops import _BNActFn, batch_norm_act


def _ref(x, rm, rv, w, b, training, momentum, eps, relu, z):
    t = x.float().movedim(-1, 1)
    y = F.batch_norm(t, rm, rv, w.float(), b.float(), training, 1.0 - momentum, eps).movedim(1, -1)
    if z is not None:
        y = y + z.float()
    return torch.relu(y) if relu else y


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(8, 14, 14, 64), (4, 7, 7, 2048), (3, 5, 7, 256), (2, 56, 56, 128), (5, 3, 3, 40)])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True), (False, True)])
def test_bn_act_train_matches_fp32(dtype, shape, relu, res):
    torch.manual_seed(0)
    dev = "cuda"
    C = shape[-1]
    x = (torch.randn(shape, device=dev) * 2 + 0.5).to(dtype).requires_grad_()
    z = torch.randn(shape, device=dev).to(dtype).requires_grad_() if res else None
    w = (torch.rand(C, device=dev) + 0.5).requires_grad_()
    b = torch.randn(C, device=dev).requires_grad_()
    rm, rv = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    rm2, rv2 = rm.clone(), rv.clone()
    y = batch_norm_act(x, rm, rv, w, b, True, 0.9, 1e-5, "relu" if relu else None, z)
    assert y.dtype == dtype
    xr = x.detach().float().requires_grad_()
    zr = z.detach().float().requires_grad_() if res else None
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr = _ref(xr, rm2, rv2, wr, br, True, 0.9, 1e-5, relu, zr)
    tol = dict(atol=2e-2, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(rm, rm2, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(rv, rv2, atol=1e-3, rtol=1e-3)
    gy = torch.randn(shape, device=dev)
    y.backward(gy.to(dtype))
    yr.backward(gy.to(dtype).float())
    gtol = dict(atol=5e-2, rtol=5e-2) if dtype == torch.bfloat16 else dict(atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(x.grad.float(), xr.grad, **gtol)
    M = x.numel() // C
    torch.testing.assert_close(w.grad, wr.grad, atol=gtol["atol"] * M ** 0.5, rtol=gtol["rtol"])
    torch.testing.assert_close(b.grad, br.grad, atol=gtol["atol"] * M ** 0.5, rtol=gtol["rtol"])
    if res:
        torch.testing.assert_close(z.grad.float(), zr.grad, **gtol)


@pytest.mark.gpu
def test_bn_act_uses_native_and_eval_apply():
    dev = "cuda"
    x = torch.randn(4, 8, 8, 64, device=dev, dtype=torch.bfloat16)
    w, b = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev)
    rm, rv = torch.randn(64, device=dev), torch.rand(64, device=dev) + 0.5
    y = batch_norm_act(x.requires_grad_(), rm, rv, w, b, True, 0.9, 1e-5, "relu")
    assert y.grad_fn is not None and type(y.grad_fn).__name__.startswith(_BNActFn.__name__)
    with torch.no_grad():
        ye = batch_norm_act(x, rm, rv, w, b, False, 0.9, 1e-5, "relu")
    torch.testing.assert_close(ye.float(), _ref(x, rm, rv, w, b, False, 0.9, 1e-5, True, None), atol=3e-2, rtol=2e-2)


@pytest.mark.gpu
def test_resnet_block_fused_matches_unfused():
    from paddle2_amd.vision.models.resnet import BottleneckBlock

    paddle.seed(3)
    paddle.set_device("gpu")
    blk = BottleneckBlock(256, 64, data_format="NHWC")
    x = paddle.randn([4, 14, 14, 256])
    y = blk(x)
    # unfused reference: same layers through the composite path on the same parameters
    def ref(t):
        def bn(l, v):
            return F.batch_norm(v.movedim(-1, 1), None, None, l.weight._t, l.bias._t, True, 0.1, l._epsilon
                                ).movedim(1, -1)

        o = torch.relu(bn(blk.bn1, blk.conv1(paddle.Tensor._wrap(t))._t))
        o = torch.relu(bn(blk.bn2, blk.conv2(paddle.Tensor._wrap(o))._t))
        return torch.relu(bn(blk.bn3, blk.conv3(paddle.Tensor._wrap(o))._t) + t)

    torch.testing.assert_close(y._t, ref(x._t), atol=1e-3, rtol=1e-3)


def test_batchnorm_layer_fused_args_cpu():
    paddle.seed(0)
    for fmt in ("NHWC", "NCHW"):
        bn = paddle.nn.BatchNorm2D(16, data_format=fmt)
        shp = [2, 5, 5, 16] if fmt == "NHWC" else [2, 16, 5, 5]
        x, z = paddle.randn(shp), paddle.randn(shp)
        y = bn(x, residual=z, act="relu")
        bn2 = paddle.nn.BatchNorm2D(16, data_format=fmt)
        yr = paddle.nn.functional.relu(bn2(x) + z)
        torch.testing.assert_close(y._t, yr._t)
        torch.testing.assert_close(bn._mean._t, bn2._mean._t)
    legacy = paddle.nn.BatchNorm(16, act="relu")
    assert float(legacy(paddle.randn([2, 16, 3, 3])).min()) >= 0
