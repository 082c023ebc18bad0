"""Channels-last 1x1 convolutions on the native MFMA GEMM (nn/functional/conv.py `_Conv1x1Fn`) against an fp32
PyTorch conv2d of the same op: forward, dx, dW and db, stride 1 and 2, channel counts off the 128/256 tiles,
the ResNet-50 bottleneck widths; plus the routing (padded / NCHW 1x1 convs do not take it).
"""
import pytest
import torch
import torch.nn.functional as F

import paddle2_amd as paddle
from paddle2_amd.ops import conv_gemm as CG

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(autouse=True)
def _native_conv(monkeypatch):
    """These tests pin the native kernels (the default "auto" mode may route a shape to MIOpen)."""
    monkeypatch.setattr(CG, "MODE", "native")


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("N,H,W,Ci,Co,stride,bias", [
    (2, 8, 8, 64, 256, 1, False),      # K = 64: below the 128 K-tile
    (4, 14, 14, 256, 64, 1, True),
    (2, 28, 28, 512, 128, 2, False),   # the downsample projection
    (2, 7, 7, 2048, 512, 1, False),
    (3, 5, 9, 72, 200, 1, True),       # ragged everything
    (32, 56, 56, 64, 256, 1, False),   # a full ResNet-50 stage-1 expansion at batch 32
])
def test_conv1x1_native_matches_fp32(N, H, W, Ci, Co, stride, bias):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, W, Ci, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(Co, Ci, 1, 1, device=dev, generator=g) * Ci ** -0.5).to(torch.bfloat16)
    b = torch.randn(Co, device=dev, generator=g).to(torch.bfloat16) if bias else None
    dy = torch.randn(N, (H - 1) // stride + 1, (W - 1) // stride + 1, Co, device=dev, generator=g).to(torch.bfloat16)

    xr, wr = x.float().permute(0, 3, 1, 2).requires_grad_(), w.float().requires_grad_()
    br = b.float().requires_grad_() if bias else None
    yr = F.conv2d(xr, wr, br, stride).permute(0, 2, 3, 1)
    yr.backward(dy.float())

    px = paddle.to_tensor(x, stop_gradient=False)
    pw = paddle.to_tensor(w, stop_gradient=False)
    pb = paddle.to_tensor(b, stop_gradient=False) if bias else None
    before = CG.calls["1x1"]
    y = paddle.nn.functional.conv2d(px, pw, pb, stride=stride, data_format="NHWC")
    assert CG.calls["1x1"] == before + 1, "the 1x1 conv did not take the native GEMM path"
    y.backward(paddle.to_tensor(dy))
    assert tuple(y.shape) == tuple(yr.shape)
    assert _rel(y._t, yr) < 8e-3
    assert _rel(px.grad._t.float(), xr.grad.permute(0, 2, 3, 1)) < 8e-3
    assert _rel(pw.grad._t.float(), wr.grad) < 8e-3
    if bias:
        assert _rel(pb.grad._t.float(), br.grad) < 8e-3


def test_other_convs_stay_on_miopen():
    x = paddle.to_tensor(torch.randn(2, 8, 8, 64, device=dev).to(torch.bfloat16))
    w3 = paddle.to_tensor(torch.randn(64, 64, 3, 3, device=dev).to(torch.bfloat16))
    w1 = paddle.to_tensor(torch.randn(64, 64, 1, 1, device=dev).to(torch.bfloat16))
    before = CG.calls["1x1"]
    paddle.nn.functional.conv2d(x, w3, padding=1, data_format="NHWC")
    paddle.nn.functional.conv2d(x, w1, padding=1, data_format="NHWC")
    xn = paddle.to_tensor(x._t.permute(0, 3, 1, 2).contiguous())
    paddle.nn.functional.conv2d(xn, w1)
    assert CG.calls["1x1"] == before


def test_auto_route_times_once_and_matches(monkeypatch):
    """MODE auto: the first call of a shape times native vs MIOpen and caches the decision; either route gives
    the fp32 reference's result."""
    monkeypatch.setattr(CG, "MODE", "auto")
    monkeypatch.setattr(CG, "_ROUTE", {})
    x = torch.randn(4, 14, 14, 64, device=dev, dtype=torch.bfloat16)
    w = torch.randn(128, 64, 1, 1, device=dev, dtype=torch.bfloat16) * 0.1
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float()).permute(0, 2, 3, 1)
    for _ in range(2):
        y = paddle.nn.functional.conv2d(paddle.to_tensor(x), paddle.to_tensor(w), data_format="NHWC")
        assert _rel(y._t, ref) < 1e-2
    assert len(CG._ROUTE) == 1
