"""3x3 / stride 1 / padding 1 NHWC convolution on the implicit-GEMM MFMA kernel (ops/conv_gemm.py, gemm7.hip SCHED
bit 11) against an fp32 PyTorch conv2d: forward, dx and dW, including Cin = 64 (K = 576: odd K-tile count, padded
with a zero tap), channel counts 64..256 and a ResNet-50 stage-1 shape; plus the routing (strided 3x3 stays on
MIOpen)."""
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


@pytest.mark.parametrize("N,H,W,Ci,Co", [(2, 8, 8, 64, 64), (2, 14, 14, 128, 64), (4, 7, 7, 64, 128),
                                         (1, 5, 9, 256, 128), (16, 56, 56, 64, 64)])
def test_conv3x3_native_matches_fp32(N, H, W, Ci, Co):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, W, Ci, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(Co, Ci, 3, 3, device=dev, generator=g) * (9 * Ci) ** -0.5).to(torch.bfloat16)
    dy = torch.randn(N, H, W, Co, device=dev, generator=g).to(torch.bfloat16)
    xr, wr = x.float().permute(0, 3, 1, 2).requires_grad_(), w.float().requires_grad_()
    yr = F.conv2d(xr, wr, None, 1, 1).permute(0, 2, 3, 1)
    yr.backward(dy.float())

    px = paddle.to_tensor(x, stop_gradient=False)
    pw = paddle.to_tensor(w, stop_gradient=False)
    before = CG.calls["3x3"]
    y = paddle.nn.functional.conv2d(px, pw, padding=1, data_format="NHWC")
    assert CG.calls["3x3"] == before + 1, "the 3x3 conv did not take the implicit-GEMM path"
    y.backward(paddle.to_tensor(dy))
    assert tuple(y.shape) == tuple(yr.shape)
    assert _rel(y._t, yr) < 8e-3
    assert _rel(px.grad._t.float(), xr.grad.permute(0, 2, 3, 1)) < 8e-3
    assert _rel(pw.grad._t.float(), wr.grad) < 8e-3


def test_strided_3x3_stays_on_miopen():
    x = paddle.to_tensor(torch.randn(2, 8, 8, 64, device=dev).to(torch.bfloat16))
    w = paddle.to_tensor(torch.randn(64, 64, 3, 3, device=dev).to(torch.bfloat16))
    before = CG.calls["3x3"]
    paddle.nn.functional.conv2d(x, w, stride=2, padding=1, data_format="NHWC")
    assert CG.calls["3x3"] == before
