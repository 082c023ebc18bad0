"""Fused masked softmax (paddle.incubate.softmax_mask_fuse / softmax_mask_fuse_upper_triangle) and
_C_ops.fused_linear_param_grad_add.  Reference tests: test/legacy_test/test_softmax_mask_fuse_op.py,
test_softmax_mask_fuse_upper_triangle_op.py, test_fused_linear_param_grad_add.py.  The HIP kernel
(csrc/kernels/softmax_mask.hip) is compared against a plain fp32 PyTorch softmax, forward and backward."""
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd import _C_ops
from paddle2_amd.ops import torch_ops as T


def _ref(x, mask, causal):
    xf = x.float()
    if causal:
        S = x.shape[-1]
        xf = xf.masked_fill(~torch.ones(S, S, dtype=torch.bool, device=x.device).tril(), float("-inf"))
    else:
        xf = xf + mask.float()
    return torch.softmax(xf, -1)


def test_softmax_mask_fuse_api_cpu():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 3, 5, 7, generator=g)
    m = torch.where(torch.rand(2, 1, 5, 7, generator=g) > 0.3, 0.0, -1e4)
    y = paddle.incubate.softmax_mask_fuse(paddle.to_tensor(x), paddle.to_tensor(m))
    torch.testing.assert_close(y._t, _ref(x, m, False))
    x2 = torch.randn(2, 3, 6, 6, generator=g)
    y2 = paddle.incubate.softmax_mask_fuse_upper_triangle(paddle.to_tensor(x2))._t
    torch.testing.assert_close(y2, _ref(x2, None, True))
    assert float(y2.triu(1).abs().max()) == 0.0
    with pytest.raises(ValueError):
        T.softmax_mask(torch.randn(1, 1, 4, 5), None, causal=True)


def test_fused_linear_param_grad_add_cpu():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(4, 6, 8, generator=g)
    dy = torch.randn(4, 6, 5, generator=g)
    dw0 = torch.randn(8, 5, generator=g)
    db0 = torch.randn(5, generator=g)
    dw, db = _C_ops.fused_linear_param_grad_add(paddle.to_tensor(x), paddle.to_tensor(dy),
                                                paddle.to_tensor(dw0.clone()), paddle.to_tensor(db0.clone()), True,
                                                True)
    torch.testing.assert_close(dw._t, dw0 + x.reshape(-1, 8).t() @ dy.reshape(-1, 5), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(db._t, db0 + dy.reshape(-1, 5).sum(0), rtol=1e-5, atol=1e-5)
    dw1, db1 = _C_ops.fused_linear_param_grad_add(paddle.to_tensor(x), paddle.to_tensor(dy), None, None, True, False)
    assert db1 is None and dw1._t.dtype == torch.float32


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("S", [37, 128, 1000, 4096])
def test_softmax_mask_hip_matches_fp32(dtype, causal, S):
    g = torch.Generator().manual_seed(S)
    B, H = 2, 3
    Sq = S if causal else min(S, 64)
    x = (torch.randn(B, H, Sq, S, generator=g) * 3).to("cuda", dtype).requires_grad_(True)
    m = torch.where(torch.rand(B, 1, Sq, S, generator=g) > 0.2, 0.0, -1e4).to("cuda", dtype)
    y = T.softmax_mask(x, None if causal else m, causal=causal)
    assert isinstance(y.grad_fn, torch.autograd.function.BackwardCFunction), "HIP path not taken"
    ref = _ref(x.detach(), m, causal)
    tol = {torch.float32: 1e-5, torch.bfloat16: 1e-2, torch.float16: 2e-3}[dtype]
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    if causal:
        assert float(y.detach().float().triu(1).abs().max()) == 0.0
    dy = torch.randn(B, H, Sq, S, generator=g).to("cuda", dtype)
    (dx,) = torch.autograd.grad(y, x, dy)
    xr = x.detach().float().requires_grad_(True)
    (dxr,) = torch.autograd.grad(_ref(xr, m, causal), xr, dy.float())
    torch.testing.assert_close(dx.float(), dxr, rtol=tol * 4, atol=tol * 4)


@pytest.mark.gpu
def test_softmax_mask_hip_max_len():
    x = torch.randn(1, 2, 4, 8192, device="cuda", dtype=torch.bfloat16)
    m = torch.zeros(1, 1, 4, 8192, device="cuda", dtype=torch.bfloat16)
    y = paddle.incubate.softmax_mask_fuse(paddle.to_tensor(x), paddle.to_tensor(m))._t
    torch.testing.assert_close(y.float(), _ref(x, m, False), rtol=1e-2, atol=1e-4)


def _flpga_bf16_case(device):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 300, 64, generator=g).to(torch.bfloat16)
    dy = torch.randn(2, 300, 48, generator=g).to(torch.bfloat16)
    dw0 = torch.randn(64, 48, generator=g)
    ref = dw0.double() + x.reshape(-1, 64).double().t() @ dy.reshape(-1, 48).double()
    dw, _ = _C_ops.fused_linear_param_grad_add(paddle.to_tensor(x.to(device)), paddle.to_tensor(dy.to(device)),
                                               paddle.to_tensor(dw0.clone().to(device)), None, True, False)
    assert dw._t.dtype == torch.float32
    # fp32 accumulation of exact bf16 products: far below one bf16 ulp of the product
    err = float((dw._t.double().cpu() - ref).abs().max() / ref.abs().max())
    assert err < 1e-6, err


def test_fused_linear_param_grad_add_bf16_fp32_main_grad_cpu():
    _flpga_bf16_case("cpu")


@pytest.mark.gpu
def test_fused_linear_param_grad_add_bf16_fp32_main_grad_gpu():
    _flpga_bf16_case("cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("S", [4097, 1001])
def test_softmax_mask_ragged_long_rows_gpu(S):
    """Sk not a multiple of the 16-byte vector (scalar-chunk path): fwd + bwd vs fp32."""
    g = torch.Generator().manual_seed(S)
    x = (torch.randn(1, 2, 8, S, generator=g) * 3).to("cuda", torch.bfloat16).requires_grad_(True)
    m = torch.where(torch.rand(1, 1, 8, S, generator=g) > 0.2, 0.0, -1e9)  # fp32 mask, huge negatives
    y = T.softmax_mask(x, m.to("cuda"), causal=False)
    ref = _ref(x.detach(), m.to("cuda", torch.float32), False)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
    dy = torch.randn(1, 2, 8, S, generator=g).to("cuda", torch.bfloat16)
    (dx,) = torch.autograd.grad(y, x, dy)
    yf = ref
    dref = yf * (dy.float() - (dy.float() * yf).sum(-1, keepdim=True))
    torch.testing.assert_close(dx.float(), dref, rtol=2e-2, atol=2e-2)


def test_softmax_mask_rejects_per_head_mask():
    x = torch.randn(1, 2, 4, 8)
    with pytest.raises(ValueError):
        T.softmax_mask(x, torch.zeros(1, 2, 4, 8))
