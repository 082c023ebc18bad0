"""Fused bias+activation and dropout+add (csrc/kernels/fused_act.hip, ops/fused.py) vs fp32 PyTorch
definitions; the dropout mask is a counter hash shared bit-for-bit by the kernel and the host model
(reference: fused_bias_act_kernel.cu, fused_dropout_add_kernel.cu; test_fused_bias_act_op.py)."""
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.incubate.nn import functional as IF
from paddle2_amd.ops import fused as FU

DEVS = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _ref_act(name, t):
    F = torch.nn.functional
    H = t.shape[-1] // 2
    return {"gelu": F.gelu, "gelu_tanh": lambda v: F.gelu(v, approximate="tanh"), "relu": torch.relu, "silu": F.silu, "identity": lambda v: v,
            "swiglu": lambda v: F.silu(v[..., :H]) * v[..., H:],
            "geglu": lambda v: F.gelu(v[..., :H]) * v[..., H:]}[name](t)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("act", ["gelu", "gelu_tanh", "relu", "silu", "identity", "swiglu", "geglu"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bias_act_fwd_bwd(dev, act, dtype):
    g = torch.Generator().manual_seed(0)
    x0, b0 = torch.randn(37, 64, generator=g), torch.randn(64, generator=g)
    dy0 = torch.randn(37, 32 if act in ("swiglu", "geglu") else 64, generator=g)
    x = x0.to(dev, dtype).requires_grad_()
    b = b0.to(dev, dtype).requires_grad_()
    y = FU.bias_act(x, b, act)
    y.backward(dy0.to(dev, dtype))
    xr = x0.to(dtype).float().requires_grad_()
    br = b0.to(dtype).float().requires_grad_()
    yr = _ref_act(act, xr + br)
    yr.backward(dy0.to(dtype).float())
    tol = 1e-5 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=tol, atol=tol)
    torch.testing.assert_close(x.grad.float().cpu(), xr.grad, rtol=tol, atol=tol)
    torch.testing.assert_close(b.grad.float().cpu(), br.grad, rtol=tol, atol=max(tol, 0.3 if dtype != torch.float32 else 0))


@pytest.mark.parametrize("dev", DEVS)
def test_dropout_add_mask_and_grads(dev):
    n, p, seed = 4096, 0.3, 12345
    x = torch.randn(16, 256, device=dev).requires_grad_()
    y = torch.randn(16, 256, device=dev).requires_grad_()
    out = FU.dropout_add(x, y, p, seed)
    keep = FU.dropout_keep(seed, n, p).reshape(16, 256).to(dev)
    torch.testing.assert_close(out, x.detach() * keep / (1 - p) + y.detach())
    assert abs(keep.float().mean().item() - (1 - p)) < 0.03
    out.sum().backward()
    torch.testing.assert_close(x.grad, keep.float() / (1 - p))
    torch.testing.assert_close(y.grad, torch.ones_like(y))


def test_incubate_entry_points():
    x = paddle.randn([4, 16])
    b = paddle.randn([16])
    out = IF.fused_bias_act(x, b, act_method="swiglu")
    assert out.shape == [4, 8]
    r = IF.fused_dropout_add(paddle.ones([4, 8]), paddle.zeros([4, 8]), p=0.5, training=True)
    vals = set(r._t.unique().tolist())
    assert vals <= {0.0, 2.0}
    assert IF.fused_dropout_add(paddle.ones([2, 8]), paddle.ones([2, 8]), p=0.5, training=False)._t.eq(2).all()


@pytest.mark.gpu
@pytest.mark.parametrize("approximate", [False, True])
def test_functional_gelu_native_on_gpu(approximate):
    """paddle.nn.functional.gelu on a bf16 GPU tensor runs the native kernel: forward and grad vs fp32."""
    g = torch.Generator().manual_seed(1)
    x0 = torch.randn(64, 256, generator=g)
    x = paddle.to_tensor(x0.to("cuda", torch.bfloat16))
    x.stop_gradient = False
    y = paddle.nn.functional.gelu(x, approximate=approximate)
    assert y._t.grad_fn is not None and "BiasAct" in type(y._t.grad_fn).__name__
    y.sum().backward()
    xr = x0.to(torch.bfloat16).float().requires_grad_()
    yr = torch.nn.functional.gelu(xr, approximate="tanh" if approximate else "none")
    yr.sum().backward()
    torch.testing.assert_close(y._t.float().cpu(), yr.detach(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x.grad._t.float().cpu(), xr.grad, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("act", ["gelu", "gelu_tanh", "silu", "swiglu"])
def test_bias_act_double_backward(dev, act):
    """create_graph through the fused bias-act: the second-order terms (d/dx of the input gradient) match torch's
    own double backward of the same function in fp32 (bf16 inputs on the GPU)."""
    from paddle2_amd.ops import fused as Fz

    dt = torch.bfloat16 if dev == "cuda" else torch.float32
    g = torch.Generator().manual_seed(3)
    W = 64
    x0 = torch.randn(16, W, generator=g).to(dt)
    b0 = torch.randn(W, generator=g).to(dt)
    x = x0.to(dev).requires_grad_(True)
    b = b0.to(dev).requires_grad_(True)
    y = Fz.bias_act(x, b, act)
    (gx,) = torch.autograd.grad(y.float().pow(2).sum(), x, create_graph=True)
    (hx,) = torch.autograd.grad(gx.float().sum(), x)
    xr = x0.float().requires_grad_(True)
    t = xr + b0.float()
    F = torch.nn.functional
    if act == "swiglu":
        yr = F.silu(t[:, :W // 2]) * t[:, W // 2:]
    else:
        yr = {"gelu": F.gelu, "gelu_tanh": lambda v: F.gelu(v, approximate="tanh"), "silu": F.silu}[act](t)
    (gr,) = torch.autograd.grad(yr.pow(2).sum(), xr, create_graph=True)
    (hr,) = torch.autograd.grad(gr.sum(), xr)
    tol = 8e-2 if dt == torch.bfloat16 else 1e-4
    assert hx.abs().sum() > 0
    torch.testing.assert_close(hx.float().cpu(), hr, rtol=tol, atol=tol * hr.abs().max().item())
