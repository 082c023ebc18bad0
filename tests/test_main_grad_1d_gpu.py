"""1-D parameter gradients (linear / fp8-linear biases, RMSNorm / LayerNorm weights and biases) written by their
column-sum kernels straight into the sharding unit's fp32 main-grad slot (``_p2_bt``, ops.torch_ops.main_slot):
the slot gets beta * slot + the fp32 column sum, the unit is told (param_grad_done) and autograd gets no gradient.
Compared against the fp32 PyTorch sums of the same op (reference: the main_grad path of
python/paddle/distributed/fleet/meta_parallel/sharding/group_sharded_stage3.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _Unit:
    def __init__(self, n_params, n, beta):
        self.bufs = [torch.full((n,), 0.5, device=DEV, dtype=torch.float32) for _ in range(n_params)]
        self.beta = beta
        self.done = []

    def grad_target(self, i):
        return self.bufs[i], self.beta

    def param_grad_done(self, i):
        self.done.append(i)


@pytest.mark.parametrize("beta", [0, 1])
def test_linear_bias_into_main_slot(beta):
    from paddle2_amd.ops import torch_ops as T

    torch.manual_seed(0)
    M, K, Nn = 300, 256, 384
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(K, Nn, device=DEV) * 0.05).bfloat16().requires_grad_()
    b = torch.zeros(Nn, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    u = _Unit(1, Nn, beta)
    b._p2_bt = (u, 0)
    g = torch.randn(M, Nn, device=DEV, dtype=torch.bfloat16)
    T.linear(x, w, b).backward(g)
    assert b.grad is None and u.done == [0]
    ref = g.float().sum(0) + (0.5 if beta else 0.0)
    torch.testing.assert_close(u.bufs[0], ref, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("layernorm", [False, True])
@pytest.mark.parametrize("beta", [0, 1])
def test_norm_weights_into_main_slot(layernorm, beta):
    from paddle2_amd.ops import torch_ops as T

    torch.manual_seed(1)
    M, Nn = 1500, 512
    x = torch.randn(M, Nn, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(Nn, device=DEV)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(Nn, device=DEV)).bfloat16().requires_grad_() if layernorm else None
    u = _Unit(2, Nn, beta)
    w._p2_bt = (u, 0)
    if b is not None:
        b._p2_bt = (u, 1)
    g = torch.randn(M, Nn, device=DEV, dtype=torch.bfloat16)
    y = T.layer_norm(x, w, b) if layernorm else T.rms_norm(x, w)
    y.backward(g)
    assert w.grad is None and sorted(u.done) == ([0, 1] if layernorm else [0])
    xf = x.detach().float()
    if layernorm:
        xh = (xf - xf.mean(-1, keepdim=True)) * torch.rsqrt(xf.var(-1, unbiased=False, keepdim=True) + 1e-5)
    else:
        xh = xf * torch.rsqrt(xf.square().mean(-1, keepdim=True) + 1e-6)
    add = 0.5 if beta else 0.0
    torch.testing.assert_close(u.bufs[0], (g.float() * xh).sum(0) + add, rtol=1e-4, atol=2e-2)
    if layernorm:
        assert b.grad is None
        torch.testing.assert_close(u.bufs[1], g.float().sum(0) + add, rtol=1e-5, atol=1e-3)
    assert x.grad is not None and torch.isfinite(x.grad.float()).all()


def test_norm_partial_slots_fall_back():
    """LayerNorm whose bias has no slot: both gradients take the autograd path (one output dtype per launch)."""
    from paddle2_amd.ops import torch_ops as T

    M, Nn = 256, 512
    x = torch.randn(M, Nn, device=DEV, dtype=torch.bfloat16)
    w = torch.ones(Nn, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = torch.zeros(Nn, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    u = _Unit(1, Nn, 0)
    w._p2_bt = (u, 0)
    T.layer_norm(x, w, b).sum().backward()
    assert u.done == [] and w.grad is not None and b.grad is not None


def test_fp8_linear_bias_into_main_slot():
    from paddle2_amd.ops import fp8

    torch.manual_seed(2)
    M, K, Nn = 320, 256, 512
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(K, Nn, device=DEV) * 0.05).bfloat16().requires_grad_()
    b = torch.zeros(Nn, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    u = _Unit(1, Nn, 1)
    b._p2_bt = (u, 0)
    metas = [fp8.FP8TensorMeta(f, device=torch.device(DEV)) for f in (fp8.E4M3, fp8.E4M3, fp8.E5M2)]
    g = torch.randn(M, Nn, device=DEV, dtype=torch.bfloat16)
    fp8.fp8_linear(x, w, b, *metas).backward(g)
    fp8.flush_updates()
    assert b.grad is None and u.done == [0]
    torch.testing.assert_close(u.bufs[0], g.float().sum(0) + 0.5, rtol=1e-5, atol=1e-3)
