"""_C_ops op table: Paddle positional signatures vs fp32 PyTorch references; AsyncLoad offload/reload."""
import numpy as np
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd import _C_ops


def _r(*shape, dtype=torch.float32, dev="cpu", seed=0):
    g = torch.Generator().manual_seed(seed)
    return paddle.Tensor._wrap(torch.randn(*shape, generator=g).to(dev, dtype))


def test_registry_lists_and_info():
    ops = _C_ops.list_ops()
    for n in ("rms_norm", "flash_attn", "swiglu", "adamw_", "fused_rotary_position_embedding", "c_embedding"):
        assert n in ops
    info = _C_ops.kernel_info("flash_attn")
    assert info["native_kernel"] == "flash_fwd"
    with pytest.raises(AttributeError):
        _C_ops.definitely_not_an_op
    from paddle2_amd.ops.registry import select

    with pytest.raises(NotImplementedError):
        select("definitely_not_an_op")


def test_fallback_to_public_api():
    x = _r(4, 5)
    np.testing.assert_allclose(_C_ops.relu(x).numpy(), np.maximum(x.numpy(), 0))
    assert "relu" in _C_ops.list_ops()


def _check_core(dev, dtype, tol):
    x, w = _r(6, 64, dev=dev, dtype=dtype, seed=1), _r(64, dev=dev, dtype=dtype, seed=2)
    out, res, inv = _C_ops.rms_norm(x, None, None, w, None, 1e-6, 1)
    xf, wf = x._t.float(), w._t.float()
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6) * wf
    torch.testing.assert_close(out._t.float(), ref, atol=tol, rtol=tol)
    assert res is None and inv.shape == [6]
    a, b = _r(8, 96, dev=dev, dtype=dtype, seed=3), _r(8, 96, dev=dev, dtype=dtype, seed=4)
    torch.testing.assert_close(_C_ops.swiglu(a, b)._t.float(),
                               torch.nn.functional.silu(a._t.float()) * b._t.float(), atol=tol, rtol=tol)
    q, k, v = (_r(2, 128, 4, 64, dev=dev, dtype=dtype, seed=s) for s in (5, 6, 7))
    o, _, _, _ = _C_ops.flash_attn(q, k, v, None, None, 0.0, True, False, False, "")
    ref = torch.nn.functional.scaled_dot_product_attention(
        *(t._t.float().transpose(1, 2) for t in (q, k, v)), is_causal=True).transpose(1, 2)
    torch.testing.assert_close(o._t.float(), ref, atol=5 * tol, rtol=5 * tol)
    wt, ids = _r(10, 8, dev=dev, dtype=dtype, seed=8), paddle.Tensor._wrap(torch.tensor([[0, 5, 12, 19]], device=dev))
    ce = _C_ops.c_embedding(wt, ids, 10, -1)._t.float()
    assert float(ce[0, 0].abs().sum()) == 0 and float(ce[0, 1].abs().sum()) == 0
    torch.testing.assert_close(ce[0, 2], wt._t.float()[2])


def test_core_ops_cpu():
    _check_core("cpu", torch.float32, 1e-4)


@pytest.mark.gpu
def test_core_ops_gpu_native():
    from paddle2_amd.ops import _native

    _native.require()
    _check_core("cuda", torch.bfloat16, 2e-2)
    assert _C_ops.kernel_info("rms_norm")["native_loaded"]


def test_adamw_matches_optimizer_formula():
    p = paddle.Tensor._wrap(torch.randn(16))
    g = paddle.Tensor._wrap(torch.randn(16))
    m, v = paddle.Tensor._wrap(torch.zeros(16)), paddle.Tensor._wrap(torch.zeros(16))
    b1p, b2p = paddle.Tensor._wrap(torch.tensor([0.9])), paddle.Tensor._wrap(torch.tensor([0.999]))
    p0 = p._t.clone()
    _C_ops.adamw_(p, g, 0.1, m, v, b1p, b2p, None, None, 0.9, 0.999, 1e-8, 1.0, 0.01, True)
    gt = g._t
    mh, vh = 0.1 * gt / 0.1, 0.001 * gt * gt / 0.001
    ref = p0 * (1 - 0.1 * 0.01) - 0.1 * mh / (vh.sqrt() + 1e-8)
    torch.testing.assert_close(p._t, ref, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(b1p._t, torch.tensor([0.81]))


def test_loss_scaling_ops():
    xs = [paddle.Tensor._wrap(torch.tensor([2.0, 4.0])), paddle.Tensor._wrap(torch.tensor([float("inf")]))]
    _, found = _C_ops.check_finite_and_unscale_(xs, paddle.Tensor._wrap(torch.tensor([2.0])))
    assert bool(found._t[0])
    np.testing.assert_allclose(xs[0].numpy(), [1.0, 2.0])
    s, good, bad = (paddle.Tensor._wrap(torch.tensor([v])) for v in (1024.0, 0.0, 0.0))
    _C_ops.update_loss_scaling_(xs, found, s, good, bad, 1000, 1, 2.0, 0.5)
    assert float(s._t) == 512.0 and float(xs[0]._t.abs().sum()) == 0


def _roundtrip(dev):
    from paddle2_amd.incubate.tensor import async_offload, async_reload, create_async_load

    al = create_async_load()
    x = paddle.Tensor._wrap(torch.arange(1 << 16, dtype=torch.float32, device=dev))
    h, t = async_offload(x, al)
    t.cpu_wait()
    assert h._t.device.type == "cpu" and t.is_completed()
    d, t2 = async_reload(h, al)
    t2.cuda_wait() if dev == "cuda" else t2.wait()
    torch.testing.assert_close(d._t.cpu(), x._t.cpu())


def test_async_load_cpu():
    _roundtrip("cpu")


@pytest.mark.gpu
def test_async_load_gpu():
    _roundtrip("cuda")
