"""paddle.incubate.nn.functional.fused_moe: sort-grouped top-k MoE FFN vs a dense every-token-through-every-
expert reference (reference test: test/legacy_test/test_fused_moe_op.py, whose CUTLASS kernel is NVIDIA-only;
parity against the reference's numbers is unpinned — this checks the op's definition)."""
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.incubate.nn.functional import fused_moe

DEVS = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dense_ref(x, gw, w1, b1, w2, b2, k):
    t = x.reshape(-1, x.shape[-1]).float()
    p = torch.softmax(t @ gw.float(), -1)
    w, idx = torch.topk(p, k, -1)
    w = w / w.sum(-1, keepdim=True)
    out = torch.zeros_like(t)
    for e in range(w1.shape[0]):
        h = t @ w1[e].float() + b1[e].float()
        a, g = h.chunk(2, -1)
        o = (torch.nn.functional.silu(a) * g) @ w2[e].float() + b2[e].float()
        we = (w * (idx == e)).sum(-1, keepdim=True)
        out += we * o
    return out.reshape(x.shape)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("k", [1, 2])
def test_fused_moe_matches_dense(dev, k):
    g = torch.Generator().manual_seed(k)
    B, S, H, F, E = 2, 9, 32, 48, 5
    dt = torch.float32 if dev == "cpu" else torch.bfloat16
    x = torch.randn(B, S, H, generator=g)
    gw = torch.randn(H, E, generator=g)
    w1 = torch.randn(E, H, 2 * F, generator=g) / H ** 0.5
    b1 = torch.randn(E, 2 * F, generator=g) * 0.1
    w2 = torch.randn(E, F, H, generator=g) / F ** 0.5
    b2 = torch.randn(E, H, generator=g) * 0.1
    P = lambda a: paddle.to_tensor(a.to(dev, dt))  # noqa: E731
    # positional call in the reference order (test_fused_moe_op.py:168): x, gate, w1, w2, b1, s1, b2, s2, quant, k, norm
    out = fused_moe(P(x), paddle.to_tensor(gw.to(dev)), P(w1), P(w2), P(b1.reshape(E, 1, 2 * F)), None,
                    P(b2.reshape(E, 1, H)), None, "None", k, True)
    ref = _dense_ref(x, gw, w1.to(dt).float(), b1.to(dt).float(), w2.to(dt).float(), b2.to(dt).float(), k)
    tol = 1e-4 if dt == torch.float32 else 5e-2
    torch.testing.assert_close(out._t.float().cpu(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("algo", ["weight_only_int8", "weight_only_int4"])
def test_fused_moe_weight_only(algo):
    """quant_method: expert weights from nn.quant.weight_quantize (reshaped to the float weight's shape as in
    the reference test) + per-channel scales == the same MoE on the dequantized weights."""
    from paddle2_amd.nn.quant import weight_dequantize, weight_quantize

    g = torch.Generator().manual_seed(7)
    B, S, H, F, E, k = 2, 8, 64, 64, 4, 2
    x = torch.randn(B, S, H, generator=g)
    gw = torch.randn(H, E, generator=g)
    w1 = torch.randn(E, H, 2 * F, generator=g) / H ** 0.5
    w2 = torch.randn(E, F, H, generator=g) / F ** 0.5
    q1, s1, q2, s2, d1, d2 = [], [], [], [], [], []
    for e in range(E):
        qa, sa = weight_quantize(paddle.to_tensor(w1[e]), algo=algo)
        qb, sb = weight_quantize(paddle.to_tensor(w2[e]), algo=algo)
        d1.append(weight_dequantize(qa, sa, algo=algo, out_dtype="float32")._t)
        d2.append(weight_dequantize(qb, sb, algo=algo, out_dtype="float32")._t)
        q1.append(qa._t.reshape(H, -1))
        q2.append(qb._t.reshape(F, -1))
        s1.append(sa._t)
        s2.append(sb._t)
    P = paddle.to_tensor
    out = fused_moe(P(x), P(gw), P(torch.stack(q1)), P(torch.stack(q2)), None, P(torch.stack(s1)), None,
                    P(torch.stack(s2)), algo, k, True)
    ref = fused_moe(P(x), P(gw), P(torch.stack(d1)), P(torch.stack(d2)), None, None, None, None, "None", k, True)
    torch.testing.assert_close(out._t, ref._t, rtol=1e-4, atol=1e-4)
    with pytest.raises(ValueError):
        fused_moe(P(x), P(gw), P(torch.stack(q1)), P(torch.stack(q2)), None, None, None, None, algo, k, True)


def _ragged_goff(counts, dev):
    g = torch.zeros(len(counts) + 1, dtype=torch.int32)
    g[1:] = torch.tensor(counts).cumsum(0)
    return g.to(dev)


@pytest.mark.parametrize("dev", DEVS)
def test_grouped_linear_and_swiglu_autograd(dev):
    """ops.moe grouped ops (one launch per projection on the MI355X) vs per-expert fp32 math, ragged groups
    including empty experts; forward and all three gradients."""
    from paddle2_amd.ops import moe as MOE

    counts = [0, 300, 17, 260, 0, 5, 91, 256] if dev == "cuda" else [0, 7, 3, 0, 5]
    E, K, N = len(counts), 64, 128
    Tn = sum(counts)
    g = torch.Generator().manual_seed(3)
    dt = torch.bfloat16 if dev == "cuda" else torch.float32
    xs0 = torch.randn(Tn, K, generator=g)
    w0 = torch.randn(E, K, N, generator=g) / K ** 0.5
    goff = _ragged_goff(counts, dev)
    xs = xs0.to(dev, dt).requires_grad_()
    w = w0.to(dev, dt).requires_grad_()
    y = MOE.grouped_linear(xs, w, goff)
    a = MOE.grouped_swiglu(xs, w, goff)
    dy = torch.randn(Tn, N, generator=g)
    da = torch.randn(Tn, N // 2, generator=g)
    (y.float() * dy.to(dev)).sum().add((a.float() * da.to(dev)).sum()).backward()
    # fp32 reference on the rounded operands
    xr = xs0.to(dt).float().requires_grad_()
    wr = w0.to(dt).float().requires_grad_()
    o = goff.cpu().tolist()
    yr = torch.cat([xr[o[e]:o[e + 1]] @ wr[e] for e in range(E)])
    gu = torch.cat([xr[o[e]:o[e + 1]] @ wr[e] for e in range(E)])
    ar = torch.nn.functional.silu(gu[:, :N // 2]) * gu[:, N // 2:]
    ((yr * dy).sum() + (ar * da).sum()).backward()
    tol = 1e-4 if dt == torch.float32 else 3e-2
    for got, ref in ((y, yr), (a, ar), (xs.grad, xr.grad), (w.grad, wr.grad)):
        err = (got.float().cpu() - ref.detach()).abs().max() / ref.detach().abs().max()
        assert err < tol, err
    assert torch.count_nonzero(w.grad[0]) == 0 and torch.count_nonzero(w.grad[4 if dev == "cuda" else 3]) == 0


def test_route_topk_offsets():
    from paddle2_amd.ops import moe as MOE

    logits = torch.randn(10, 4)
    tok, gate, goff = MOE.route_topk(logits, 2)
    assert goff[-1] == 20 and tok.shape == (20,) and torch.all(goff[1:] >= goff[:-1])
    _, idx = torch.topk(torch.softmax(logits, -1), 2, -1)
    for e in range(4):
        assert sorted(tok[goff[e]:goff[e + 1]].tolist()) == sorted((idx == e).nonzero()[:, 0].tolist())
