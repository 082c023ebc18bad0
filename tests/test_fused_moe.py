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
    out = fused_moe(P(x), paddle.to_tensor(gw.to(dev)), P(w1), None, P(b1), P(w2), None, P(b2), moe_topk=k)
    ref = _dense_ref(x, gw, w1.to(dt).float(), b1.to(dt).float(), w2.to(dt).float(), b2.to(dt).float(), k)
    tol = 1e-4 if dt == torch.float32 else 5e-2
    torch.testing.assert_close(out._t.float().cpu(), ref, rtol=tol, atol=tol)
