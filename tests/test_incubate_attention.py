"""paddle.incubate.nn.functional attention entry points: variable_length_memory_efficient_attention (one
FlashMask launch over the padded batch) and masked_multihead_attention (flash-decoding kernel) vs per-sequence
fp32 definitions (reference tests: test_variable_length_memory_efficient_attention.py,
test_masked_multihead_attention_op.py; their CUTLASS/CUDA kernels are NVIDIA-only, so parity is against the
op definition)."""
import math

import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.incubate.nn import functional as IF

DEVS = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _ref_varlen(q, k, v, sl, kl, causal, scale, mask=None):
    b, h, sq, d = q.shape
    out = torch.zeros(b, h, sq, d)
    for i in range(b):
        qs, ks, vs = q[i, :, :sl[i]].float(), k[i, :, :kl[i]].float(), v[i, :, :kl[i]].float()
        s = qs @ ks.transpose(-1, -2) * scale
        if mask is not None:
            s = s + mask[i, :, :sl[i], :kl[i]].float()
        if causal:
            r = torch.arange(sl[i])[:, None]
            c = torch.arange(kl[i])[None, :]
            s = s.masked_fill(c > r + (kl[i] - sl[i]), float("-inf"))
        out[i, :, :sl[i]] = torch.softmax(s, -1) @ vs
    return out


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("with_mask", [False, True])
def test_varlen_mem_efficient_attention(dev, causal, with_mask):
    g = torch.Generator().manual_seed(1)
    b, h, s, d = 3, 2, 80, 64
    dt = torch.bfloat16 if dev == "cuda" else torch.float32
    q, k, v = (torch.randn(b, h, s, d, generator=g).to(dt) for _ in range(3))
    sl, kl = [80, 33, 57], [80, 50, 57]
    mask = torch.randn(b, 1, s, s, generator=g) if with_mask else None
    P = lambda a: paddle.to_tensor(a.to(dev))  # noqa: E731
    out = IF.variable_length_memory_efficient_attention(
        P(q), P(k), P(v), P(torch.tensor(sl, dtype=torch.int32)), P(torch.tensor(kl, dtype=torch.int32)),
        mask=None if mask is None else P(mask), scale=1 / math.sqrt(d), causal=causal)
    ref = _ref_varlen(q, k, v, sl, kl, causal, 1 / math.sqrt(d), mask)
    tol = 1e-4 if dt == torch.float32 else 3e-2
    torch.testing.assert_close(out._t.float().cpu(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("dev", DEVS)
def test_incubate_mmha_uses_serving_kernel(dev):
    g = torch.Generator().manual_seed(2)
    b, nh, hd, max_s = 2, 4, 128, 64
    dt = torch.bfloat16 if dev == "cuda" else torch.float32
    cache = torch.randn(2, b, nh, max_s, hd, generator=g).to(dev, dt)
    x = torch.randn(b, 3 * nh * hd, generator=g).to(dev, dt)
    lens = torch.tensor([5, 17], dtype=torch.int32)
    c_ref = cache.float().cpu().clone()
    out, cache_out = IF.masked_multihead_attention(paddle.to_tensor(x), paddle.to_tensor(cache),
                                           sequence_lengths=paddle.to_tensor(lens.to(dev)))
    qkv = x.float().cpu().reshape(b, 3, nh, hd)
    for i in range(b):
        c_ref[0, i, :, lens[i]] = qkv[i, 1]
        c_ref[1, i, :, lens[i]] = qkv[i, 2]
        kk, vv = c_ref[0, i, :, :lens[i] + 1], c_ref[1, i, :, :lens[i] + 1]
        p = torch.softmax((qkv[i, 0][:, None, :] * kk).sum(-1) / math.sqrt(hd), -1)
        o = (p[..., None] * vv).sum(1)
        tol = 1e-4 if dt == torch.float32 else 3e-2
        torch.testing.assert_close(out._t.float().cpu().reshape(b, nh, hd)[i], o, rtol=tol, atol=tol)
    torch.testing.assert_close(cache_out._t.float().cpu(), c_ref, rtol=1e-2, atol=1e-2)
