"""Attention dropout contract on CPU: counter-hash keep mask (host emulation of the kernel's drop_keep),
seed/offset determinism and the Paddle-level API (reference flash_attention.py `dropout`, `fixed_seed_offset`).
The GPU kernel is checked against the same host mask in tests/test_flash_ext_gpu.py."""
import torch

import paddle2_amd as paddle
from paddle2_amd.ops import torch_ops as T


def _hash_scalar(seed, bh, q, k):
    """Plain-int transcription of drop_keep's hash (uint32 arithmetic)."""
    m = 0xFFFFFFFF
    x = seed ^ ((bh * 0x27D4EB2D) & m)
    x = (x + q * 0x9E3779B1) & m
    x ^= x >> 15
    x = (x * 0x85EBCA77) & m
    x = (x + k * 0xC2B2AE3D) & m
    x ^= x >> 13
    x = (x * 0x27D4EB2F) & m
    x ^= x >> 16
    return x


def test_mask_matches_scalar_hash():
    seed, p = 0xDEADBEEF, 0.37
    keep = T.attn_dropout_mask(seed, 2, 3, 5, 7, p)
    th = T.attn_dropout_threshold(p)
    for b, h, q, k in [(0, 0, 0, 0), (1, 2, 4, 6), (1, 0, 3, 1), (0, 2, 2, 5)]:
        assert bool(keep[b, h, q, k]) == (_hash_scalar(seed, b * 3 + h, q, k) >= th)


def test_mask_rate_and_seed_dependence():
    p = 0.1
    a = T.attn_dropout_mask(1, 2, 4, 128, 128, p)
    b = T.attn_dropout_mask(2, 2, 4, 128, 128, p)
    assert abs(1 - a.float().mean().item() - p) < 0.01
    assert (a != b).float().mean().item() > 0.1
    assert torch.equal(a, T.attn_dropout_mask(1, 2, 4, 128, 128, p))
    # large indices stay exact (no int64 overflow in the emulation)
    big = T.attn_dropout_keep(7, torch.tensor([2 ** 20]), torch.tensor([2 ** 31 - 1]), torch.tensor([2 ** 31 - 5]), p)
    assert bool(big[0]) == (_hash_scalar(7, 2 ** 20, 2 ** 31 - 1, 2 ** 31 - 5) >= T.attn_dropout_threshold(p))


def test_threshold_clamps():
    assert T.attn_dropout_threshold(0.5) == 2 ** 31
    assert T.attn_dropout_threshold(0.9999999999) == 4294967040


def test_paddle_flash_attention_dropout_api():
    paddle.seed(5)
    g = torch.Generator().manual_seed(0)
    q, k, v = (paddle.Tensor._wrap(torch.randn(2, 16, 2, 8, generator=g).requires_grad_(True)) for _ in range(3))
    F = paddle.nn.functional
    fso = torch.tensor([3, 0])
    o1, _ = F.flash_attention(q, k, v, dropout=0.25, causal=True, fixed_seed_offset=fso)
    o2, _ = F.flash_attention(q, k, v, dropout=0.25, causal=True, fixed_seed_offset=fso)
    assert torch.equal(o1._t, o2._t)
    o3, _ = F.flash_attention(q, k, v, dropout=0.25, causal=True)
    o4, _ = F.flash_attention(q, k, v, dropout=0.25, causal=True)
    assert not torch.equal(o3._t, o4._t)  # the (seed, offset) counter advances between calls
    o0, _ = F.flash_attention(q, k, v, dropout=0.25, causal=True, training=False)
    ref, _ = T._attn_reference(q._t, k._t, v._t, True, 8 ** -0.5)
    assert torch.allclose(o0._t.float(), ref, atol=1e-5)
    o1._t.sum().backward()
    assert q._t.grad is not None and torch.isfinite(q._t.grad).all()
    # expectation over masks ~ undropped output
    acc = torch.zeros_like(ref)
    for s in range(200):
        o, _ = T.flash_attention_dropout(q._t.detach(), k._t.detach(), v._t.detach(), 0.25, True, seed32=s)
        acc += o.float()
    assert (acc / 200 - ref).abs().mean().item() < 0.05


def test_varlen_dropout_cpu_matches_dense_per_sequence():
    """Sequence i of a varlen batch uses batch*head index i * H + h, like the kernel's kVarlen mode."""
    H, D, p, seed = 2, 8, 0.3, 1234
    lens = [5, 9]
    cu = torch.tensor([0, 5, 14], dtype=torch.int32)
    g = torch.Generator().manual_seed(1)
    q, k, v = (torch.randn(14, H, D, generator=g) for _ in range(3))
    o, _ = T.flash_attention_varlen(q, k, v, cu, cu, 9, 9, False, dropout=p, seed32=seed)
    keep = T.attn_dropout_mask(seed, 2, H, 9, 9, p)  # dense [B=2, H, 9, 9]
    for i, (a, n) in enumerate([(0, 5), (5, 9)]):
        oi, _ = T._attn_reference_dropout(q[a:a + n][None], k[a:a + n][None], v[a:a + n][None], False, D ** -0.5,
                                          keep[i:i + 1, :, :n, :n], p)
        assert torch.allclose(o[a:a + n], oi[0], atol=1e-5)
