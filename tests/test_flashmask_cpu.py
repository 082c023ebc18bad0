"""FlashMask semantics on CPU: the interval normalisation used by the kernel reproduces the reference's
flashmask_to_densemask construction (python/paddle/nn/functional/flash_attention.py docstring of
flashmask_attention), and the varlen fallback matches per-sequence attention."""
import pytest
import torch

from paddle2_amd.ops import torch_ops as T


def _densemask(idx, causal):
    """Direct transcription of the documented dense-mask rule (True = masked)."""
    B, H, S, n = idx.shape
    m = torch.zeros(B, H, S, S, dtype=torch.bool)
    has_end = (causal and n == 2) or ((not causal) and n == 4)
    for b in range(B):
        for h in range(H):
            for j in range(S):
                ds = int(idx[b, h, j, 0])
                if has_end:
                    m[b, h, ds:int(idx[b, h, j, 1]), j] = True
                else:
                    m[b, h, ds:, j] = True
                if causal:
                    m[b, h, :j, j] = True
                elif has_end:
                    m[b, h, int(idx[b, h, j, 2]):int(idx[b, h, j, 3]), j] = True
                else:
                    m[b, h, :int(idx[b, h, j, 1]), j] = True
    return m


@pytest.mark.parametrize("causal,n", [(True, 1), (True, 2), (False, 2), (False, 4)])
def test_flashmask_matches_dense_rule(causal, n):
    torch.manual_seed(n)
    B, H, S, D = 1, 2, 24, 16
    idx = torch.sort(torch.randint(0, S + 1, (B, H, S, n)), -1).values.int()
    if not causal and n == 2:
        idx = torch.stack([idx[..., 1], idx[..., 0]], -1)  # LTS (lower start) above UTE
    q, k, v = torch.randn(B, S, H, D), torch.randn(B, S, H, D), torch.randn(B, S, H, D)
    out, _ = T.flash_attention_mask(q, k, v, idx, causal)
    dense = _densemask(idx, causal)
    bias = torch.zeros(B, H, S, S).masked_fill(dense, float("-inf"))
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * D ** -0.5 + bias
    p = torch.nan_to_num(torch.softmax(s, -1), nan=0.0)
    ref = torch.einsum("bhqk,bkhd->bqhd", p, v)
    assert torch.allclose(out, ref, atol=1e-5)


def test_varlen_fallback_matches_per_sequence():
    torch.manual_seed(0)
    lens = [5, 17, 9]
    cu = torch.tensor([0, 5, 22, 31], dtype=torch.int32)
    q, k, v = torch.randn(31, 4, 16), torch.randn(31, 2, 16), torch.randn(31, 2, 16)
    out, lse = T.flash_attention_varlen(q, k, v, cu, cu, max(lens), max(lens), causal=True)
    assert lse.shape == (4, 31)
    for i in range(3):
        a, b = int(cu[i]), int(cu[i + 1])
        o, _ = T._attn_reference(q[a:b][None], k[a:b][None], v[a:b][None], True, 16 ** -0.5)
        assert torch.allclose(out[a:b], o[0], atol=1e-5)
