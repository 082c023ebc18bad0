"""RoPE^T folded into the flash backward (csrc/kernels/flash_attn.hip: dK epilogue + dq_reduce_rope_kernel) and the
one-node Llama QKV projection + RoPE + attention (_QKVProjRopeAttnFn), against fp32 autograd references of the same
composition (projection -> rotate-half RoPE on q / k -> causal softmax attention)."""
import math

import pytest
import torch

from paddle2_amd.ops import torch_ops as T

pytestmark = pytest.mark.gpu
dev = "cuda"


def _tables(S, D=128):
    c, s = T.rope_tables(S, D, interleaved=False, device=dev)
    return c.reshape(S, D).float().contiguous(), s.reshape(S, D).float().contiguous()


def _rope_ref(x, c, s):   # x [B, S, H, 128] fp32, rotate-half
    x1, x2 = x[..., :64], x[..., 64:]
    cc, ss = c[None, :, None, :64], s[None, :, None, :64]
    return torch.cat([x1 * cc - x2 * ss, x2 * cc + x1 * ss], -1)


def _attn_ref(q, k, v):
    B, S, Hq, D = q.shape
    g = Hq // k.shape[2]
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    kf, vf = kf.repeat_interleave(g, 1), vf.repeat_interleave(g, 1)
    s = (qf @ kf.transpose(-1, -2)) / math.sqrt(D)
    s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    return (torch.softmax(s, -1) @ vf).transpose(1, 2)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("B,S,nh,nkv", [(2, 512, 4, 4), (1, 1000, 8, 2)])
def test_qkv_rope_attention_fold_matches_unfused(monkeypatch, B, S, nh, nkv):
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, S, nh + 2 * nkv, 128, generator=g, device=dev).to(torch.bfloat16)
    do = torch.randn(B, S, nh, 128, generator=g, device=dev).to(torch.bfloat16)
    c, s = _tables(S)
    grads = {}
    for fold in (True, False):
        monkeypatch.setattr(T, "_ROPE_BWD_IN_FLASH", fold)
        x = qkv.clone().requires_grad_()
        o = T._QKVRopeAttnFn.apply(x, nh, nkv, c, s, None, True, 1 / math.sqrt(128))
        o.backward(do)
        grads[fold] = (o.detach(), x.grad)
    assert torch.equal(grads[True][0], grads[False][0])
    assert _rel(grads[True][1], grads[False][1]) < 1e-2
    # fp32 reference of the same composition
    xr = qkv.float().requires_grad_()
    q = _rope_ref(xr[:, :, :nh], c, s)
    k = _rope_ref(xr[:, :, nh:nh + nkv], c, s)
    _attn_ref(q, k, xr[:, :, nh + nkv:]).backward(do.float())
    assert _rel(grads[True][1], xr.grad) < 2e-2


def test_qkv_proj_rope_attention_node(monkeypatch):
    monkeypatch.setattr(T, "_ROPE_IN_GEMM", True)    # opt-in route (profiles/r4_rope_fusion.md)
    B, S, K, nh, nkv = 2, 512, 1024, 8, 8
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(B, S, K, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, (nh + 2 * nkv) * 128, generator=g, device=dev) * K ** -0.5).to(torch.bfloat16)
    do = torch.randn(B, S, nh, 128, generator=g, device=dev).to(torch.bfloat16)
    c, s = _tables(S)
    assert T.qkv_rope_linear_ok(x, w, None, 128, None)
    xi, wi = x.clone().requires_grad_(), w.clone().requires_grad_()
    o = T.qkv_proj_rope_attention(xi, wi, c, s, nh, nkv, S)
    o.backward(do)
    xr, wr = x.float().requires_grad_(), w.float().requires_grad_()
    y = (xr @ wr).view(B, S, nh + 2 * nkv, 128)
    ref = _attn_ref(_rope_ref(y[:, :, :nh], c, s), _rope_ref(y[:, :, nh:nh + nkv], c, s), y[:, :, nh + nkv:])
    ref.backward(do.float())
    assert _rel(o, ref) < 2e-2
    assert _rel(xi.grad, xr.grad) < 3e-2
    wg = wi.grad if wi.grad is not None else getattr(wi, "main_grad", None)
    assert wg is not None and _rel(wg, wr.grad) < 3e-2
