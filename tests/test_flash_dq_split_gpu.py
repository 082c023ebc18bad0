"""Split dQ (csrc/kernels/flash_attn.hip dq_gemm_kernel, the dense D = 128 default): the backward stores dS per
(query tile, key block) into a compact bf16 buffer and a second kernel computes dQ = scale * dS . K with RoPE^T
fused.  Checked against an fp32 reference (causal / full, Sq != Sk, ragged lengths, GQA, fp16, RoPE^T) and against
the fused atomic path; dQ must be bit-reproducible (no atomics)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def split_env():
    old = os.environ.get("PADDLE2_AMD_FA_DQ_SPLIT")
    yield
    if old is None:
        os.environ.pop("PADDLE2_AMD_FA_DQ_SPLIT", None)
    else:
        os.environ["PADDLE2_AMD_FA_DQ_SPLIT"] = old


def _ref(q, k, v, do, causal, scale):
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    qf, kf, vf, dof = (t.float().transpose(1, 2).detach().requires_grad_(True) for t in (q, k, v, do))
    kr, vr = kf.repeat_interleave(Hq // Hk, 1), vf.repeat_interleave(Hq // Hk, 1)
    s = qf @ kr.transpose(-1, -2) * scale
    if causal:
        i = torch.arange(Sq, device=s.device)[:, None]
        j = torch.arange(Sk, device=s.device)[None, :]
        s = s.masked_fill(j > i + (Sk - Sq), float("-inf"))
    p = torch.nan_to_num(torch.softmax(s, -1), nan=0.0)
    o = p @ vr
    (o * dof).sum().backward()
    return [t.grad.transpose(1, 2) for t in (qf, kf, vf)]


@pytest.mark.parametrize("B,Sq,Sk,Hq,Hk,causal,dt", [
    (2, 1024, 1024, 4, 4, True, torch.bfloat16),
    (2, 1024, 1024, 4, 4, False, torch.bfloat16),
    (1, 777, 1291, 4, 2, True, torch.bfloat16),     # ragged, bottom-right causal offset, GQA
    (1, 1291, 777, 4, 4, True, torch.bfloat16),     # more queries than keys: rows that see no key
    (2, 300, 300, 8, 2, False, torch.float16),
])
def test_split_dq_matches_reference(split_env, B, Sq, Sk, Hq, Hk, causal, dt):
    from paddle2_amd.ops import _native
    from paddle2_amd.ops import torch_ops as T

    _native.require()
    D = 128
    g = torch.Generator(device="cpu").manual_seed(11)
    q, do = (torch.randn(B, Sq, Hq, D, generator=g).to(dt).cuda() for _ in range(2))
    k, v = (torch.randn(B, Sk, Hk, D, generator=g).to(dt).cuda() for _ in range(2))
    scale = D ** -0.5
    out, lse = T._flash_fwd_native(q, k, v, causal, scale)
    os.environ["PADDLE2_AMD_FA_DQ_SPLIT"] = "1"
    assert _native.native().flash_ds_elems(B, Sq, Sk, Hq, D, int(causal)) > 0
    grads = []
    for _ in range(2):
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        T._flash_bwd_native(q, k, v, out, do, lse, dq, dk, dv, scale, causal)
        torch.cuda.synchronize()
        grads.append((dq, dk, dv))
    assert torch.equal(grads[0][0], grads[1][0])   # no atomics: bitwise reproducible dQ
    ref = _ref(q, k, v, do, causal, scale)
    for got, r, name in zip(grads[0], ref, ("dq", "dk", "dv")):
        err = (got.float() - r).abs().max() / r.abs().max().clamp_min(1e-6)
        assert err < 2e-2, (name, err.item())
    os.environ["PADDLE2_AMD_FA_DQ_SPLIT"] = "0"
    dq0 = torch.empty_like(q)
    T._flash_bwd_native(q, k, v, out, do, lse, dq0, torch.empty_like(k), torch.empty_like(v), scale, causal)
    d = (dq0.float() - grads[0][0].float()).abs().max() / ref[0].abs().max()
    assert d < 1e-2, d.item()


def test_split_dq_rope_fold_matches_fused(split_env):
    """RoPE^T of dQ in the dq_gemm epilogue == the fused path's RoPE^T in its reduce pass."""
    from paddle2_amd.ops import _native
    from paddle2_amd.ops import torch_ops as T

    _native.require()
    B, S, H, D = 2, 1024, 4, 128
    g = torch.Generator(device="cpu").manual_seed(5)
    q, k, v, do = (torch.randn(B, S, H, D, generator=g).to(torch.bfloat16).cuda() for _ in range(4))
    pos = torch.arange(S, dtype=torch.float32)[:, None]
    inv = 1.0 / (10000 ** (torch.arange(0, 64, dtype=torch.float32) / 64))
    ang = torch.cat([pos * inv, pos * inv], -1)
    cos, sin = ang.cos().cuda().contiguous(), ang.sin().cuda().contiguous()
    scale = D ** -0.5
    out, lse = T._flash_fwd_native(q, k, v, True, scale)
    res = {}
    for mode in ("1", "0"):
        os.environ["PADDLE2_AMD_FA_DQ_SPLIT"] = mode
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        T._flash_bwd_native(q, k, v, out, do, lse, dq, dk, dv, scale, True, rope=(cos, sin))
        torch.cuda.synchronize()
        res[mode] = (dq, dk, dv)
    for a, b_, name in zip(res["1"], res["0"], ("dq", "dk", "dv")):
        d = (a.float() - b_.float()).abs().max() / b_.float().abs().max()
        assert d < 1e-2, (name, d.item())
