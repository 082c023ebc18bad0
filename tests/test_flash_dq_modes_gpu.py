"""Flash-attention backward dQ accumulation modes (csrc/kernels/flash_attn.hip fa_dq_atomic): fp32 atomics into
one slab (default) vs per-key-block slabs summed in order (PADDLE2_AMD_FA_DQ_ATOMIC=0, set by
FLAGS_cudnn_deterministic).  Both against an fp32 reference; the ordered mode must be bit-reproducible."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def restore_env():
    old = os.environ.get("PADDLE2_AMD_FA_DQ_ATOMIC")
    yield
    if old is None:
        os.environ.pop("PADDLE2_AMD_FA_DQ_ATOMIC", None)
    else:
        os.environ["PADDLE2_AMD_FA_DQ_ATOMIC"] = old


@pytest.mark.parametrize("causal", [True, False])
def test_dq_atomic_vs_ordered(restore_env, causal):
    from paddle2_amd.ops import _native
    from paddle2_amd.ops import torch_ops as T

    _native.require()
    B, S, H, D = 2, 1536, 4, 128
    g = torch.Generator(device="cpu").manual_seed(3)
    q, k, v, do = (torch.randn(B, S, H, D, generator=g).to(torch.bfloat16).cuda() for _ in range(4))
    scale = D ** -0.5
    out, lse = T._flash_fwd_native(q, k, v, causal, scale)
    res = {}
    for mode in ("1", "0", "0"):
        os.environ["PADDLE2_AMD_FA_DQ_ATOMIC"] = mode
        assert T.dq_atomic() == (mode == "1")
        dq, dk, dv = (torch.empty_like(q) for _ in range(3))
        T._flash_bwd_native(q, k, v, out, do, lse, dq, dk, dv, scale, causal)
        torch.cuda.synchronize()
        res.setdefault(mode, []).append(dq.clone())
    assert torch.equal(res["0"][0], res["0"][1])  # ordered slab sum: bit-reproducible
    # fp32 reference dQ
    qf, kf, vf, dof = (t.float().transpose(1, 2) for t in (q, k, v, do))
    qf.requires_grad_(True)
    s = qf @ kf.transpose(-1, -2) * scale
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=s.device), 1), float("-inf"))
    o = torch.softmax(s, -1) @ vf
    (o * dof).sum().backward()
    ref = qf.grad.transpose(1, 2)
    for mode in ("1", "0"):
        err = (res[mode][0].float() - ref).abs().max() / ref.abs().max()
        assert err < 2e-2, (mode, err.item())
    d = (res["1"][0].float() - res["0"][0].float()).abs().max() / ref.abs().max()
    assert d < 1e-2, d.item()
