"""Flash attention coverage beyond the bf16 / D in {64, 128} core (csrc/kernels/flash_attn.hip):
fp16 inputs (f16 MFMA), D = 256 (4-wave backward with 128-key blocks), padded head dims (D = 96, 80),
and the long-sequence shapes the Llama bench runs (S = 4096 / 8192, many key blocks, the causal grid
reorder and the XCD remap).  Reference: the same autograd.Function's fp32 math branch, run on the GPU
in fp32 (reference registers fp16+bf16 with hd <= 256: phi/kernels/gpu/flash_attn_kernel.cu:698-746)."""
import pytest
import torch

from paddle2_amd.ops import torch_ops as T

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _err(a, b):
    a, b = a.float(), b.float()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-6)


def _run(B, Sq, Sk, Hq, Hk, D, dtype, causal, seed=0, tol=2e-2):
    g = torch.Generator(device=DEV).manual_seed(seed)
    mk = lambda *s: torch.randn(*s, generator=g, device=DEV)  # noqa: E731
    q32, k32, v32 = mk(B, Sq, Hq, D), mk(B, Sk, Hk, D), mk(B, Sk, Hk, D)
    go32 = mk(B, Sq, Hq, D)
    q, k, v = (t.to(dtype).requires_grad_() for t in (q32, k32, v32))
    # fp32 reference on the rounded inputs
    qr, kr, vr = (t.to(dtype).float().requires_grad_() for t in (q32, k32, v32))
    o, lse = T.flash_attention(q, k, v, causal)
    orf, lr = T.flash_attention(qr, kr, vr, causal)
    assert o.dtype == dtype and o.shape == (B, Sq, Hq, D)
    assert _err(o, orf) < tol
    fin = torch.isfinite(lr)
    assert (lse[fin] - lr[fin]).abs().max().item() < 1e-2
    o.backward(go32.to(dtype))
    orf.backward(go32.to(dtype).float())
    for a, b in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        assert a.dtype == dtype and torch.isfinite(a.float()).all()
        assert _err(a, b) < 3 * tol


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("D", [64, 128, 256, 96, 80])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_dtypes_and_head_dims(dtype, D, causal):
    _run(2, 300, 300, 4, 2, D, dtype, causal)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_flash_d256_cross_lengths(dtype):
    _run(1, 130, 517, 2, 1, 256, dtype, True, seed=3)


@pytest.mark.parametrize("S", [4096, 8192])
def test_flash_long_sequences_bf16_causal(S):
    """The bench's per-layer shape at full sequence length (fewer heads/batch to bound the fp32 reference)."""
    _run(1, S, S, 4, 4, 128, torch.bfloat16, True, seed=S)


def test_flash_long_sequence_fp16_gqa():
    _run(1, 4096, 4096, 8, 2, 128, torch.float16, True, seed=7)


def test_flash_varlen_fp16_and_d256():
    """varlen (cu_seqlens) path with fp16 and D = 256 against per-sequence dense calls."""
    for dtype, D in ((torch.float16, 128), (torch.bfloat16, 256)):
        lens = [37, 300, 129]
        cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
        tot = sum(lens)
        q = torch.randn(tot, 4, D, device=DEV, dtype=dtype)
        k = torch.randn(tot, 2, D, device=DEV, dtype=dtype)
        v = torch.randn(tot, 2, D, device=DEV, dtype=dtype)
        o, _ = T.flash_attention_varlen(q, k, v, cu, cu, max(lens), max(lens), causal=True)
        for i in range(len(lens)):
            a, b = int(cu[i]), int(cu[i + 1])
            ref, _ = T.flash_attention(q[a:b].float()[None], k[a:b].float()[None], v[a:b].float()[None], True)
            assert _err(o[a:b], ref[0]) < 2e-2


@pytest.mark.parametrize("causal,Sq,Sk,Hq,Hk", [(False, 2304, 2304, 4, 4), (True, 1000, 1000, 4, 2),
                                                (True, 512, 1536, 2, 2), (False, 300, 700, 4, 1)])
def test_fwd_8wave_matches_4wave_and_fp32(monkeypatch, causal, Sq, Sk, Hq, Hk):
    """The 8-wave forward (256 query rows per workgroup, per-wave causal tile skip) against the 4-wave kernel
    (bit for bit: same per-row accumulation order) and the fp32 math reference; ragged Sq, Sk > Sq (bottom-right
    causal alignment) and GQA included."""
    g = torch.Generator(device=DEV).manual_seed(3)
    q = torch.randn(2, Sq, Hq, 128, generator=g, device=DEV).to(torch.bfloat16)
    k = torch.randn(2, Sk, Hk, 128, generator=g, device=DEV).to(torch.bfloat16)
    v = torch.randn(2, Sk, Hk, 128, generator=g, device=DEV).to(torch.bfloat16)
    outs = {}
    for w in ("4", "8"):
        monkeypatch.setenv("PADDLE2_AMD_FA_FWD_WAVES", w)
        o, lse = T.flash_attention(q, k, v, causal)
        torch.cuda.synchronize()
        outs[w] = (o, lse)
    assert torch.equal(outs["4"][0], outs["8"][0]) and torch.equal(outs["4"][1], outs["8"][1])
    orf, _ = T.flash_attention(q.float(), k.float(), v.float(), causal)
    assert _err(outs["8"][0], orf) < 2e-2


@pytest.mark.parametrize("nh,nkv", [(4, 4), (8, 2)])
def test_qkv_packed_attention_matches_sliced(nh, nkv):
    """qkv_attention (GPT path: dQ/dK/dV written straight into one dQKV buffer) equals flash_attention on the
    sliced views, forward and gradients, bit for bit (same kernels, same accumulation)."""
    g = torch.Generator(device=DEV).manual_seed(5)
    qkv = torch.randn(2, 300, nh + 2 * nkv, 128, generator=g, device=DEV).to(torch.bfloat16).requires_grad_()
    o = T.qkv_attention(qkv, nh, nkv, causal=True)
    go = torch.randn(o.shape, generator=g, device=DEV).to(torch.bfloat16)
    o.backward(go)
    ref_in = qkv.detach().clone().requires_grad_()
    o2, _ = T.flash_attention(ref_in[:, :, :nh], ref_in[:, :, nh:nh + nkv], ref_in[:, :, nh + nkv:], True)
    o2.backward(go)
    assert torch.equal(o, o2) and torch.equal(qkv.grad, ref_in.grad)
