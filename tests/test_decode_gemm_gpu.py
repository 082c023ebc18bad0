"""Native decode GEMM (csrc/kernels/weight_only.hip dec_gemm_kernel: bf16 weights streamed once, split-K MFMA) vs an
fp32 PyTorch reference, at the Llama-2-7B decode projections for 1..64 tokens, ragged M, with bias."""
import pytest
import torch

from paddle2_amd.ops import weight_only as WO

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("N,K", [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008), (32000, 4096), (128, 64)])
@pytest.mark.parametrize("M", [1, 8, 33, 64])
def test_decode_gemm_matches_fp32(M, N, K, monkeypatch):
    monkeypatch.setattr(WO, "DECODE_GEMM", "native")
    g = torch.Generator(device=dev).manual_seed(M + N)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    wt = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g).to(torch.bfloat16)
    assert WO.decode_ok(x, wt)
    y = WO.decode_matmul(x, wt, b)
    ref = x.float() @ wt.float().t() + b.float()
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert _rel(y, ref) < 8e-3


@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("M", [17, 40, 64])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 11008), (12288, 4096), (48, 192)])
def test_dec64_whole_k_kernel(M, N, K, waves, monkeypatch):
    """The M > 16 whole-K kernel (dec64_kernel) at both workgroup widths, ragged M, K not a multiple of the wave
    count's 64-wide steps (11008 = 172 steps), a tiny shape with fewer steps than waves."""
    monkeypatch.setattr(WO, "DECODE_GEMM", "auto")
    monkeypatch.setattr(WO, "DEC64_WAVES", waves)
    g = torch.Generator(device=dev).manual_seed(7 * M + N)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    wt = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g).to(torch.bfloat16)
    assert WO.decode_ok(x, wt)
    y = WO.decode_matmul(x, wt, b)
    ref = x.float() @ wt.float().t() + b.float()
    assert _rel(y, ref) < 8e-3
    y2 = WO.decode_matmul(x, wt)
    assert _rel(y2, x.float() @ wt.float().t()) < 8e-3
