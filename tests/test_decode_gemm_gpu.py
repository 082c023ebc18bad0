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


@pytest.mark.parametrize("rt", [0, 1, 2, 4])
@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("M", [17, 40, 64])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 11008), (12288, 4096), (48, 192), (192, 128)])
def test_dec64_whole_k_kernel(M, N, K, waves, rt, monkeypatch):
    """The M > 16 whole-K kernel (dec64_kernel) at both workgroup widths and every channel-tile count (rt, 0 =
    auto), ragged M, K not a multiple of the wave count's 64-wide steps (11008 = 172 steps), tiny shapes with fewer
    steps than waves."""
    if rt and N % (16 * rt):
        pytest.skip("N not a multiple of the workgroup's channels")
    monkeypatch.setattr(WO, "DECODE_GEMM", "native")
    monkeypatch.setattr(WO, "DEC64_WAVES", waves)
    monkeypatch.setattr(WO, "DEC64_RT", rt)
    monkeypatch.setattr(WO, "DEC64_IMPL", "r")
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


def test_auto_routing(monkeypatch):
    """auto: native split-K at M <= 8 on every width and at M <= 16 on N <= 8192, the M > 16 kernels only on the
    4096 x 4096 projection, hipBLASLt elsewhere (profiles/r4_decode_gemm.md, profiles/r5_decode_serving.md)."""
    monkeypatch.setattr(WO, "DECODE_GEMM", "auto")

    def ok(M, N, K):
        return WO.decode_ok(torch.empty(M, K, device=dev, dtype=torch.bfloat16),
                            torch.empty(N, K, device=dev, dtype=torch.bfloat16))

    assert ok(1, 4096, 4096) and ok(16, 4096, 11008) and ok(1, 12288, 4096) and ok(8, 22016, 4096)
    assert not ok(9, 12288, 4096) and not ok(16, 22016, 4096)
    assert ok(32, 4096, 4096) and ok(64, 4096, 4096) and not ok(32, 4096, 11008) and not ok(64, 12288, 4096)


@pytest.mark.parametrize("cfg", [(0, 0, 0), (8, 1, 1), (16, 1, 3), (8, 2, 1), (11, 2, 2)])
@pytest.mark.parametrize("M", [17, 40, 64])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 11008), (12288, 4096), (192, 128), (256, 320)])
def test_dec64s_lds_x_kernel(M, N, K, cfg, monkeypatch):
    """The LDS-X M > 16 kernel (dec64s_kernel): ring depths 8 / 11 / 16, one or two channel tiles per wave, split-K
    1-3 (fp32 partials + reduce), auto; ragged M, tiny K with fewer steps than the ring, K not a multiple of S."""
    dw, rt, S = cfg
    if (rt and N % (64 * rt)) or S > K // 64:
        pytest.skip("outside this configuration's domain")
    monkeypatch.setattr(WO, "DECODE_GEMM", "native")
    monkeypatch.setattr(WO, "DEC64_IMPL", "s")
    monkeypatch.setattr(WO, "DEC64S_CFG", cfg)
    g = torch.Generator(device=dev).manual_seed(11 * M + N + K)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    wt = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g).to(torch.bfloat16)
    y = WO.decode_matmul(x, wt, b)
    ref = x.float() @ wt.float().t() + b.float()
    assert y.shape == (M, N) and _rel(y, ref) < 8e-3
    y2 = WO.decode_matmul(x, wt)
    assert _rel(y2, x.float() @ wt.float().t()) < 8e-3


@pytest.mark.parametrize("M", [1, 5, 16])
@pytest.mark.parametrize("N,K", [(4096, 11008), (256, 704), (128, 64)])
def test_decode_glu_matmul_matches_fp32(M, N, K):
    """The SwiGLU-staged split-K decode GEMM (dec_gemm_kernel<GLU>): (silu(gate) * up, rounded to bf16 like
    swiglu_fwd) @ W^T against fp32, for the Llama-2-7B down projection and small shapes (K = 64: one K step)."""
    g = torch.Generator(device=dev).manual_seed(5 * M + N + K)
    gu = torch.randn(M, 2 * K, device=dev, generator=g).to(torch.bfloat16)
    wt = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
    assert WO.decode_glu_ok(gu, wt)
    y = WO.decode_glu_matmul(gu, wt)
    gate, up = gu.float()[:, :K], gu.float()[:, K:]
    a = (gate * torch.sigmoid(gate) * up).to(torch.bfloat16).float()
    ref = a @ wt.float().t()
    assert y.shape == (M, N) and _rel(y, ref) < 8e-3


@pytest.mark.gpu
@pytest.mark.parametrize("M,Nn,K,glu,has_bias", [(1, 4096, 4096, False, False), (4, 12288, 4096, False, True),
                                                 (16, 22016, 4096, False, False), (1, 4096, 11008, True, False),
                                                 (8, 4096, 11008, True, False), (3, 1024, 512, False, True)])
def test_dec_gemm_fused_reduce_bit_exact(monkeypatch, M, Nn, K, glu, has_bias):
    """Split-K partials summed by the last-arriving workgroup of each column block (PADDLE2_AMD_DEC_FUSED_REDUCE)
    equal the separate wo_reduce launch bit for bit (same split order), over repeated calls and HIP-graph replays
    (the kernel re-arms its arrival counters)."""
    from paddle2_amd.ops import weight_only as WO

    torch.manual_seed(M * 7 + K)
    x = torch.randn(M, 2 * K if glu else K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(Nn, K, device="cuda") * 0.02).bfloat16()
    b = (torch.randn(Nn, device="cuda") * 0.1).bfloat16() if has_bias else None

    def run():
        return WO.decode_glu_matmul(x, w) if glu else WO.decode_matmul(x, w, b)

    monkeypatch.setattr(WO, "DECODE_GEMM", "native")   # the split-K kernel for every shape here
    assert glu or WO.decode_ok(x, w)
    monkeypatch.setattr(WO, "DEC_FUSED_REDUCE", False)
    ref = run()
    exact = x.float() @ w.float().t() if not glu else None
    if exact is not None:
        exact = exact + (b.float() if b is not None else 0)
        assert float((ref.float() - exact).norm() / exact.norm()) < 1e-2
    monkeypatch.setattr(WO, "DEC_FUSED_REDUCE", True)
    for _ in range(3):
        assert torch.equal(run(), ref)
    y = run()   # warm the counter buffer outside the capture
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = run()
    for _ in range(3):
        y.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, ref)
    assert WO._DEC_CNT and all(int(c.abs().sum()) == 0 for c in WO._DEC_CNT.values())
