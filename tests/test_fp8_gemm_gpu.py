"""Native fp8 GEMM (csrc/kernels/gemm8.hip, v_mfma_f32_16x16x128_f8f6f4) vs fp32 references of the same op.

Exact-integer operands first (every product and partial sum is exact in fp32, so any lane / k mapping or row /
column swap shows as a mismatch, not as noise), then random data at the GPT-3 13B shapes, the three format pairs of
an fp8 linear (forward e4m3 x e4m3, dgrad e5m2 x e4m3, wgrad e4m3 x e5m2 with bf16 or fp32 dW), ragged M / N,
the bias epilogue and the device dequant factors.
"""
import pytest
import torch

from paddle2_amd.ops import fp8 as F8

pytestmark = pytest.mark.gpu
dev = "cuda"
E4, E5 = torch.float8_e4m3fn, torch.float8_e5m2


def _ints(shape, lo, hi, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    return torch.randint(lo, hi, shape, generator=g, device=dev).float()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("fa,fb,od", [(E4, E4, torch.bfloat16), (E5, E4, torch.bfloat16), (E4, E5, torch.bfloat16),
                                      (E4, E5, torch.float32)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (512, 768, 512), (300, 520, 768),
                                   (1024, 1024, 4096), (1000, 1000, 4096)])   # 16 tiles: tail split-K, 4 slices
def test_exact_integers(fa, fb, od, M, N, K):
    a = _ints((M, K), -4, 5, 1)          # |products| <= 16, sums < 2^24: exact in fp32
    b = _ints((N, K), -4, 5, 2)
    one = torch.ones(1, device=dev)
    c = F8.mm_native(a.to(fa), b.to(fb), one, one, od)
    assert c is not None
    ref = a @ b.t()
    if od == torch.float32:
        assert torch.equal(c, ref)
    else:
        assert torch.equal(c, ref.to(torch.bfloat16))


def test_identity_asymmetric():
    """A = I, asymmetric B: a transposed C write cannot pass."""
    n = 256
    eye = torch.eye(n, device=dev)
    b = (torch.arange(n * n, device=dev, dtype=torch.float32).reshape(n, n) % 15) - 7
    one = torch.ones(1, device=dev)
    c = F8.mm_native(eye.to(E4), b.t().contiguous().to(E5), one, one, torch.float32)   # |b| <= 7: exact in e5m2
    assert torch.equal(c, b)


@pytest.mark.parametrize("fa,fb,od", [(E4, E4, torch.bfloat16), (E5, E4, torch.bfloat16), (E4, E5, torch.float32)])
@pytest.mark.parametrize("M,N,K", [(2048, 5120, 5120), (1000, 15360, 5120), (4096, 5120, 20480)])
def test_random_scaled(fa, fb, od, M, N, K):
    g = torch.Generator(device=dev).manual_seed(3)
    a = torch.randn(M, K, generator=g, device=dev) * 4
    b = torch.randn(N, K, generator=g, device=dev) * 0.5
    a8, b8 = a.to(fa), b.to(fb)
    sa = torch.full((1,), 0.25, device=dev)
    sb = torch.full((1,), 3.0, device=dev)
    c = F8.mm_native(a8, b8, sa, sb, od)
    ref = (a8.float() @ b8.float().t()) * 0.75
    assert _rel(c, ref) < (1e-4 if od == torch.float32 else 8e-3)


def test_bias_epilogue():
    M, N, K = 600, 1024, 512
    g = torch.Generator(device=dev).manual_seed(4)
    a8 = torch.randn(M, K, generator=g, device=dev).to(E4)
    b8 = torch.randn(N, K, generator=g, device=dev).to(E4)
    bias = torch.randn(N, generator=g, device=dev).to(torch.bfloat16)
    one = torch.ones(1, device=dev)
    c = F8.mm_native(a8, b8, one, one, torch.bfloat16, bias)
    ref = a8.float() @ b8.float().t() + bias.float()
    assert _rel(c, ref) < 8e-3


def test_outside_domain_returns_none():
    one = torch.ones(1, device=dev)
    a = torch.zeros(256, 200, device=dev).to(E4)   # K % 256 != 0
    assert F8.mm_native(a, a, one, one, torch.bfloat16) is None


def test_fp8_linear_native_matches_blas(monkeypatch):
    """The fp8 linear's three GEMMs on the native kernel vs on hipBLASLt (same casts, same scales)."""
    M, K, Nn = 1024, 512, 768
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, Nn, generator=g, device=dev) * 0.05).to(torch.bfloat16)
    dy = torch.randn(M, Nn, generator=g, device=dev).to(torch.bfloat16)
    outs = {}
    for mode in ("native", "blas"):
        monkeypatch.setattr(F8, "GEMM", mode)
        metas = [F8.FP8TensorMeta(f, device=torch.device(dev)) for f in (E4, E4, E5)]
        xi, wi = x.clone().requires_grad_(), w.clone().requires_grad_()
        y = F8._FP8LinearFn.apply(xi, wi, None, *metas)
        y.backward(dy)
        outs[mode] = (y.float(), xi.grad.float(), wi.grad.float())
    for a, b in zip(outs["native"], outs["blas"]):
        assert _rel(a, b) < 1e-2
