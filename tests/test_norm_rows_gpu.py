"""Few-row norm forward (csrc/kernels/norm.hip norm_fwd_row_kernel, M <= 64: one workgroup per row, 4 waves
splitting it) vs an fp32 PyTorch reference and vs the one-wave-per-row kernel on the same rows inside a large batch.
Covers RMSNorm / LayerNorm, residual in / out, bias, fp32 weights, and row widths that leave threads idle."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(x, w, b, res, eps, ln):
    h = x.float() + res.float() if res is not None else x.float()
    h = h.to(x.dtype).float()
    if ln:
        yf = (h - h.mean(-1, keepdim=True)) * torch.rsqrt(h.var(-1, unbiased=False, keepdim=True) + eps)
    else:
        yf = h * torch.rsqrt(h.square().mean(-1, keepdim=True) + eps)
    yf = yf * w.float() + (b.float() if b is not None else 0)
    return yf, h


@pytest.mark.parametrize("M", [1, 3, 16, 64])
@pytest.mark.parametrize("N", [4096, 5120, 1000, 8192])
@pytest.mark.parametrize("ln,has_res,has_b,w32", [(False, True, False, False), (False, False, False, False),
                                                  (True, True, True, False), (True, False, True, True)])
def test_norm_forward_few_rows(M, N, ln, has_res, has_b, w32):
    from paddle2_amd.ops import torch_ops as T

    torch.manual_seed(M + N)
    x = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16) if has_res else None
    wdt = torch.float32 if w32 else torch.bfloat16
    w = (1 + 0.1 * torch.randn(N, device=DEV)).to(wdt)
    b = (0.1 * torch.randn(N, device=DEV)).to(wdt) if (ln and has_b) else None
    eps = 1e-5 if ln else 1e-6
    with torch.no_grad():
        out = T.layer_norm(x, w, b, eps, residual=res) if ln else T.rms_norm(x, w, eps, residual=res)
        y, h = out if has_res else (out, None)
        yf, hf = _ref(x, w, b, res, eps, ln)
        torch.testing.assert_close(y.float(), yf, rtol=2e-2, atol=2e-2)
        if has_res:
            torch.testing.assert_close(h.float(), hf, rtol=0, atol=0)
        # the same rows inside a 320-row batch take the one-wave-per-row kernel
        big = torch.randn(320, N, device=DEV, dtype=torch.bfloat16)
        big[:M] = x
        bres = None
        if has_res:
            bres = torch.randn(320, N, device=DEV, dtype=torch.bfloat16)
            bres[:M] = res
        ob = T.layer_norm(big, w, b, eps, residual=bres) if ln else T.rms_norm(big, w, eps, residual=bres)
        yb = ob[0] if has_res else ob
        assert float((yb[:M].float() - y.float()).abs().max()) <= 0.0625
