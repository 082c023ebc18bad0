"""A native GEMM schedule variant vs the default variant 0 on every layout / epilogue, incl. ragged shapes
and tail split-K; prints max |diff| relative to max |ref| (variants accumulate in the same order, so 0 is
expected) and the error of the variant vs an fp64 product.  Usage: check_gemm_variant.py VARIANT"""
import sys

import torch

sys.path.insert(0, ".")
from paddle2_amd.ops import gemm as G  # noqa: E402

V = int(sys.argv[1]) if len(sys.argv) > 1 else 4
torch.manual_seed(0)
dev = "cuda"
worst = 0.0
for (M, K, N) in [(1000, 200, 520), (4096, 4096, 4096), (777, 1032, 264), (2048, 11008, 4096), (300, 64, 136),
                  (8192, 4096, 22016)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, N, device=dev) * 0.05).to(torch.bfloat16)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    res = {}
    for v in (0, V):
        G.VARIANT = v
        o32 = torch.ones(K, N, device=dev)
        res[v] = [G.mm_fwd(x, w).float(), G.mm_dgrad(dy, w).float(), G.mm_wgrad(x, dy, o32, 1.0).float().clone(),
                  G.mm_wgrad_bf16(x, dy).float()]
        if N % 64 == 0:
            a, gu = G.mm_swiglu(x, w)
            res[v] += [a.float(), gu.float()]
        torch.cuda.synchronize()
    if M * K * N <= 4096 ** 3:
        ref64 = x.double() @ w.double()
        e_ref = ((res[V][0].double() - ref64).abs().max() / ref64.abs().max()).item()
        refw = x.double().t() @ dy.double() + 1.0
        e_w = ((res[V][2].double() - refw).abs().max() / refw.abs().max()).item()
    else:
        e_ref = e_w = float("nan")
    for i, (a, b) in enumerate(zip(res[0], res[V])):
        d = ((a - b).abs().max() / a.abs().max().clamp_min(1e-6)).item()
        worst = max(worst, d)
        print(f"M={M} K={K} N={N} out{i}: rel max diff v{V} vs v0 = {d:.3e}", flush=True)
    print(f"  fwd v{V} vs fp64: {e_ref:.3e}   wgrad(fp32, beta=1) vs fp64: {e_w:.3e}", flush=True)
    del x, w, dy, res
    torch.cuda.empty_cache()
print("WORST", worst, flush=True)
assert worst < 1e-2, worst
