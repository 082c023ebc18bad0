"""Variant 3 (4-wave, VGPR-staged) native GEMM vs the default variant 0 on every layout / epilogue,
incl. ragged shapes; prints max |diff| relative to max |ref|.  Then times both on the Llama shapes."""
import sys

import torch

sys.path.insert(0, ".")
from paddle2_amd.ops import gemm as G  # noqa: E402

torch.manual_seed(0)
dev = "cuda"
worst = 0.0
for (M, K, N) in [(1000, 200, 520), (4096, 4096, 4096), (777, 1032, 264), (2048, 11008, 4096)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, N, device=dev) * 0.05).to(torch.bfloat16)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    res = {}
    for v in (0, 3):
        G.VARIANT = v
        o32 = torch.zeros(K, N, device=dev)
        res[v] = [G.mm_fwd(x, w).float(), G.mm_dgrad(dy, w).float(), G.mm_wgrad(x, dy, o32, 1.0).float().clone()]
        if N % 64 == 0:
            sw = G.mm_swiglu(x, w)
            res[v] += [t.float() for t in (sw if isinstance(sw, (tuple, list)) else (sw,))]
        torch.cuda.synchronize()
    ref64 = x.double().cpu() @ w.double().cpu()
    e_ref = ((res[3][0].cpu().double() - ref64).abs().max() / ref64.abs().max()).item()
    for i, (a, b) in enumerate(zip(res[0], res[3])):
        d = ((a - b).abs().max() / a.abs().max().clamp_min(1e-6)).item()
        worst = max(worst, d)
        print(f"M={M} K={K} N={N} out{i}: rel max diff v3 vs v0 = {d:.3e}", flush=True)
    print(f"  fwd v3 vs fp64: {e_ref:.3e}", flush=True)
print("WORST", worst, flush=True)
assert worst < 2e-2, worst
