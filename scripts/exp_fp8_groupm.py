"""fp8 GEMM tile-group height sweep (PADDLE2_AMD_FP8_GROUP_M equivalent, set per run through ops.fp8.GROUP_M) at the
GPT-3 13B forward shapes WITH the bias epilogue (as the step runs them), against hipBLASLt with bias."""
import json

import torch

from paddle2_amd.ops import fp8 as F8


def bench(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


E4, E5 = torch.float8_e4m3fn, torch.float8_e5m2
one = torch.ones(1, device="cuda")
for M, N, K, fa, fb in [(4096, 15360, 5120, E4, E4), (4096, 5120, 5120, E4, E4), (4096, 20480, 5120, E4, E4),
                        (4096, 5120, 20480, E4, E4), (4096, 5120, 15360, E5, E4), (4096, 20480, 5120, E5, E4),
                        (4096, 5120, 5120, E5, E4), (8192, 8192, 8192, E4, E4)]:
    a8 = torch.randn(M, K, device="cuda", dtype=torch.bfloat16).to(fa)
    b8 = torch.randn(N, K, device="cuda", dtype=torch.bfloat16).to(fb)
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16) if fa == E4 else None
    fl = 2.0 * M * N * K
    rec = {"M": M, "N": N, "K": K, "fmt": f"{str(fa)[-6:]}x{str(fb)[-6:]}", "bias": bias is not None}
    for gm in (2, 4, 8, 16):
        F8.GROUP_M = gm
        t = bench(lambda: F8.mm_native(a8, b8, one, one, torch.bfloat16, bias))
        rec[f"g{gm}_TFs"] = round(fl / t / 1e9, 1)
    F8.GROUP_M = 4
    t = bench(lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, bias=bias, out_dtype=torch.bfloat16))
    rec["blas_TFs"] = round(fl / t / 1e9, 1)
    print(json.dumps(rec), flush=True)
