"""Micro-benchmark on one MI355X: the native fp8 GEMM (csrc/kernels/gemm8.hip, K=128 f8f6f4 MFMA) vs hipBLASLt's fp8
GEMM (torch._scaled_mm) vs the bf16 GEMM, at the GPT-3 13B linear shapes (fwd / dgrad / wgrad format pairs)."""
import json

import torch

from paddle2_amd.ops import fp8 as F8


def bench(fn, iters=20):
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
for M, N, K, fa, fb, od in [(8192, 8192, 8192, E4, E4, torch.bfloat16), (4096, 15360, 5120, E4, E4, torch.bfloat16),
                            (4096, 5120, 5120, E4, E4, torch.bfloat16), (4096, 20480, 5120, E4, E4, torch.bfloat16),
                            (4096, 5120, 20480, E4, E4, torch.bfloat16), (4096, 5120, 15360, E5, E4, torch.bfloat16),
                            (5120, 15360, 4096, E4, E5, torch.float32), (16384, 16384, 16384, E4, E4, torch.bfloat16)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    bT = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    a8, b8 = a.to(fa), bT.to(fb)
    fl = 2.0 * M * N * K
    rec = {"M": M, "N": N, "K": K, "fmt": f"{str(fa)[-6:]}x{str(fb)[-6:]}", "out": str(od)[6:]}
    t = bench(lambda: a @ bT.t())
    rec["bf16_TFs"] = round(fl / t / 1e9, 1)
    t = bench(lambda: F8.mm_native(a8, b8, one, one, od))
    rec["native_TFs"] = round(fl / t / 1e9, 1)
    try:
        t = bench(lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=od))
        rec["hipblaslt_TFs"] = round(fl / t / 1e9, 1)
    except Exception as ex:  # pragma: no cover
        rec["hipblaslt_TFs"] = None
        rec["hipblaslt_err"] = str(ex)[:80]
    ref = torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.float32) if fa == E4 or fb == E4 \
        else None
    if ref is not None:
        got = F8.mm_native(a8, b8, one, one, torch.float32 if (fa, fb) == (E4, E5) else od).float()
        rec["rel_vs_hipblaslt"] = float((got - ref).norm() / ref.norm())
    print(json.dumps(rec), flush=True)
