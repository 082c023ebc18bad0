"""Micro-benchmark: bf16 GEMM vs fp8 (e4m3, per-tensor scaled) GEMM through hipBLASLt on one MI355X."""
import json

import torch


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


out = []
for M, N, K in [(8192, 8192, 8192), (16384, 5120, 5120), (16384, 15360, 5120), (16384, 20480, 5120)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    t_bf16 = bench(lambda: a @ b)
    a8 = a.to(torch.float8_e4m3fn)
    b8 = b.t().contiguous().to(torch.float8_e4m3fn).t()
    one = torch.ones(1, device="cuda")
    try:
        t_fp8 = bench(lambda: torch._scaled_mm(a8, b8, scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
    except Exception as ex:  # pragma: no cover
        t_fp8 = float("nan")
        print("fp8 failed:", ex)
    fl = 2.0 * M * N * K
    out.append({"M": M, "N": N, "K": K, "bf16_ms": round(t_bf16, 4), "bf16_TFs": round(fl / t_bf16 / 1e9, 1),
                "fp8_ms": round(t_fp8, 4), "fp8_TFs": round(fl / t_fp8 / 1e9, 1)})
    print(json.dumps(out[-1]), flush=True)
