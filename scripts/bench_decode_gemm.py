"""Decode GEMM bandwidth on one MI355X: the native stream kernel vs hipBLASLt (torch.matmul on the cached W^T) at the
Llama-2-7B projections, b = 1..64 tokens; TB/s counts the weight bytes (read once)."""
import json

import torch

from paddle2_amd.ops import weight_only as WO


def bench(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for M in (1, 16, 64):
    for name, N, K in (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008),
                       ("lm_head", 32000, 4096)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        wt = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        wb = N * K * 2
        t_n = bench(lambda: WO.decode_matmul(x, wt))
        t_b = bench(lambda: torch.matmul(x, wt.t()))
        rel = float((WO.decode_matmul(x, wt).float() - (x.float() @ wt.float().t())).norm() /
                    (x.float() @ wt.float().t()).norm())
        print(json.dumps({"M": M, "proj": name, "N": N, "K": K, "native_us": round(t_n * 1e3, 1),
                          "native_TBs": round(wb / t_n / 1e9, 2), "blas_us": round(t_b * 1e3, 1),
                          "blas_TBs": round(wb / t_b / 1e9, 2), "rel": rel}), flush=True)
