"""Decode GEMM at 17-64 tokens: the whole-K dec64 kernel (8 waves, 1 / 2 / 4 channel tiles per workgroup) vs hipBLASLt on the Llama-2-7B projections,
weights rotated over copies totalling > 512 MB so every call streams them from HBM (a single weight stays in the
256 MB Infinity Cache across a loop and reads at cache speed).  TB/s counts the weight bytes."""
import json

import torch

from paddle2_amd.ops import _native as N
from paddle2_amd.ops import weight_only as WO

WO.DECODE_GEMM = "native"   # time the kernel on every shape (auto routes only the ones it wins)


def bench(fn, copies, iters=60):
    for i in range(6):
        fn(copies[i % len(copies)])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(copies[i % len(copies)])
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for M in (24, 32, 48, 64):
    for name, Nn, K in (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008),
                        ("lm_head", 32000, 4096)):
        wb = Nn * K * 2
        ncp = max(2, (640 << 20) // wb + 1)
        copies = [torch.randn(Nn, K, device="cuda").to(torch.bfloat16) for _ in range(ncp)]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        rec = {"M": M, "proj": name, "N": Nn, "K": K, "copies": ncp}
        WO.DEC64_WAVES = 8
        for rt in (1, 2, 4):
            if Nn % (16 * rt):
                continue
            WO.DEC64_RT = rt
            t = bench(lambda w: WO.decode_matmul(x, w), copies)
            rec[f"dec64_rt{rt}_us"] = round(t * 1e3, 1)
            rec[f"dec64_rt{rt}_TBs"] = round(wb / t / 1e9, 2)
        WO.DEC64_RT = 0
        WO.DEC64_IMPL = "s"
        for cfg in ((0, 0, 0), (16, 1, 1), (16, 1, 2), (8, 1, 2), (11, 2, 1), (8, 2, 2)):
            dw, rt, S = cfg
            if rt and Nn % (64 * rt):
                continue
            WO.DEC64S_CFG = cfg
            t = bench(lambda w: WO.decode_matmul(x, w), copies)
            key = "s_auto" if cfg == (0, 0, 0) else f"s{dw}_{rt}_{S}"
            rec[f"{key}_TBs"] = round(wb / t / 1e9, 2)
        WO.DEC64_IMPL = "r"
        t = bench(lambda w: torch.matmul(x, w.t()), copies)
        rec["blas_us"], rec["blas_TBs"] = round(t * 1e3, 1), round(wb / t / 1e9, 2)
        y = WO.decode_matmul(x, copies[0])
        ref = x.float() @ copies[0].float().t()
        rec["rel"] = float((y.float() - ref).norm() / ref.norm())
        print(json.dumps(rec), flush=True)
        del copies
        torch.cuda.empty_cache()
