"""SwiGLU-epilogue forward vs the plain forward at the Llama-2-7B gate|up shape, over the tile-group height
(PASS_GROUP_M) — is the epilogue or the B-operand reuse what costs the SwiGLU GEMM its 15 %?"""
import json

import torch

from paddle2_amd.ops import gemm as G

dev = "cuda"
M, K, H = 32768, 4096, 11008
x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
w = (torch.randn(K, 2 * H, device=dev) * K ** -0.5).to(torch.bfloat16)
flop = 2.0 * M * K * 2 * H


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / n)
    return best


wt = G._wt(w)
for g in (1, 2, 4, 8, 16, 32):
    G.PASS_GROUP_M["swiglu"] = g
    G.PASS_GROUP_M["fwd"] = g
    t_swi = timeit(lambda: G.mm_swiglu(x, w))
    t_fwd = timeit(lambda: G.mm_fwd(x, w))
    print(json.dumps({"group_m": g, "swiglu_ms": round(t_swi, 3), "swiglu_TFs": round(flop / t_swi / 1e9, 1),
                      "fwd_ms": round(t_fwd, 3), "fwd_TFs": round(flop / t_fwd / 1e9, 1)}), flush=True)
