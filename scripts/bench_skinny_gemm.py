"""Decode-shaped (M = batch) GEMMs on the Llama-2-7B weights: hipBLASLt on the Paddle [K, N] layout, hipBLASLt on
a pre-transposed [N, K] weight (inference weights are static, so the transpose is paid once at load) and the
native MFMA kernel.  Prints one JSON line per shape with the weight-streaming bandwidth."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from paddle2_amd.ops import gemm as G  # noqa: E402


def timeit(f, iters=50):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for M in (64, 128):
    for K, N in ((4096, 12288), (4096, 4096), (4096, 22016), (11008, 4096)):
        x = torch.randn(M, K, device="cuda").bfloat16()
        ws = [torch.randn(K, N, device="cuda").bfloat16() for _ in range(8)]   # rotate: > L2 / MALL reuse
        wts = [w.t().contiguous() for w in ws]
        ref = x.float() @ ws[0].float()
        res = {"M": M, "K": K, "N": N}
        i = [0]

        def nxt(lst):
            i[0] = (i[0] + 1) % len(lst)
            return lst[i[0]]

        cases = {"blas_KN": lambda: torch.matmul(x, nxt(ws)), "blas_NK": lambda: torch.matmul(x, nxt(wts).t())}
        if G.supported_fwd(x, ws[0]):
            cases["native"] = lambda: G.mm_fwd(x, nxt(ws))
        for name, f in cases.items():
            ms = timeit(f)
            res[name + "_ms"] = round(ms, 4)
            res[name + "_TBs"] = round(K * N * 2 / ms / 1e9, 2)
        fixed = {"blas_KN": lambda: torch.matmul(x, ws[0]), "blas_NK": lambda: torch.matmul(x, wts[0].t())}
        if "native" in cases:
            fixed["native"] = lambda: G.mm_fwd(x, ws[0])
        err = {n: float((f().float() - ref).abs().max() / ref.abs().max()) for n, f in fixed.items()}
        res["max_err"] = err
        print(json.dumps(res), flush=True)
