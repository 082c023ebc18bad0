"""Weight gradient into the fp32 main grad (x^T @ dy, both operands MN-major): v4's spread kernel (variant 5) vs the
persistent v7 spread kernel with MN-major operands (G.V7_MN, gemm7.hip SCHED bit 15), beta 0 (the step's first write)
and beta 1 (accumulation), at the Llama-2-7B token count (32768) and the GPT-3 13B one (4096); rel_vs_v5 compares the
beta-0 outputs (tail split-K plans differ, so not bitwise).  One JSON line per (tokens, shape, kernel, beta)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from paddle2_amd.ops import gemm as G  # noqa: E402

CASES = [(32768, "qkv", 4096, 12288), (32768, "o", 4096, 4096), (32768, "gate_up", 4096, 22016),
         (32768, "down", 11008, 4096),
         (4096, "g13_qkv", 5120, 15360), (4096, "g13_o", 5120, 5120), (4096, "g13_fc1", 5120, 20480),
         (4096, "g13_fc2", 20480, 5120)]


def timeit(fn, iters=8):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


g = torch.Generator(device="cuda").manual_seed(0)
for T, name, K, N in CASES:
    x = torch.randn(T, K, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
    fl = 2.0 * T * N * K
    outs = {}
    for rnd in range(2):
        for v in (5, G.V7_MN):
            G.VARIANT = v
            o = torch.zeros(K, N, device="cuda")
            G.mm_wgrad(x, dy, o, 0.0)
            outs[v] = o.clone()
            for beta in (0.0, 1.0):
                ms = timeit(lambda: G.mm_wgrad(x, dy, o, beta))
                print(json.dumps(dict(tokens=T, shape=name, kernel="v5" if v == 5 else "v7mn", beta=beta, round=rnd,
                                      ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1),
                                      rel_vs_v5=float((outs[v] - outs[5]).norm() / outs[5].norm()))), flush=True)
    del x, dy, outs
    torch.cuda.empty_cache()
