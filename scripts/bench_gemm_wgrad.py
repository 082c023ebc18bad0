"""wgrad (x^T @ dy into the fp32 main grad, both operands MN-major) at M = 32768: v4 vs the spread schedule (v5),
bit-compared, plus hipBLASLt's bf16-out NT product for scale.  One JSON line per (shape, kernel)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from paddle2_amd.ops import gemm as G  # noqa: E402

M = 32768
SHAPES = [("qkv", 4096, 12288), ("o", 4096, 4096), ("gate_up", 4096, 22016), ("down", 11008, 4096),
          ("lm_head", 4096, 32000)]


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
for name, K, N in SHAPES:
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    fl = 2.0 * M * N * K
    outs = {}
    for v in (4, 5):
        G.VARIANT = v
        o = torch.zeros(K, N, device="cuda")
        G.mm_wgrad(x, dy, o, 0.0)
        outs[v] = o
        ms = timeit(lambda: G.mm_wgrad(x, dy, o, 1.0))
        print(json.dumps(dict(shape=name, kernel=f"v{v}", ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1),
                              bitwise_eq_v4=bool(torch.equal(outs[v], outs[4])))), flush=True)
    ms = timeit(lambda: torch.matmul(x.t(), dy))
    print(json.dumps(dict(shape=name, kernel="hipblaslt_bf16", ms=round(ms, 4), TFs=round(fl / ms / 1e9, 1))),
          flush=True)
    del x, dy, outs
    torch.cuda.empty_cache()
