"""v7 (TN schedule, gemm7.hip) vs v4/v6 and hipBLASLt on the Llama-2-7B GEMMs at M = 32768 tokens.

fwd: y = x @ W — v6 on W [K, N] (layout AK), v7 on W^T [N, K] (layout AK|BK, transpose excluded: timed separately),
hipBLASLt on W^T (torch.matmul(x, wT.t()), the TN layout it is fastest on).  dgrad: dx = dy @ W^T in place.
swiglu: gate|up forward with the SwiGLU epilogue (v4 on W, v7 on W^T).  Each v7 result is checked against the
v6 / v4 result bit for bit (same accumulation order).  One JSON line per (shape, pass, kernel)."""
import json
import sys

import torch

from paddle2_amd.ops import _native as N
from paddle2_amd.ops import gemm as G
from paddle2_amd.ops.torch_ops import transpose2d

M = 32768
SHAPES = [("qkv", 4096, 12288), ("o", 4096, 4096), ("gate_up", 4096, 22016), ("down", 11008, 4096),
          ("lm_head", 4096, 32000)]
VARS = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "7,8,9,10".split(","))]
ITERS = 10


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(ITERS):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / ITERS)
    return best


def emit(shape, pas, kern, ms, flop, **kw):
    print(json.dumps(dict(shape=shape, pass_=pas, kernel=kern, ms=round(ms, 4), TFs=round(flop / ms / 1e9, 1), **kw)),
          flush=True)


def with_variant(v, fn):
    old = G.VARIANT
    G.VARIANT = v
    try:
        return fn()
    finally:
        G.VARIANT = old


g = torch.Generator(device="cuda").manual_seed(0)
for name, K, Nn in SHAPES:
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(K, Nn, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    dy = torch.randn(M, Nn, device="cuda", generator=g).to(torch.bfloat16)
    wt = transpose2d(w)
    flop = 2.0 * M * K * Nn
    emit(name, "transpose_w", "transpose16", timeit(lambda: transpose2d(w)), 0.0)
    # forward
    ref = with_variant(6, lambda: G.mm_fwd(x, w))
    emit(name, "fwd", "v6", timeit(lambda: with_variant(6, lambda: G.mm_fwd(x, w))), flop)
    emit(name, "fwd", "hipblaslt", timeit(lambda: torch.matmul(x, wt.t())), flop)
    out = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
    for v in VARS:
        def f7():
            G._launch(3, 0, x, K, wt, K, out, Nn, None, 0, None, M, Nn, K)
        with_variant(v, f7)
        same = bool(torch.equal(out, ref))
        emit(name, "fwd", f"v{v}", timeit(lambda: with_variant(v, f7)), flop, bitwise_eq_v6=same)
    # dgrad: dx[M, K] = dy[M, Nn] @ W^T
    ref = with_variant(6, lambda: G.mm_dgrad(dy, w))
    emit(name, "dgrad", "v6", timeit(lambda: with_variant(6, lambda: G.mm_dgrad(dy, w))), flop)
    emit(name, "dgrad", "hipblaslt", timeit(lambda: torch.matmul(dy, w.t())), flop)
    for v in VARS:
        o = with_variant(v, lambda: G.mm_dgrad(dy, w))
        same = bool(torch.equal(o, ref))
        emit(name, "dgrad", f"v{v}", timeit(lambda: with_variant(v, lambda: G.mm_dgrad(dy, w))), flop,
             bitwise_eq_v6=same)
    if name == "gate_up":
        ra, rgu = with_variant(4, lambda: G.mm_swiglu(x, w))
        emit(name, "swiglu", "v4", timeit(lambda: with_variant(4, lambda: G.mm_swiglu(x, w))), flop)
        for v in [v for v in VARS if v <= 10 or v in (192, 448, 960, 1472, 1984)]:   # with a SwiGLU instance
            a, gu = with_variant(v, lambda: G.mm_swiglu(x, w))
            same = bool(torch.equal(a, ra) and torch.equal(gu, rgu))
            emit(name, "swiglu", f"v{v}+T", timeit(lambda: with_variant(v, lambda: G.mm_swiglu(x, w))), flop,
                 bitwise_eq_v4=same)
    del x, w, dy, wt, ref
    torch.cuda.empty_cache()
