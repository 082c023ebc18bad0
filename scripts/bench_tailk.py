"""v7 forward / dgrad with and without the tail split-K (ops/gemm.py V7_TAILK) at the GPT-3 13B (M = 4096) and
Llama-2-7B shapes: one JSON line per (shape, pass) with both times and TF/s."""
import json

import torch

from paddle2_amd.ops import gemm as G


def _t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


SHAPES = [(4096, 5120, 5120), (4096, 5120, 20480), (4096, 15360, 5120), (4096, 20480, 5120),
          (32768, 11008, 4096), (32768, 4096, 11008), (32768, 32000, 4096)]
for M, N, K in SHAPES:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(K, N, device="cuda", dtype=torch.bfloat16) * K ** -0.5
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    for name, fn in (("fwd", lambda: G.mm_fwd(x, w)), ("dgrad", lambda: G.mm_dgrad(dy, w))):
        G.V7_TAILK = True
        t1 = _t(fn)
        G.V7_TAILK = False
        t0 = _t(fn)
        G.V7_TAILK = True
        lib = _t((lambda: x @ w) if name == "fwd" else (lambda: dy @ w.t()))
        fl = 2.0 * M * N * K
        print(json.dumps({"M": M, "N": N, "K": K, "pass": name, "ms_tailk": round(t1, 4), "ms_whole": round(t0, 4),
                          "ms_hipblaslt": round(lib, 4), "tf_tailk": round(fl / t1 / 1e9, 1),
                          "tf_whole": round(fl / t0 / 1e9, 1), "tf_hipblaslt": round(fl / lib / 1e9, 1)}), flush=True)
    del x, w, dy

# fp8 (gemm8.hip) forward shapes of GPT-3 13B at M = 4096: native with / without the tail split vs hipBLASLt
from paddle2_amd.ops import fp8 as F8  # noqa: E402

one = torch.ones(1, device="cuda")
for M, N, K in [(4096, 5120, 5120), (4096, 15360, 5120), (4096, 20480, 5120), (4096, 5120, 20480)]:
    a = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
    b = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
    F8.TAILK = True
    t1 = _t(lambda: F8.mm_native(a, b, one, one, torch.bfloat16))
    F8.TAILK = False
    t0 = _t(lambda: F8.mm_native(a, b, one, one, torch.bfloat16))
    F8.TAILK = True
    lib = _t(lambda: torch._scaled_mm(a, b.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
    fl = 2.0 * M * N * K
    print(json.dumps({"fp8": True, "M": M, "N": N, "K": K, "ms_tailk": round(t1, 4), "ms_whole": round(t0, 4),
                      "ms_hipblaslt": round(lib, 4), "tf_tailk": round(fl / t1 / 1e9, 1),
                      "tf_whole": round(fl / t0 / 1e9, 1), "tf_hipblaslt": round(fl / lib / 1e9, 1)}), flush=True)
