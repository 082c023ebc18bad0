"""Native MFMA GEMM vs hipBLASLt (torch.matmul) on the Llama-2-7B Linear shapes at M = 32768 tokens.

For each weight shape [K, N]: forward x@W, dgrad dy@W^T, wgrad x^T@dy (native: fp32 main-grad epilogue;
hipBLASLt: bf16 out via the fastest layout it has — the NT product x^T @ dy).  Random N(0,1)
activations, N(0, 0.02) weights.  Prints one JSON line per (shape, pass).
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from paddle2_amd.ops import gemm as G  # noqa: E402

dev = "cuda"
M = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
VARIANTS = [int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1"])]
SHAPES = {"qkv": (4096, 12288), "o_proj": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096),
          "lm_head": (4096, 32000)}


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for name, (K, N) in SHAPES.items():
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, N, device=dev) * 0.02).to(torch.bfloat16)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    out32 = torch.zeros(K, N, device=dev)
    fl = 2.0 * M * N * K
    rows = []

    def nat(fn):
        res = {}
        for v in VARIANTS:
            G.VARIANT = v
            res[v] = timeit(fn)
        return res

    rows.append(("fwd", nat(lambda: G.mm_fwd(x, w)), timeit(lambda: torch.matmul(x, w))))
    rows.append(("dgrad", nat(lambda: G.mm_dgrad(dy, w)), timeit(lambda: torch.matmul(dy, w.t()))))
    rows.append(("wgrad", nat(lambda: G.mm_wgrad(x, dy, out32, 1.0)), timeit(lambda: torch.matmul(x.t(), dy))))
    if name == "gate_up":
        rows.append(("fwd_swiglu", nat(lambda: G.mm_swiglu(x, w)), None))
    for p, tn, tb in rows:
        rec = {"shape": name, "M": M, "K": K, "N": N, "pass": p}
        for v, t in tn.items():
            rec[f"native_v{v}_TFs"] = round(fl / t / 1e9, 1)
        rec["hipblaslt_TFs"] = None if tb is None else round(fl / tb / 1e9, 1)
        print(json.dumps(rec), flush=True)
    del x, w, dy, out32
    torch.cuda.empty_cache()
