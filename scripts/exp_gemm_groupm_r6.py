"""Tile-group height (rows of 256 x 256 tiles walked together, ops/gemm.py PASS_GROUP_M) of the round-6 GEMM routes at
the Llama-2-7B shapes (argv[1] = 32768 tokens) or the GPT-3 13B ones (4096): the forward on W as stored (fwd_nn,
V7_NNF), the MN-major weight gradient (wgrad, V7_MN) and the TN dgrad (argv[2] = comma-separated passes).  One JSON line per (pass, shape, group_m, round): ms and TF/s, best of 3 x 8."""
import json
import sys

import torch

sys.path.insert(0, ".")
from paddle2_amd.ops import gemm as G  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
SHAPES = ([("qkv", 4096, 12288), ("o", 4096, 4096), ("gate_up", 4096, 22016), ("down", 11008, 4096)] if T == 32768 else
          [("g13_qkv", 5120, 15360), ("g13_o", 5120, 5120), ("g13_fc1", 5120, 20480), ("g13_fc2", 20480, 5120)])
PASSES = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fwd_nn", "wgrad"]


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
    x = torch.randn(T, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(K, N, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    dy = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
    o32 = torch.zeros(K, N, device="cuda")
    fl = 2.0 * T * K * N
    for rnd in range(2):
        for gm in (2, 4, 8, 16):
            for k in ("fwd_nn", "fwd_nn_wide", "wgrad", "dgrad"):
                G.PASS_GROUP_M[k] = gm
            fns = {"fwd_nn": lambda: G.mm_fwd(x, w), "wgrad": lambda: G.mm_wgrad(x, dy, o32, 0.0),
                   "dgrad": lambda: G.mm_dgrad(dy, w)}
            for pas, fn in ((p_, fns[p_]) for p_ in PASSES):
                ms = timeit(fn)
                print(json.dumps(dict(pass_=pas, shape=name, group_m=gm, round=rnd, ms=round(ms, 4),
                                      TFs=round(fl / ms / 1e9, 1))), flush=True)
    del x, w, dy, o32
    torch.cuda.empty_cache()
