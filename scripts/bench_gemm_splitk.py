"""Tail split-K on/off for the Llama-2-7B Linear GEMMs at 32768 tokens (wgrad fp32 main grad, fwd bf16).
CUDA-event timing, 20 iterations after 3 warm-ups; PF/s = 2MNK / time.  One JSON line per (pass, shape)."""
import json

import torch

from paddle2_amd.ops import gemm as G

T = 32768
SHAPES = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


for name, (K, N) in SHAPES.items():
    x = torch.randn(T, K, device="cuda").bfloat16()
    dy = torch.randn(T, N, device="cuda").bfloat16()
    w = (torch.randn(K, N, device="cuda") * 0.02).bfloat16()
    out = torch.zeros(K, N, device="cuda")
    row = {"shape": name, "K": K, "N": N}
    for split in (False, True):
        G.SPLITK = split
        ms = timeit(lambda: G.mm_wgrad(x, dy, out, beta=1.0))
        row[f"wgrad_{'split' if split else 'nosplit'}_pfs"] = round(2 * T * K * N / ms / 1e12, 3)
        ms = timeit(lambda: G.mm_fwd(x, w))
        row[f"fwd_{'split' if split else 'nosplit'}_pfs"] = round(2 * T * K * N / ms / 1e12, 3)
    print(json.dumps(row), flush=True)
    del x, dy, w, out
