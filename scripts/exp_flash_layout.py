"""Flash attention at the Llama-2-7B shape (B8 S4096 H32 D128 causal, bf16): does the operand layout matter?

The training step hands the kernels q / k as contiguous rotated copies and v as a token-strided view of the fused
qkv projection output (row stride (Hq + 2 Hk) * D = 12288 elements), while the isolated benches use contiguous
[B, S, H, D] tensors.  One JSON line per (layout, pass): forward / backward time and TF/s, best of 3 x 10 launches.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
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


def main():
    B, S, H, D = 8, 4096, 32, 128
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, S, 3 * H, D, device=dev, dtype=torch.bfloat16, generator=g)
    qs, ks, vs = qkv[:, :, :H], qkv[:, :, H:2 * H], qkv[:, :, 2 * H:]
    qc, kc, vc = qs.contiguous(), ks.contiguous(), vs.contiguous()
    scale = D ** -0.5
    fl = 4 * B * H * D * S * S * 0.5
    layouts = {"contig": (qc, kc, vc), "v_strided": (qc, kc, vs), "all_strided": (qs, ks, vs)}
    do = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
    for rnd in range(2):
        for name, (q, k, v) in layouts.items():
            ms = timeit(lambda: T._flash_fwd_native(q, k, v, True, scale))
            out, lse = T._flash_fwd_native(q, k, v, True, scale)
            print(json.dumps({"layout": name, "pass": "fwd", "round": rnd, "ms": round(ms, 4),
                              "TFs": round(fl / ms / 1e9, 1)}), flush=True)
            dq = torch.empty_like(qc)
            dk = torch.empty_like(kc)
            dv = torch.empty_like(vc)
            msb = timeit(lambda: T._flash_bwd_native(q, k, v, out, do, lse, dq, dk, dv, scale, True), iters=5)
            print(json.dumps({"layout": name, "pass": "bwd", "round": rnd, "ms": round(msb, 4),
                              "TFs": round(2.5 * fl / msb / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
