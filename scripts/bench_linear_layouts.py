"""Layout-aware Linear node vs plain hipBLASLt layouts on the Llama-2-7B training GEMMs (M = 8 x 4096).

For each projection: fwd ms and bwd (dX + dW) ms with PADDLE2_AMD_LINEAR_LAYOUT off / all / auto.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    M = 32768
    x16 = torch.randn(4096 * 8, 4096, device="cuda", dtype=torch.bfloat16)
    tr = t(lambda: T.transpose2d(x16))
    print(json.dumps({"transpose_32768x4096_ms": round(tr, 3), "GB_per_s": round(2 * x16.numel() * 2 / tr / 1e6, 1)}))
    shapes = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096),
              "lm_head": (4096, 32000)}
    for name, (K, N) in shapes.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        w = (torch.randn(K, N, device="cuda", dtype=torch.bfloat16) * 0.02).requires_grad_(True)
        go = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        row = {"gemm": name}
        for mode in ("off", "all", "auto"):
            T._LINEAR_LAYOUT = mode
            f = t(lambda: T.linear(x, w))

            def fb():
                x.grad = None
                w.grad = None
                T.linear(x, w).backward(go)

            row[mode] = {"fwd": round(f, 3), "bwd": round(t(fb) - f, 3)}
        print(json.dumps(row), flush=True)
        del x, w, go


if __name__ == "__main__":
    main()
