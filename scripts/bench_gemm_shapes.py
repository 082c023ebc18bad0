"""hipBLASLt (torch.matmul) throughput on the exact Llama-2-7B training GEMMs at M = 8 x 4096 tokens.

fwd  Y[M,N]  = X[M,K] @ W[K,N]        (weights stored [in, out], Paddle layout)
dX   dX[M,K] = dY[M,N] @ W[K,N]^T
dW   dW[K,N] = X[M,K]^T @ dY[M,N]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    if len(sys.argv) > 1 and sys.argv[1] == "tuned":
        from paddle2_amd.incubate import autotune

        autotune.enable_gemm_autotune(tuning=False)
    M = int(os.environ.get("GEMM_M", 32768))
    shapes = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096),
              "lm_head": (4096, 32000)}
    dev = "cuda"
    tot_ms, tot_fl = 0.0, 0.0
    for name, (K, N) in shapes.items():
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(K, N, device=dev, dtype=torch.bfloat16) * 0.02
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * K * N
        for kind, fn in (("fwd", lambda: x @ w), ("dX", lambda: dy @ w.t()), ("dW", lambda: x.t() @ dy)):
            ms = t(fn)
            tot_ms += ms
            tot_fl += fl
            print(json.dumps({"gemm": name, "kind": kind, "M": M, "K": K, "N": N, "ms": round(ms, 3),
                              "tflops": round(fl / ms / 1e9, 1)}), flush=True)
        del x, w, dy
    print(json.dumps({"total_ms_per_layer_set": round(tot_ms, 2), "avg_tflops": round(tot_fl / tot_ms / 1e9, 1)}))


if __name__ == "__main__":
    main()
