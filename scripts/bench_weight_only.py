#!/usr/bin/env python
"""Decode-shape GEMM timing: bf16 weights (hipBLASLt) vs the weight-only int8/int4 HIP kernel.

Timed as HIP-graph replays (GPU time only, as in a captured decode step).  Each call in the graph
uses a different copy of the weights (>= 1 GB of copies per format), so weights stream from HBM as
in a real decode step instead of staying in the MI355X's 256 MB Infinity Cache.
Shapes are Llama-2-7B's per-layer projections (qkv 4096->12288, o 4096->4096, gate_up 4096->22016,
down 11008->4096) at decode batch sizes; one JSON line per (shape, M) with microseconds per call
and the effective weight bandwidth (weight bytes / time).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
from paddle2_amd.nn import quant as Q  # noqa: E402
from paddle2_amd.ops import weight_only as WO  # noqa: E402


def timeit(fn, iters=50):
    """GPU time per call: ``iters`` calls captured in one HIP graph, replayed (no host overhead)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(5):
        g.replay()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / (5 * iters) * 1e3  # us


def main():
    shapes = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}
    for name, (K, N) in shapes.items():
        w = torch.randn(K, N, device="cuda") * 0.02
        wb = w.t().contiguous().to(torch.bfloat16)  # [N, K]
        q8, s8 = Q.weight_quantize(paddle.Tensor._wrap(w), "weight_only_int8")
        q4, s4 = Q.weight_quantize(paddle.Tensor._wrap(w), "weight_only_int4", group_size=128)
        R = max(2, -(-(1 << 30) // (K * N)))  # copies so each format cycles through >= 1 GB
        wbs = [wb.clone() for _ in range(R)]
        q8s = [q8._t.clone() for _ in range(R)]
        q4s = [q4._t.clone() for _ in range(R)]
        del w
        for M in (1, 8, 32, 64):
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            it = [0]

            def rot(seq):
                it[0] = (it[0] + 1) % R
                return seq[it[0]]

            t_bf = timeit(lambda: x @ rot(wbs).t(), iters=2 * R)
            t_8 = timeit(lambda: WO.weight_only_matmul(x, rot(q8s), s8._t, "int8", -1), iters=2 * R)
            t_4 = timeit(lambda: WO.weight_only_matmul(x, rot(q4s), s4._t, "int4", 128), iters=2 * R)
            print(json.dumps({"shape": name, "M": M, "K": K, "N": N, "bf16_us": round(t_bf, 1),
                              "int8_us": round(t_8, 1), "int4_g128_us": round(t_4, 1),
                              "bf16_GBs": round(2 * K * N / t_bf / 1e3, 0),
                              "int8_GBs": round(K * N / t_8 / 1e3, 0), "int4_GBs": round(K * N / 2 / t_4 / 1e3, 0),
                              "speedup_int8": round(t_bf / t_8, 2), "speedup_int4": round(t_bf / t_4, 2)}),
                  flush=True)
        del wbs, q8s, q4s
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
