"""Timing-only ablations of the v4 native GEMM (exp/libgemm_dbg.so = csrc/kernels/gemm.hip built with
-DPD_GEMM_DEBUG_VARIANTS), dgrad layout (both operands K-major), M=32768 N=4096, K from argv (default 4096).
Ablated kernels give WRONG results by construction; only their time matters.  Interleaved rounds, one process."""
import ctypes
import json
import sys

import torch

lib = ctypes.CDLL("exp/libgemm_dbg.so")
f = lib.pd_gemm
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long,
              ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int,
              ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
              ctypes.c_long, ctypes.c_void_p]
M, N = 32768, 4096
K = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
st = torch.cuda.current_stream().cuda_stream
VARS = [("v4", 0, 4), ("no_vmcnt", 11, 4), ("no_dma", 12, 4), ("no_barrier", 13, 4), ("no_lds_reads", 14, 4),
        ("same_tile", 15, 4), ("A_sc0sc1", 16, 4), ("B_sc0sc1", 17, 4), ("dma_burst", 18, 4), ("half_dma", 19, 4),
        ("v5_regstage", 0, 5)]


def run(epi, variant):
    rc = f(3, epi, dy.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N, None, 0, None, M, N, K, 0.0, 0, 8, variant,
           None, 0, st)
    assert rc == 0, rc


res = {}
for rnd in range(3):
    for name, epi, var in VARS:
        for _ in range(2):
            run(epi, var)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            run(epi, var)
        e.record()
        torch.cuda.synchronize()
        res.setdefault(name, []).append(s.elapsed_time(e) / 10)
for name, ts in res.items():
    print(json.dumps({"K": K, "variant": name, "ms": [round(t, 3) for t in ts],
                      "TFs_best": round(2 * M * N * K / min(ts) / 1e9, 1)}), flush=True)
