"""Timing-only ablations of the native GEMM (exp/libgemm_dbg.so built with -DPD_GEMM_DEBUG_VARIANTS):
dgrad layout 32768x4096x4096; variants drop the barrier's vmcnt, the per-sub-phase lgkm syncs, or the
barrier.  Results of the ablated kernels are WRONG by construction; only the time is of interest."""
import ctypes
import json
import sys

import torch

lib = ctypes.CDLL("exp/libgemm_dbg.so")
f = lib.pd_gemm
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long,
              ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int,
              ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
M, N, K = 32768, 4096, 4096
dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
st = torch.cuda.current_stream().cuda_stream


zero = torch.zeros(64, dtype=torch.uint8, device="cuda")


def run(epi):
    rc = f(3, epi, dy.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N, None, 0, zero.data_ptr() if epi == 10 else None,
           M, N, K, 0.0, 0, 8, 0, st)
    assert rc == 0, rc


ref = None
for name, epi in [("base", 0), ("global_load_lds", 10), ("no_dma", 7), ("base", 0), ("global_load_lds", 10),
                  ("same_tile_loads", 9), ("base", 0), ("global_load_lds", 10)]:
    for _ in range(3):
        run(epi)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        run(epi)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    if epi == 0:
        ref = out.clone()
    elif epi == 10:
        assert torch.equal(out, ref), "global_load_lds variant differs"
    print(json.dumps({"variant": name, "ms": round(ms, 4), "TFs": round(2 * M * N * K / ms / 1e9, 1)}), flush=True)
