"""fp8 cast + transpose + amax at the GPT-3 13B fp8-step shapes: time per call (the step runs 480 of them)."""
import json

import torch

from paddle2_amd.ops import fp8 as F8

for R, C, fmt in ((4096, 5120, F8.E4M3), (4096, 15360, F8.E5M2), (4096, 20480, F8.E4M3), (5120, 15360, F8.E4M3),
                  (20480, 5120, F8.E4M3)):
    x = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
    meta = F8.FP8TensorMeta(fmt, device=torch.device("cuda"))
    for keep in (True, False):
        for _ in range(3):
            F8.cast(x, meta, transpose=True, keep_rowmajor=keep)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            F8.cast(x, meta, transpose=True, keep_rowmajor=keep)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        byts = R * C * 2 + R * C * (2 if keep else 1)
        print(json.dumps({"R": R, "C": C, "fmt": str(fmt)[-6:], "rowmajor_too": keep, "us": round(us, 1),
                          "TBs": round(byts / us / 1e6, 2)}), flush=True)
