"""Round-5 experiment: where the TN GEMM's per-tile overhead goes (M = 32768, v7 spread schedule).

* K scaling at N = 12288: ms per tile-K-tile vs K (intercept = fixed per-tile cost);
* base vs the store-ablated build (SCHED bit 8192: accumulators kept live, nothing stored);
* XCD-phase stagger (bit 16384, PD_GEMM_XCD_DELAY units of ~8k cycles per XCD index).
Variants interleaved round by round in one process (cdna guide §5.4 rule 24); one JSON line per measurement."""
import json
import os
import sys

import torch

from paddle2_amd.ops import _native as N
from paddle2_amd.ops import gemm as G

M = 32768
BASE = 64 + 384
CASES = [("kscale", 2048, 12288), ("kscale", 4096, 12288), ("kscale", 8192, 12288), ("kscale", 16384, 12288),
         ("o_fwd", 4096, 4096), ("down_dgrad", 4096, 11008), ("gate_up_dgrad", 22016, 4096)]
VARS = [("base", BASE, None), ("nostore", BASE + 8192, None)] + [
    (f"xdelay{d}", BASE + 16384, d) for d in (1, 2, 4)]
ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
ITERS = 8

g = torch.Generator(device="cuda").manual_seed(0)
res = {}
for name, K, Nn in CASES:
    a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(Nn, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
    flop = 2.0 * M * K * Nn
    for r in range(ROUNDS):
        for vn, v, d in VARS:
            if d is not None:
                os.environ["PD_GEMM_XCD_DELAY"] = str(d)
            G.VARIANT = v

            def f():
                G._launch(3, 0, a, K, b, K, c, Nn, None, 0, None, M, Nn, K)

            for _ in range(2):
                f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(ITERS):
                f()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / ITERS
            res.setdefault((name, K, Nn, vn), []).append(ms)
    G.VARIANT = None
    for (n2, K2, N2, vn), v in res.items():
        if n2 == name and K2 == K and N2 == Nn:
            print(json.dumps(dict(case=name, K=K, N=Nn, var=vn, ms_min=round(min(v), 4),
                                  ms_med=round(sorted(v)[len(v) // 2], 4), TFs=round(flop / min(v) / 1e9, 1),
                                  tiles_per_cu=round((M // 256) * ((Nn + 255) // 256) / 256, 2))), flush=True)
