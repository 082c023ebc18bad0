"""Weight-gradient GEMMs with a long token reduction (K = 32768): plain hipBLASLt vs manual split-K
(batched GEMM over token chunks + sum of partials), for the o_proj and down_proj shapes of Llama-2-7B b=8."""
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


M = 32768
for name, (K, N) in {"o": (4096, 4096), "down": (11008, 4096), "qkv": (4096, 12288)}.items():
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    ref = (x.float().t() @ dy.float())
    fl = 2.0 * M * K * N
    row = {"gemm": name}
    row["nt"] = t(lambda: x.t() @ dy)
    xt, dyt = T.transpose2d(x), T.transpose2d(dy)
    row["tn_pre"] = t(lambda: xt @ dyt.t())
    for s in (2, 3, 4, 6, 8):
        if M % s:
            continue
        xs, ds = x.view(s, M // s, K), dy.view(s, M // s, N)
        row[f"split{s}_bf16"] = t(lambda: torch.bmm(xs.transpose(1, 2), ds).sum(0))
        try:
            row[f"split{s}_f32"] = t(lambda: torch.bmm(xs.transpose(1, 2), ds, out_dtype=torch.float32).sum(0))
        except Exception as e:  # noqa: BLE001
            row["f32_err"] = str(e)[:80]
        out = torch.bmm(xs.transpose(1, 2), ds).float().sum(0)
        row[f"split{s}_relerr"] = float((out - ref).norm() / ref.norm())
    row = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in row.items()}
    row["nt_PF"] = round(fl / row["nt"] / 1e12, 3)
    best = min((v, k) for k, v in row.items() if k.startswith("split") and k.endswith(("bf16", "f32")))
    row["best"] = [best[1], round(fl / best[0] / 1e12, 3)]
    print(json.dumps(row), flush=True)
    del x, dy, ref
