"""Flash backward dQ-path comparison at the Llama-2-7B shape (B8 S4096 H32 D128 causal): split dQ (dS stored,
dq_gemm_kernel; the default), fused atomic dQ, per-key-block slabs (deterministic fused), and the bench-only
ablations of the fused kernel (dQ computed but not stored; no dQ phase at all)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402

B, S, H, D = 8, 4096, 32, 128
torch.manual_seed(0)
q, k, v = (torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16) for _ in range(3))
do = torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16)
scale = D ** -0.5
out, lse = T._flash_fwd_native(q, k, v, True, scale)
dq, dk, dv = (torch.empty_like(q) for _ in range(3))
flops = 2.5 * 4 * B * H * S * S * D / 2
KEYS = ("PADDLE2_AMD_FA_DQ_ATOMIC", "PADDLE2_AMD_FA_DEBUG_DQ_ABLATE", "PADDLE2_AMD_FA_DQ_SPLIT",
        "PADDLE2_AMD_FA_BWD_ORDER")
SPLIT = {"PADDLE2_AMD_FA_DQ_SPLIT": "1"}
for name, env in (("split", SPLIT), ("atomic", {"PADDLE2_AMD_FA_DQ_SPLIT": "0"}),
                  ("split_no_ds_store", {**SPLIT, "PADDLE2_AMD_FA_DEBUG_DQ_ABLATE": "4"}),
                  ("split_no_ds", {**SPLIT, "PADDLE2_AMD_FA_DEBUG_DQ_ABLATE": "5"}),
                  ("split_pair", {**SPLIT, "PADDLE2_AMD_FA_BWD_ORDER": "pair"}),
                  ("atomic_pair", {"PADDLE2_AMD_FA_DQ_SPLIT": "0", "PADDLE2_AMD_FA_BWD_ORDER": "pair"}),
                  ("slabs", {"PADDLE2_AMD_FA_DQ_SPLIT": "0", "PADDLE2_AMD_FA_DQ_ATOMIC": "0"}),
                  ("no_dq_store", {"PADDLE2_AMD_FA_DQ_SPLIT": "0", "PADDLE2_AMD_FA_DEBUG_DQ_ABLATE": "2"}),
                  ("no_dq_phase", {"PADDLE2_AMD_FA_DQ_SPLIT": "0", "PADDLE2_AMD_FA_DEBUG_DQ_ABLATE": "3"})):
    for kk in KEYS:
        os.environ.pop(kk, None)
    os.environ.update(env)

    def bwd():
        T._flash_bwd_native(q, k, v, out, do, lse, dq, dk, dv, scale, True)

    for _ in range(3):
        bwd()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            bwd()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / 5)
    print(json.dumps({"mode": name, "bwd_ms": round(best, 3), "bwd_TFs": round(flops / best / 1e9, 1)}), flush=True)
