"""Flash-attention backward at the Llama-2-7B bench shape (B8 S4096 H32 D128 causal): time + dQ/dK/dV check
against a second run (and, with PADDLE2_AMD_FA_DQ_ATOMIC set differently in two processes, across modes)."""
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


def bwd():
    T._flash_bwd_native(q, k, v, out, do, lse, dq, dk, dv, scale, True)


for _ in range(3):
    bwd()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    bwd()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 10
flops = 2.5 * 4 * B * H * S * S * D / 2
path = os.environ.get("FA_DUMP")
if path:
    torch.save({"dq": dq.cpu(), "dk": dk.cpu(), "dv": dv.cpu()}, path)
ref = os.environ.get("FA_REF")
diff = None
if ref:
    r = torch.load(ref, weights_only=True)
    diff = {n: ((t.float().cpu() - r[n].float()).abs().max() / r[n].float().abs().max()).item()
            for n, t in (("dq", dq), ("dk", dk), ("dv", dv))}
print(json.dumps({"atomic": os.environ.get("PADDLE2_AMD_FA_DQ_ATOMIC", "0"), "bwd_ms": round(ms, 3),
                  "bwd_TFs": round(flops / ms / 1e9, 1), "rel_diff_vs_ref": diff}), flush=True)
