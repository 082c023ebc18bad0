"""One flash backward at the Llama-2-7B layer shape (B8 S4096 H32 D128 causal) per mode, for rocprofv3 kernel
tables: split dQ (default) then the fused atomic path."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402

B, S, H, D = 8, 4096, 32, 128
torch.manual_seed(0)
q, k, v, do = (torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16) for _ in range(4))
scale = D ** -0.5
out, lse = T._flash_fwd_native(q, k, v, True, scale)
dq, dk, dv = (torch.empty_like(q) for _ in range(3))
for mode in sys.argv[1:] or ["1", "0"]:
    os.environ["PADDLE2_AMD_FA_DQ_SPLIT"] = mode
    for _ in range(4):
        T._flash_bwd_native(q, k, v, out, do, lse, dq, dk, dv, scale, True)
    torch.cuda.synchronize()
