"""Minimal driver for rocprofv3 PMC passes on the flash kernels: dense causal B2 S4096 H32 D128."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402

B, S, H, D = 2, 4096, 32, 128
q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
go = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    o, _ = T.flash_attention(q, k, v, True)
    o.backward(go)
torch.cuda.synchronize()
print("done")
