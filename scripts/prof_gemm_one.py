"""Run one native GEMM pass repeatedly (for rocprofv3 counter collection).  argv: pass K N [iters] [M]
(pass: fwd | dgrad | wgrad (beta 1, accumulate) | wgrad0 (beta 0, the step's first write) | swiglu)"""
import sys

import torch

sys.path.insert(0, ".")
from paddle2_amd.ops import gemm as G  # noqa: E402

ps, K, N = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
M = int(sys.argv[5]) if len(sys.argv) > 5 else 32768
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(K, N, device="cuda") * 0.02).to(torch.bfloat16)
dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
out = torch.zeros(K, N, device="cuda")
fn = {"fwd": lambda: G.mm_fwd(x, w), "dgrad": lambda: G.mm_dgrad(dy, w),
      "wgrad": lambda: G.mm_wgrad(x, dy, out, 1.0), "wgrad0": lambda: G.mm_wgrad(x, dy, out, 0.0),
      "swiglu": lambda: G.mm_swiglu(x, w)}[ps]
for _ in range(iters):
    fn()
torch.cuda.synchronize()
print("done", ps, K, N)
