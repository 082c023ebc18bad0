"""One GEMM pass, native (variant argv[5]) or hipBLASLt (argv[5] == 'blas'), repeated for rocprofv3 counters.
argv: pass K N iters impl [M]"""
import sys

import torch

sys.path.insert(0, ".")
from paddle2_amd.ops import gemm as G  # noqa: E402

ps, K, N, iters, impl = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
M = int(sys.argv[6]) if len(sys.argv) > 6 else 32768
torch.manual_seed(0)
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(K, N, device="cuda") * 0.02).to(torch.bfloat16)
wt = w.t().contiguous()
dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
out = torch.zeros(K, N, device="cuda")
if impl == "blas":
    fn = {"fwd": lambda: torch.matmul(x, wt.t()), "dgrad": lambda: torch.matmul(dy, w.t()),
          "wgrad": lambda: torch.matmul(x.t(), dy)}[ps]
else:
    G.VARIANT = int(impl)
    fn = {"fwd": lambda: G.mm_fwd(x, w), "dgrad": lambda: G.mm_dgrad(dy, w),
          "wgrad": lambda: G.mm_wgrad(x, dy, out, 1.0), "swiglu": lambda: G.mm_swiglu(x, w)}[ps]
for _ in range(iters):
    fn()
torch.cuda.synchronize()
print("done", ps, K, N, impl)
