"""One fp8 GEMM shape, native (gemm8.hip) or hipBLASLt (torch._scaled_mm), run a few times — the target of
rocprofv3 --pmc passes.  argv: impl (native | blas) M N K [sched]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import fp8 as F8  # noqa: E402

impl, M, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
if len(sys.argv) > 5:
    os.environ["PADDLE2_AMD_FP8_SCHED"] = sys.argv[5]
E4 = torch.float8_e4m3fn
a = torch.randn(M, K, device="cuda").to(E4)
b = torch.randn(N, K, device="cuda").to(E4)
one = torch.ones(1, device="cuda")
for _ in range(6):
    if impl == "native":
        F8.mm_native(a, b, one, one, torch.bfloat16)
    else:
        torch._scaled_mm(a, b.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
torch.cuda.synchronize()
