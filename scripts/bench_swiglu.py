"""SwiGLU forward / backward bandwidth at the Llama-2-7B MLP shape (32768 x 11008, bf16, gate | up halves of one
[M, 2H] tensor as the step uses them)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402

M, H = 32768, 11008
gu = torch.randn(M, 2 * H, device="cuda").to(torch.bfloat16)
x, y = gu[:, :H], gu[:, H:]
dout = torch.randn(M, H, device="cuda").to(torch.bfloat16)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


gr = gu.detach().requires_grad_()
fwd_ms = timeit(lambda: T.swiglu(gu))
out = T.swiglu(gr)
bwd_ms = timeit(lambda: torch.autograd.grad(out, (gr,), dout, retain_graph=True))
ref = torch.nn.functional.silu(x.float()) * y.float()
err = (T.swiglu(gu).float() - ref).abs().max().item()
fb = 3 * M * H * 2
bb = 5 * M * H * 2
print(json.dumps({"fwd_ms": round(fwd_ms, 4), "fwd_TBs": round(fb / fwd_ms / 1e9, 2), "bwd_ms": round(bwd_ms, 4),
                  "bwd_TBs": round(bb / bwd_ms / 1e9, 2), "max_abs_err": err}), flush=True)
