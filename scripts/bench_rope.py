"""RoPE forward bandwidth at the Llama-2-7B q shape (B8 S4096 H32 D128 bf16, fp32 cos/sin tables), with a check
against the fp32 reference rotation."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402

B, S, H, D = 8, 4096, 32, 128
x = torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16)
cos, sin = T.rope_tables(S, D, interleaved=False, device="cuda")


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


ms = timeit(lambda: T._rope_apply(x, cos, sin, None, 0, False, False))
y = T._rope_apply(x, cos, sin, None, 0, False, False).float()
xf = x.float()
c, s_ = cos[:, None, :], sin[:, None, :]
rot = torch.cat([-xf[..., D // 2:], xf[..., :D // 2]], -1)
ref = xf * c + rot * s_
err = (y - ref).abs().max().item()
print(json.dumps({"rope_ms": round(ms, 4), "TBs": round(2 * x.numel() * 2 / ms / 1e9, 2), "max_abs_err": err}),
      flush=True)
