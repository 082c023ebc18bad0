"""Fused masked softmax (csrc/kernels/softmax_mask.hip) vs the unfused PyTorch-ROCm sequence
(masked_fill / add + softmax): forward and backward time and effective HBM bandwidth on one MI355X."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    rows = []
    for causal, (B, H, S) in [(True, (4, 32, 2048)), (True, (1, 32, 4096)), (False, (4, 32, 2048)),
                              (False, (2, 16, 8192))]:
        Sq = S if causal else 512
        x = torch.randn(B, H, Sq, S, device="cuda", dtype=torch.bfloat16)
        m = torch.where(torch.rand(B, 1, Sq, S, device="cuda") > 0.2, 0.0, -1e4).to(torch.bfloat16)
        dy = torch.randn_like(x)
        keep = torch.ones(S, S, dtype=torch.bool, device="cuda").tril()

        def unfused():
            if causal:
                return torch.softmax(x.masked_fill(~keep, float("-inf")), -1)
            return torch.softmax(x + m, -1)

        fused = lambda: T.softmax_mask(x, None if causal else m, causal=causal)  # noqa: E731
        y = fused()
        t_f = timeit(fused)
        t_u = timeit(unfused)
        t_fb = timeit(lambda: torch.ops.aten._softmax_backward_data(dy, y, -1, torch.bfloat16))
        from paddle2_amd.ops import _native as N

        dx = torch.empty_like(x)
        t_b = timeit(lambda: N.native().softmax_mask_bwd(N.DT_CODE[x.dtype], y.data_ptr(), dy.data_ptr(),
                                                         dx.data_ptr(), y.numel() // S, S, N.stream()))
        nbytes = x.numel() * 2 * (2 if causal else 3)
        rows.append({"causal": causal, "shape": [B, H, Sq, S], "fwd_fused_ms": round(t_f, 4),
                     "fwd_unfused_ms": round(t_u, 4), "fwd_fused_TBps": round(nbytes / t_f / 1e9, 2),
                     "bwd_fused_ms": round(t_b, 4), "bwd_torch_ms": round(t_fb, 4),
                     "bwd_fused_TBps": round(x.numel() * 6 / t_b / 1e9, 2)})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
