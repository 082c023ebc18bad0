"""Flash backward at the Llama-2-7B shape (B8 S4096 H32 D128 causal, bf16): the 8-wave kernel's wave-role options
(PADDLE2_AMD_FA_BWD_OPT, read per launch: bit 0 = waves 4-7 at s_setprio 1, bit 1 = dQ slices on waves 4-7).
argv[1] (optional) = comma-separated PADDLE2_AMD_FA_BWD_ORDER values to A/B instead ("heavy" = the default order).
One JSON line per (option, order, round): time, TF/s, and the max |difference| of dQ / dK / dV against option 0."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402


def timeit(fn, iters=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


def main():
    B, S, H, D = 8, 4096, 32, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(4))
    scale = D ** -0.5
    out, lse = T._flash_fwd_native(q, k, v, True, scale)
    fl = 2.5 * 4 * B * H * D * S * S * 0.5
    ref = None
    orders = sys.argv[1].split(",") if len(sys.argv) > 1 else None   # e.g. "heavy,pair": PADDLE2_AMD_FA_BWD_ORDER A/B
    for rnd in range(2):
        for opt in ((0,) if orders else (0, 1, 2, 3)):
            for order in (orders or ["heavy"]):
                os.environ["PADDLE2_AMD_FA_BWD_OPT"] = str(opt)
                os.environ["PADDLE2_AMD_FA_BWD_ORDER"] = order
                grads = [torch.empty_like(q) for _ in range(3)]
                fn = lambda: T._flash_bwd_native(q, k, v, out, do, lse, *grads, scale, True)  # noqa: E731
                ms = timeit(fn)
                fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = [t.clone() for t in grads]
                diff = [float((a.float() - b.float()).abs().max()) for a, b in zip(grads, ref)]
                print(json.dumps({"opt": opt, "order": order, "round": rnd, "bwd_ms": round(ms, 4), "TFs": round(fl / ms / 1e9, 1),
                                  "max_diff_dq_dk_dv": [round(x, 6) for x in diff]}), flush=True)
    os.environ.pop("PADDLE2_AMD_FA_BWD_OPT", None)
    os.environ.pop("PADDLE2_AMD_FA_BWD_ORDER", None)


if __name__ == "__main__":
    main()
