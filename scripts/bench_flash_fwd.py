"""Flash forward: 4-wave (128 query rows / workgroup) vs 8-wave (256 rows) kernel, timed and checked bit for bit.

PADDLE2_AMD_FA_FWD_WAVES is read per call by the launcher.  One JSON line per (case, waves)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
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
    dev = "cuda"
    cases = [("b8_s4096_h32_d128_causal", 8, 4096, 32, 32, 128, True),
             ("b8_s4096_h32_d128_full", 8, 4096, 32, 32, 128, False),
             ("b4_s8192_h32kv8_d128_causal", 4, 8192, 32, 8, 128, True),
             ("b8_s4096_h32_d64_causal", 8, 4096, 32, 32, 64, True),
             ("b2_s1000_h16_d128_causal", 2, 1000, 16, 16, 128, True)]
    for name, B, S, H, HK, D, causal in cases:
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
        k = torch.randn(B, S, HK, D, device=dev, dtype=torch.bfloat16, generator=g)
        v = torch.randn(B, S, HK, D, device=dev, dtype=torch.bfloat16, generator=g)
        flops = 4 * B * H * D * S * S * (0.5 if causal else 1.0)
        outs = {}
        for w, skip in (("4", "0"), ("4", "1"), ("8", "0")):
            os.environ["PADDLE2_AMD_FA_FWD_WAVES"] = w
            os.environ["PADDLE2_AMD_FA_FWD_WAVE_SKIP"] = skip
            fn = lambda: T.flash_attention(q, k, v, causal)  # noqa: E731
            ms = timeit(fn)
            o, lse = fn()[:2]
            outs[(w, skip)] = (o.clone(), lse.clone())
            print(json.dumps({"case": name, "waves": int(w), "wave_skip": int(skip), "fwd_ms": round(ms, 4),
                              "TFs": round(flops / ms / 1e9, 1)}), flush=True)
        base = outs[("4", "0")]
        for key, (o, lse) in outs.items():
            same = torch.equal(base[0], o) and torch.equal(base[1], lse)
            if not same:
                print(json.dumps({"case": name, "variant": key, "bitwise_equal": False}), flush=True)
                sys.exit(1)
        print(json.dumps({"case": name, "bitwise_equal_all": True}), flush=True)


if __name__ == "__main__":
    main()
