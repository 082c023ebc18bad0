"""Flash forward: one row block per wave (RB = 1, two 128-row workgroups per CU) vs two (RB = 2, one 256-row
workgroup per CU, csrc/kernels/flash_fwd2.hip).  PADDLE2_AMD_FA_FWD_RB is read per call by the launcher.  One JSON
line per (case, RB) with the time, TF/s and the max |O - fp32 reference| over a (batch 0, two heads) slice."""
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


def ref_slice(q, k, v, causal, scale):
    hq, hk = q.shape[2], k.shape[2]
    qs = q[:1, :, :2].float().transpose(1, 2)
    heads = [h // (hq // hk) for h in range(2)]
    ks = k[:1, :, heads].float().transpose(1, 2)
    vs = v[:1, :, heads].float().transpose(1, 2)
    s = qs @ ks.transpose(-1, -2) * scale
    if causal:
        sq, sk = q.shape[1], k.shape[1]
        i = torch.arange(sq, device=s.device)[:, None]
        j = torch.arange(sk, device=s.device)[None, :]
        s = s.masked_fill(j > i + (sk - sq), float("-inf"))
    return (torch.softmax(s, -1) @ vs).transpose(1, 2)


def main():
    dev = "cuda"
    cases = [("b8_s4096_h32_d128_causal", 8, 4096, 32, 32, 128, True),
             ("b8_s4096_h32_d128_full", 8, 4096, 32, 32, 128, False),
             ("b4_s8192_h32kv8_d128_causal", 4, 8192, 32, 8, 128, True),
             ("b16_s2048_h64kv8_d128_full", 16, 2048, 64, 8, 128, False),
             ("b2_s1000_h16_d128_causal", 2, 1000, 16, 16, 128, True)]
    rounds = int(os.environ.get("ROUNDS", "2"))
    for name, B, S, H, HK, D, causal in cases:
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, generator=g)
        k = torch.randn(B, S, HK, D, device=dev, dtype=torch.bfloat16, generator=g)
        v = torch.randn(B, S, HK, D, device=dev, dtype=torch.bfloat16, generator=g)
        flops = 4 * B * H * D * S * S * (0.5 if causal else 1.0)
        scale = D ** -0.5
        ro = ref_slice(q, k, v, causal, scale)
        for rnd in range(rounds):
            for rb, mf in (("1", "32"), ("2", "32"), ("1", "16")):
                os.environ["PADDLE2_AMD_FA_FWD_RB"] = rb
                os.environ["PADDLE2_AMD_FA_FWD_MFMA"] = mf
                fn = lambda: T._flash_fwd_native(q, k, v, causal, scale)  # noqa: E731
                ms = timeit(fn)
                o = fn()[0]
                err = (o[:1, :, :2].float() - ro).abs().max().item()
                print(json.dumps({"case": name, "rb": int(rb), "mfma": int(mf), "round": rnd, "fwd_ms": round(ms, 4),
                                  "TFs": round(flops / ms / 1e9, 1), "max_abs_err": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
