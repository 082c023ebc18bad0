"""Decode-attention kernel benchmark: vector vs MFMA kernel (csrc/kernels/decode_attn.hip) on the serving shapes.

Effective bandwidth = bytes of K and V the step must read (sum over sequences of len * Hk * D * 2 * 2) / time.
Also checks each kernel against an fp32 reference on a sample of sequences.  Prints one JSON line per case."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from paddle2_amd import serving  # noqa: E402


def run(B, Hq, Hk, D, L, layout, bs=64, iters=50):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    if layout == "paged":
        maxb = (L + bs - 1) // bs
        nblk = B * maxb
        kc = torch.randn(nblk, bs, Hk, D, device=dev, generator=g).bfloat16()
        vc = torch.randn(nblk, bs, Hk, D, device=dev, generator=g).bfloat16()
        bt = torch.randperm(nblk, device=dev, generator=g)[: B * maxb].reshape(B, maxb).int()
    else:
        kc = torch.randn(B, Hk, L, D, device=dev, generator=g).bfloat16()
        vc = torch.randn(B, Hk, L, D, device=dev, generator=g).bfloat16()
        bt = None
    q = torch.randn(B, Hq, D, device=dev, generator=g).bfloat16()
    lens = torch.full((B,), L, dtype=torch.int32, device=dev)
    byts = B * L * Hk * D * 2 * 2
    res = {"B": B, "Hq": Hq, "Hk": Hk, "D": D, "L": L, "layout": layout}
    outs = {}
    for impl, code in (("vec", 1), ("mfma", 2)):
        serving._DECODE_IMPL = code
        f = lambda: serving.decode_attention(q, kc, vc, lens, bt, layout=layout)  # noqa: E731
        try:
            outs[impl] = f()
        except Exception as e:  # noqa: BLE001
            res[impl] = f"error: {e}"
            continue
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / iters
        res[impl + "_us"] = round(us, 2)
        res[impl + "_TBps"] = round(byts / us / 1e6, 3)
    serving._DECODE_IMPL = 0
    # fp32 reference on 2 sequences
    G = Hq // Hk
    err = {}
    for b in (0, B - 1):
        if layout == "paged":
            idx = torch.arange(L, device=dev)
            K = kc[bt[b, idx // bs].long(), idx % bs].float()       # [L, Hk, D]
            V = vc[bt[b, idx // bs].long(), idx % bs].float()
        else:
            K = kc[b].transpose(0, 1).float()
            V = vc[b].transpose(0, 1).float()
        k = K.repeat_interleave(G, 1)
        v = V.repeat_interleave(G, 1)
        s = torch.einsum("hd,lhd->hl", q[b].float(), k) / math.sqrt(D)
        ref = torch.einsum("hl,lhd->hd", torch.softmax(s, -1), v)
        for impl, o in outs.items():
            err[impl] = max(err.get(impl, 0.0), float((o[b].float() - ref).abs().max()))
    res["max_err"] = {k: round(v, 5) for k, v in err.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    cases = [(64, 32, 32, 128, 1088, "paged"), (64, 32, 32, 128, 1088, "bhsd"), (64, 32, 8, 128, 1088, "paged"),
             (16, 32, 32, 128, 4096, "paged"), (8, 64, 8, 128, 8192, "paged"), (1, 32, 32, 128, 8192, "paged"),
             (128, 32, 32, 128, 2048, "paged"), (64, 32, 2, 128, 2048, "paged")]
    for c in cases:
        run(*c)
