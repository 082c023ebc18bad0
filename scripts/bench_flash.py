"""Flash-attention kernel timings on one MI355X: dense causal vs. varlen vs. FlashMask (document mask).

python scripts/bench_flash.py  -> one JSON line per case (fwd / bwd ms and effective TF/s over the unmasked work).
"""
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
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def run(name, fwd, inputs, flops):
    def f():
        return fwd()

    tf = timeit(f)
    out = f()
    go = torch.randn_like(out)

    def fb():
        for t in inputs:
            t.grad = None
        fwd().backward(go)

    tfb = timeit(fb)
    tb = tfb - tf
    print(json.dumps({"case": name, "fwd_ms": round(tf, 3), "bwd_ms": round(tb, 3),
                      "fwd_tflops": round(flops / tf / 1e9, 1), "bwd_tflops": round(2.5 * flops / tb / 1e9, 1)}),
          flush=True)


def main():
    dev = "cuda"
    B, S, H, D = 2, 4096, 32, 128
    q = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    causal_flops = 4 * B * H * D * S * S / 2
    run("dense_causal_b2_s4096", lambda: T.flash_attention(q, k, v, True)[0], (q, k, v), causal_flops)

    # 8 documents of 512 tokens per sequence: varlen over 16 packed sequences, and the same as a FlashMask
    doc = 512
    cu = torch.arange(0, B * S + 1, doc, dtype=torch.int32, device=dev)
    qp, kp, vp = (t.detach().reshape(B * S, H, D).requires_grad_(True) for t in (q, k, v))
    doc_flops = 4 * (B * S // doc) * H * D * doc * doc / 2
    run("varlen_causal_16x512", lambda: T.flash_attention_varlen(qp, kp, vp, cu, cu, doc, doc, True)[0],
        (qp, kp, vp), doc_flops)
    j = torch.arange(S, device=dev)
    idx = ((j // doc + 1) * doc).to(torch.int32).view(1, 1, S, 1).expand(B, 1, S, 1).contiguous()
    run("flashmask_causal_doc512", lambda: T.flash_attention_mask(q, k, v, idx, True)[0], (q, k, v), doc_flops)
    # sliding window 1024 (causal): ~1/4 of the causal work survives
    idx_w = (j + 1025).clamp(max=S).to(torch.int32).view(1, 1, S, 1).expand(B, 1, S, 1).contiguous()
    win_flops = 4 * B * H * D * (S * 1024 - 1024 * 1024 / 2)
    run("flashmask_causal_window1024", lambda: T.flash_attention_mask(q, k, v, idx_w, True)[0], (q, k, v),
        win_flops)


if __name__ == "__main__":
    main()
