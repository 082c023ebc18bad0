"""Grouped-GEMM MoE FFN (ops/moe.py, one native launch per projection) vs the per-expert hipBLASLt loop
(host-synced counts) on a Mixtral-like layer: 16384 tokens, top-2 of 8 experts, H 4096, F 14336, bf16.
Prints one JSON line per variant (forward; and forward+backward of the expert FFN)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle2_amd.ops import moe as MOE  # noqa: E402
from paddle2_amd.ops import torch_ops as T  # noqa: E402

dev = "cuda"
Tn, H, F, E, k = 16384, 4096, 14336, 8, 2
torch.manual_seed(0)
x = torch.randn(Tn, H, device=dev, dtype=torch.bfloat16)
gw = torch.randn(H, E, device=dev) * 0.02
w1 = (torch.randn(E, H, 2 * F, device=dev) * 0.02).to(torch.bfloat16)
w2 = (torch.randn(E, F, H, device=dev) * 0.02).to(torch.bfloat16)
flops = 2.0 * Tn * k * (H * 2 * F + F * H)


def loop_ffn(x2):
    tok, gate, goff = MOE.route_topk(x2.float() @ gw, k)
    xs = x2.index_select(0, tok)
    o = goff.tolist()
    ys = torch.empty(xs.shape[0], H, dtype=x2.dtype, device=dev)
    for e in range(E):
        if o[e + 1] > o[e]:
            h = T.swiglu(xs[o[e]:o[e + 1]] @ w1[e])
            ys[o[e]:o[e + 1]] = h @ w2[e]
    out = torch.zeros(Tn, H, dtype=torch.float32, device=dev).index_add(0, tok, ys.float() * gate[:, None])
    return out.to(x2.dtype)


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


ref = loop_ffn(x)
got = MOE.moe_ffn(x, gw, w1, w2, k)
err = float((got.float() - ref.float()).abs().max() / ref.float().abs().max())
for name, fn in (("grouped_native", lambda: MOE.moe_ffn(x, gw, w1, w2, k)), ("per_expert_hipblaslt", lambda: loop_ffn(x))):
    t = timeit(fn)
    print(json.dumps({"variant": name, "pass": "fwd", "ms": round(t * 1e3, 3), "expert_TFs": round(flops / t / 1e12, 1),
                      "max_rel_err_vs_loop": round(err, 5)}), flush=True)
xg = x.clone().requires_grad_()
w1g, w2g = w1.clone().requires_grad_(), w2.clone().requires_grad_()


def fb():
    y = MOE.moe_ffn(xg, gw, w1g, w2g, k)
    y.backward(torch.ones_like(y))


t = timeit(fb, 5)
print(json.dumps({"variant": "grouped_native", "pass": "fwd+bwd", "ms": round(t * 1e3, 3),
                  "expert_TFs": round(3 * flops / t / 1e12, 1)}), flush=True)
