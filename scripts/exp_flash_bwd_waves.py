"""Flash backward at the Llama-2-7B shape (B8 S4096 H32 D128 causal, dense atomic dQ): the 8-wave (256-key,
one workgroup per CU) vs the 4-wave (128-key, two per CU) kernel, interleaved rounds in one process, plus the
dQ / dK / dV difference between them and against an fp32 SDPA reference on a small slice."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import torch_ops as T  # noqa: E402

B, S, H, D = 8, 4096, 32, 128
torch.manual_seed(0)
q, k, v = (torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16) for _ in range(3))
do = torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16)
scale = D ** -0.5
out, lse = T._flash_fwd_native(q, k, v, True, scale)
flops = 2.5 * 4 * B * H * S * S * D / 2
res = {}
grads = {}
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for w in ("8", "4"):
        os.environ["PADDLE2_AMD_FA_BWD_WAVES"] = w
        dq, dk, dv = (torch.empty_like(q) for _ in range(3))

        def bwd():
            T._flash_bwd_native(q, k, v, out, do, lse, dq, dk, dv, scale, True)

        for _ in range(2):
            bwd()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(8):
            bwd()
        e.record()
        torch.cuda.synchronize()
        res.setdefault(w, []).append(s.elapsed_time(e) / 8)
        grads[w] = (dq, dk, dv)
for w, t in res.items():
    print(json.dumps({"waves": int(w), "bwd_ms_min": round(min(t), 3), "bwd_ms_all": [round(x, 3) for x in t],
                      "bwd_TFs": round(flops / min(t) / 1e9, 1)}), flush=True)
rel = {n: ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()
       for n, a, b in zip(("dq", "dk", "dv"), grads["4"], grads["8"])}
# fp32 reference on batch 0, heads 0-1, first 1024 tokens (the kernel ran causal on the full 4096; the first 1024
# query rows only see keys < 1024, so the slice's dq / dk / dv ... dk/dv of keys < 1024 also get rows >= 1024:
# compare dq only on the slice)
qs, ks_, vs = (t[:1, :1024, :2].float().transpose(1, 2).requires_grad_(True) for t in (q, k, v))
o = torch.nn.functional.scaled_dot_product_attention(qs, ks_, vs, is_causal=True, scale=scale)
o.backward(do[:1, :1024, :2].float().transpose(1, 2))
ref_dq = qs.grad.transpose(1, 2)
err = {w: ((g[0][:1, :1024, :2].float() - ref_dq).abs().max() / ref_dq.abs().max()).item() for w, g in grads.items()}
print(json.dumps({"rel_diff_4_vs_8": rel, "dq_rel_err_vs_fp32": err}), flush=True)
