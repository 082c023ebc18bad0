"""Characterise v7 errors: per 16x16 output block max error vs fp32 reference, single-tile shapes."""
import torch

from paddle2_amd.ops import gemm as G

torch.manual_seed(0)
for (M, N, K) in [(256, 256, 128), (256, 256, 256), (256, 256, 4096), (512, 768, 128)]:
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    for v in (6, 7, 8):
        G.VARIANT = v
        out = G.mm_dgrad(x, w.contiguous())   # dx = x @ w^T with w [N, K]: layout AK|BK
        torch.cuda.synchronize()
        err = (out.float() - ref).abs()
        blk = err.reshape(M // 16, 16, N // 16, 16).amax(dim=(1, 3))
        bad = (blk > 0.05).nonzero().tolist()
        print(f"M{M} N{N} K{K} v{v}: maxerr {err.max().item():.4f} bad16x16 {len(bad)} / {blk.numel()}", flush=True)
        if bad and M == 256:
            rows = sorted(set(b[0] for b in bad)); cols = sorted(set(b[1] for b in bad))
            print("   bad row-blocks", rows, "col-blocks", cols, flush=True)
            # is the error a missing / doubled K-chunk? compare with partial-K references
            e = (out.float() - ref)
            for kc in range(0, K, 32):
                part = x[:, kc:kc + 32].float() @ w[:, kc:kc + 32].float().t()
                r = ((e + part).abs().amax() < 0.05).item(), ((e - part).abs().amax() < 0.05).item()
                if any(r):
                    print(f"   error == {'-' if r[0] else '+'} K-chunk {kc}", flush=True)
