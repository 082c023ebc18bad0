"""Per-tap / per-row error of the implicit-GEMM 3x3 conv forward (debug helper for gemm7.hip SCHED bit 11)."""
import torch
import torch.nn.functional as F

from paddle2_amd.ops import conv_gemm as CG

dev = "cuda"
for (Nb, H, W, C, Co) in [(2, 8, 8, 64, 64), (1, 4, 4, 64, 64), (2, 14, 14, 128, 64)]:
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(Nb, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    for tap in list(range(9)) + [-1]:
        w = torch.zeros(Co, C, 3, 3, device=dev)
        if tap >= 0:
            w[:, :, tap // 3, tap % 3] = torch.randn(Co, C, device=dev, generator=g) * C ** -0.5
        else:
            w = torch.randn(Co, C, 3, 3, device=dev, generator=g) * (9 * C) ** -0.5
        w = w.to(torch.bfloat16)
        y = CG.Conv3x3Fn.apply(x, w)
        yr = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), None, 1, 1).permute(0, 2, 3, 1)
        err = (y.float() - yr).abs().amax(-1)    # [N, H, W]
        bad = (err > 0.05 * yr.abs().amax().clamp_min(1e-3)).nonzero().tolist()
        print(f"shape {(Nb, H, W, C, Co)} tap {tap}: max err {float(err.max()):.4f} ref max {float(yr.abs().max()):.3f} "
              f"bad pixels {len(bad)} first {bad[:6]}", flush=True)
        # also the raw padded GEMM output vs an emulation of the row-shift GEMM
        buf, gg, Hp, Wp = CG._bordered(x)
        M = Nb * Hp * Wp
        wmat, K = CG._tap_weight(w.permute(0, 2, 3, 1).reshape(Co, 9, C), C)
        yp = CG._conv_gemm(buf, gg, C, Hp, Wp, M, wmat, K, Co, 1).float()
        emu = torch.zeros(M, Co, device=dev)
        for t in range(9):
            s = (t // 3 - 1) * Wp + (t % 3 - 1)
            emu += buf[gg + s:gg + s + M].float() @ wmat[:, t * C:(t + 1) * C].float().t()
        e2 = (yp - emu).abs().amax(-1)
        badr = (e2 > 0.05 * emu.abs().amax().clamp_min(1e-3)).nonzero().flatten().tolist()
        print(f"   padded-grid rows wrong: {len(badr)} of {M}; first {badr[:8]} last {badr[-4:]}", flush=True)
