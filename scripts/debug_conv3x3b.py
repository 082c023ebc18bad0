"""Per-K-tile check of the implicit-GEMM conv kernel: one-hot K-tile weights, output vs an emulation."""
import torch

from paddle2_amd.ops import conv_gemm as CG

dev = "cuda"
for (Nb, H, W, C, Co) in [(2, 8, 8, 64, 64), (2, 8, 8, 128, 64), (8, 30, 30, 64, 256)]:
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(Nb, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    buf, gg, Hp, Wp = CG._bordered(x)
    M = Nb * Hp * Wp
    K9 = 9 * C
    Kp = K9 if (K9 // 64) % 2 == 0 else K9 + 64
    for kt in range(Kp // 64):
        wmat = torch.zeros(Co, Kp, device=dev, dtype=torch.bfloat16)
        wmat[:, kt * 64:(kt + 1) * 64] = (torch.randn(Co, 64, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        yp = CG._conv_gemm(buf, gg, C, Hp, Wp, M, wmat, Kp, Co, 1).float()
        tap, kc = divmod(kt * 64, C)
        if tap < 9:
            s = (tap // 3 - 1) * Wp + (tap % 3 - 1)
            a = buf[gg + s:gg + s + M, kc:kc + 64].float()
        else:
            a = buf[gg:gg + M, 0:64].float()
        emu = a @ wmat[:, kt * 64:(kt + 1) * 64].float().t()
        rel = float((yp - emu).norm() / emu.norm().clamp_min(1e-9))
        # which A rows / which weight columns would explain the output
        best = None
        for s2 in range(-3 * Wp, 3 * Wp + 1):
            for c2 in range(0, C, 64):
                a2 = buf[gg + s2:gg + s2 + M, c2:c2 + 64].float() if 0 <= gg + s2 and gg + s2 + M <= buf.shape[0] else None
                if a2 is None:
                    continue
                r2 = float((yp - a2 @ wmat[:, kt * 64:(kt + 1) * 64].float().t()).norm() / yp.norm().clamp_min(1e-9))
                if best is None or r2 < best[0]:
                    best = (r2, s2, c2)
        print(f"C={C} M={M} kt={kt} tap={tap} kc={kc}: rel err {rel:.4f} |y|/|emu| "
              f"{float(yp.norm() / emu.norm().clamp_min(1e-9)):.3f}  best-fit shift/chan {best}", flush=True)
