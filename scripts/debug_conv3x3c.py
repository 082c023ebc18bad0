"""gemm_conv as a plain GEMM (taps = 1, no shifts) and with sign -1: which K-tiles contribute."""
import math

import torch

from paddle2_amd.ops import _native as N
from paddle2_amd.ops import conv_gemm as CG

dev = "cuda"


def run(A, lda, a_lo, a_hi, wmat, M, Nn, K, taps, kw, pitch, pad_h, pad_w, sign, kpb):
    out = torch.empty(M, Nn, dtype=torch.bfloat16, device=dev)
    rc = N.native().gemm_conv(A, lda, a_lo, a_hi, wmat.data_ptr(), K, out.data_ptr(), Nn, M, Nn, K, taps, kw, pitch,
                              pad_h, pad_w, sign, kpb, 4, CG._cus(torch.device(dev)), N.stream())
    assert rc == 0, rc
    return out.float()


g = torch.Generator(device=dev).manual_seed(0)
for (M, Nn, K) in [(512, 256, 256), (512, 256, 512), (300, 128, 1024)]:
    a = torch.randn(M + 64, K, device=dev, generator=g).to(torch.bfloat16)
    kpb = int(math.log2(K // 64))
    base = a.data_ptr()
    res = []
    for kt in range(K // 64):
        w = torch.zeros(Nn, K, device=dev, dtype=torch.bfloat16)
        w[:, kt * 64:(kt + 1) * 64] = (torch.randn(Nn, 64, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        y = run(base, K, base, base + a.numel() * 2, w, M, Nn, K, 1, 1, 0, 0, 0, 1, kpb)
        ref = a[:M].float() @ w.float().t()
        res.append(round(float(y.norm() / ref.norm()), 3))
    print(f"plain M={M} N={Nn} K={K} kpb={kpb}: |y|/|ref| per K-tile {res}", flush=True)
# the 3x3 path with several K-tile counts: C = 64 * 2^kpb
for C in (64, 128, 256):
    x = torch.randn(2, 6, 6, C, device=dev, generator=g).to(torch.bfloat16)
    buf, gg, Hp, Wp = CG._bordered(x)
    Mq = 2 * Hp * Wp
    K9 = 9 * C
    Kp = K9 if (K9 // 64) % 2 == 0 else K9 + 64
    res = []
    for kt in range(min(Kp // 64, 8)):
        w = torch.zeros(64, Kp, device=dev, dtype=torch.bfloat16)
        w[:, kt * 64:(kt + 1) * 64] = (torch.randn(64, 64, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        for sign in (1, -1):
            y = CG._conv_gemm(buf, gg, C, Hp, Wp, Mq, w, Kp, 64, sign).float()
            tap, kc = divmod(kt * 64, C)
            s = sign * ((tap // 3 - 1) * Wp + (tap % 3 - 1)) if tap < 9 else 0
            ref = buf[gg + s:gg + s + Mq, kc:kc + 64].float() @ w[:, kt * 64:(kt + 1) * 64].float().t()
            res.append((kt, sign, round(float(y.norm() / ref.norm().clamp_min(1e-9)), 3),
                        round(float((y - ref).norm() / ref.norm().clamp_min(1e-9)), 3)))
    print(f"conv C={C}: (kt, sign, |y|/|ref|, rel err) {res}", flush=True)
