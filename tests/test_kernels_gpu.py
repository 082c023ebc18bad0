"""Numerics of the hand-written CDNA4 kernels vs. plain PyTorch fp32 references of the same op.

Every test runs the op on the MI355X (native HIP path — _native.use_native raises if the .so is
missing) and on CPU fp32 copies (the reference branch of the same autograd.Function)."""
import math

import pytest
import torch

from paddle2_amd.ops import _native
from paddle2_amd.ops import torch_ops as T

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _close(a, b, atol, rtol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max abs err {err} > {tol}"


def _pair(shape, dtype, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(shape, generator=g) * scale
    return x.to(DEV, dtype).requires_grad_(True), x.clone().requires_grad_(True)


def test_native_loaded():
    assert _native.available()
    _native.require()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("N", [128, 4096, 5120])
@pytest.mark.parametrize("residual", [False, True])
def test_rms_norm(dtype, N, residual):
    M = 257
    xg, xc = _pair((M, N), dtype, seed=1)
    wg, wc = _pair((N,), dtype, seed=2)
    if residual:
        rg, rc = _pair((M, N), dtype, seed=3)
        yg, hg = T.rms_norm(xg, wg, 1e-6, rg)
        yc, hc = T.rms_norm(xc.to(dtype).float(), wc.to(dtype).float(), 1e-6, rc.to(dtype).float())
        (yg.float().sum() + (hg.float() * 0.5).sum()).backward()
        (yc.sum() + (hc * 0.5).sum()).backward()
    else:
        yg = T.rms_norm(xg, wg, 1e-6)
        yc = T.rms_norm(xc.to(dtype).float(), wc.to(dtype).float(), 1e-6)
        go = torch.randn(M, N)
        yg.backward(go.to(DEV, dtype))
        yc.backward(go.to(dtype).float())
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    _close(yg, yc, tol, tol)
    _close(xg.grad, xc.grad, tol * 3, tol * 3)
    _close(wg.grad, wc.grad, tol * 20, tol * 3)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_layer_norm(dtype):
    M, N = 300, 1024
    xg, xc = _pair((M, N), dtype, seed=4)
    wg, wc = _pair((N,), dtype, seed=5)
    bg, bc = _pair((N,), dtype, seed=6)
    yg = T.layer_norm(xg, wg, bg, 1e-5)
    yc = T.layer_norm(xc.to(dtype).float(), wc.to(dtype).float(), bc.to(dtype).float(), 1e-5)
    go = torch.randn(M, N)
    yg.backward(go.to(DEV, dtype))
    yc.backward(go.to(dtype).float())
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    _close(yg, yc, tol, tol)
    _close(xg.grad, xc.grad, tol * 3, tol * 3)
    _close(wg.grad, wc.grad, tol * 20, tol * 3)
    _close(bg.grad, bc.grad, tol * 20, tol * 3)


@pytest.mark.parametrize("packed", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_swiglu(packed, dtype):
    if packed:
        xg, xc = _pair((3, 17, 2 * 688), dtype, seed=7)
        og = T.swiglu(xg)
        oc = T.swiglu(xc.to(dtype).float())
        ins = [(xg, xc)]
    else:
        xg, xc = _pair((3, 17, 688), dtype, seed=7)
        yg, yc = _pair((3, 17, 688), dtype, seed=8)
        og = T.swiglu(xg, yg)
        oc = T.swiglu(xc.to(dtype).float(), yc.to(dtype).float())
        ins = [(xg, xc), (yg, yc)]
    go = torch.randn(oc.shape)
    og.backward(go.to(DEV, dtype))
    oc.backward(go.to(dtype).float())
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    _close(og, oc, tol, tol)
    for g, c in ins:
        _close(g.grad, c.grad, tol * 2, tol * 2)


@pytest.mark.parametrize("style", [0, 1])
@pytest.mark.parametrize("D", [128, 64, 40])
@pytest.mark.parametrize("with_pos", [False, True])
def test_rope(style, D, with_pos):
    B, S, H = 2, 67, 5
    cos, sin = T.rope_tables(128, D, 10000.0, interleaved=bool(style))
    xg, xc = _pair((B, S, H, D), torch.bfloat16, seed=9)
    pos = torch.randint(0, 128, (B, S)) if with_pos else None
    og = T.rope(xg, cos.to(DEV), sin.to(DEV), None if pos is None else pos.to(DEV), style)
    oc = T.rope(xc.to(torch.bfloat16).float(), cos, sin, pos, style)
    go = torch.randn(B, S, H, D)
    og.backward(go.to(DEV, torch.bfloat16))
    oc.backward(go.to(torch.bfloat16).float())
    _close(og, oc, 2e-2, 1e-2)
    _close(xg.grad, xc.grad, 2e-2, 1e-2)


@pytest.mark.parametrize("V", [32000, 1000, 501])
def test_softmax_cross_entropy(V):
    N = 129
    xg, xc = _pair((N, V), torch.bfloat16, scale=3.0, seed=10)
    lab = torch.randint(0, V, (N,))
    lab[5] = -100
    lg = T.softmax_cross_entropy(xg, lab.to(DEV), -100)
    lc = T.softmax_cross_entropy(xc.to(torch.bfloat16).float(), lab, -100)
    _close(lg, lc, 1e-2, 1e-3)
    lg.sum().backward()
    lc.sum().backward()
    _close(xg.grad, xc.grad, 1e-2, 2e-2)


def test_embedding():
    V, H, Nt = 1000, 256, 333
    wg, wc = _pair((V, H), torch.bfloat16, seed=11)
    ids = torch.randint(0, V, (3, Nt // 3))
    og = T.embedding(ids.to(DEV), wg)
    oc = T.embedding(ids, wc.to(torch.bfloat16).float())
    _close(og, oc, 1e-6, 1e-6)
    go = torch.randn(oc.shape)
    og.backward(go.to(DEV, torch.bfloat16))
    oc.backward(go.to(torch.bfloat16).float())
    _close(wg.grad, wc.grad, 3e-2, 1e-2)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("D", [128, 64])
@pytest.mark.parametrize("shape", [(2, 256, 256, 4, 4), (1, 200, 200, 4, 2), (1, 130, 300, 2, 1), (1, 1100, 1100, 2, 1)])
def test_flash_attention(causal, D, shape):
    B, Sq, Sk, Hq, Hk = shape
    qg, qc = _pair((B, Sq, Hq, D), torch.bfloat16, seed=12)
    kg, kc = _pair((B, Sk, Hk, D), torch.bfloat16, seed=13)
    vg, vc = _pair((B, Sk, Hk, D), torch.bfloat16, seed=14)
    og, lg = T.flash_attention(qg, kg, vg, causal)
    oc, lc = T.flash_attention(qc.to(torch.bfloat16).float(), kc.to(torch.bfloat16).float(),
                               vc.to(torch.bfloat16).float(), causal)
    _close(og, oc, 2e-2, 2e-2)
    fin = torch.isfinite(lc)
    _close(lg.cpu()[fin], lc[fin], 1e-2, 1e-3)
    go = torch.randn(oc.shape)
    og.backward(go.to(DEV, torch.bfloat16))
    oc.backward(go.to(torch.bfloat16).float())
    _close(qg.grad, qc.grad, 5e-2, 3e-2)
    _close(kg.grad, kc.grad, 5e-2, 3e-2)
    _close(vg.grad, vc.grad, 5e-2, 3e-2)


def test_flash_attention_strided_qkv():
    """q/k/v as row-strided views of a fused QKV projection output (no copies)."""
    B, S, H, D = 2, 192, 4, 128
    qkv = torch.randn(B, S, 3 * H, D, device=DEV, dtype=torch.bfloat16)
    q, k, v = qkv[:, :, :H], qkv[:, :, H:2 * H], qkv[:, :, 2 * H:]
    o, _ = T.flash_attention(q, k, v, True)
    oc, _ = T.flash_attention(q.float().cpu(), k.float().cpu(), v.float().cpu(), True)
    _close(o, oc, 2e-2, 2e-2)


@pytest.mark.parametrize("pdt,gdt,master", [(torch.bfloat16, torch.bfloat16, True), (torch.float32, torch.float32, False),
                                            (torch.bfloat16, torch.float32, True)])
def test_fused_adamw(pdt, gdt, master):
    import paddle2_amd as paddle

    paddle.set_device("gpu:0")
    shapes = [(1000,), (33, 65), (4096,), (7,)]
    ps_g, ps_c = [], []
    for i, s in enumerate(shapes):
        t = torch.randn(s, generator=torch.Generator().manual_seed(i))
        ps_g.append(paddle.framework.param.Parameter(t.to(DEV, pdt)))
        ps_c.append(paddle.framework.param.Parameter(t.to(pdt).float()))
    og = paddle.optimizer.AdamW(1e-2, parameters=ps_g, weight_decay=0.1, multi_precision=master)
    oc = paddle.optimizer.AdamW(1e-2, parameters=ps_c, weight_decay=0.1)
    for step in range(3):
        for i, (a, b) in enumerate(zip(ps_g, ps_c)):
            g = torch.randn(a.shape, generator=torch.Generator().manual_seed(100 + 10 * step + i))
            if gdt != pdt:  # fp32 grads of bf16 params travel as Paddle's main_grad
                a.main_grad = g.to(DEV, gdt)
            else:
                a._t.grad = g.to(DEV, gdt)
            b._t.grad = g.to(gdt).float()
        og.step()
        oc.step()
    for a, b in zip(ps_g, ps_c):
        _close(a._t, b._t, 2e-2 if pdt == torch.bfloat16 else 1e-5, 1e-3)


def test_clip_grad_global_norm():
    import paddle2_amd as paddle

    gs = [torch.randn(s, device=DEV) for s in [(100,), (37, 3), (5000,)]]
    ps = [paddle.framework.param.Parameter(torch.zeros_like(g)) for g in gs]
    for p, g in zip(ps, gs):
        p._t.grad = g.clone()
    clip = paddle.nn.ClipGradByGlobalNorm(1.0)
    clip([(p, p.grad) for p in ps])
    total = math.sqrt(sum(float((g.float() ** 2).sum()) for g in gs))
    for p, g in zip(ps, gs):
        _close(p._t.grad, g * min(1.0, 1.0 / total), 1e-5, 1e-4)


def test_grad_scaler_unscale_and_skip():
    import paddle2_amd as paddle

    p = paddle.framework.param.Parameter(torch.ones(64, device=DEV))
    opt = paddle.optimizer.AdamW(1e-1, parameters=[p])
    sc = paddle.amp.GradScaler(init_loss_scaling=1024.0)
    p._t.grad = torch.full((64,), 1024.0, device=DEV)
    sc.step(opt)
    sc.update()
    assert not torch.allclose(p._t, torch.ones(64, device=DEV))
    before = p._t.clone()
    p._t.grad = torch.full((64,), float("inf"), device=DEV)
    sc.step(opt)
    sc.update()
    assert torch.equal(before, p._t)
    assert float(sc._scale) == 1024.0 or float(sc._scale) == 512.0


@pytest.mark.parametrize("nh,nkv", [(4, 4), (4, 2)])
def test_qkv_rope_attention_fused(nh, nkv):
    """Fused QKV->RoPE->flash node (strided views, one dQKV buffer) vs. fp32 CPU reference."""
    B, S, D = 2, 160, 128
    cos, sin = T.rope_tables(256, D, 10000.0, interleaved=False)
    xg, xc = _pair((B, S, nh + 2 * nkv, D), torch.bfloat16, seed=21)
    og = T.qkv_rope_attention(xg, nh, nkv, cos.to(DEV), sin.to(DEV), causal=True)
    oc = T.qkv_rope_attention(xc.to(torch.bfloat16).float(), nh, nkv, cos, sin, causal=True)
    _close(og, oc, 2e-2, 2e-2)
    go = torch.randn(oc.shape)
    og.backward(go.to(DEV, torch.bfloat16))
    oc.backward(go.to(torch.bfloat16).float())
    _close(xg.grad, xc.grad, 5e-2, 3e-2)


@pytest.mark.parametrize("M,N", [(4096, 4096), (1000, 72), (136, 8), (8192, 264)])
def test_transpose16(M, N):
    x = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    assert torch.equal(T.transpose2d(x), x.t().contiguous())
    big = torch.randn(M, N + 16, device=DEV, dtype=torch.float16)[:, :N]  # row-strided view
    assert torch.equal(T.transpose2d(big), big.t().contiguous())


@pytest.mark.parametrize("layout", ["off", "all", "auto"])
def test_linear_layouts(layout, monkeypatch):
    """Layout-aware Linear node (W^T forward GEMM, X^T/dY^T weight-gradient GEMM) vs fp32 reference."""
    monkeypatch.setattr(T, "_LINEAR_LAYOUT", layout)
    M, K, Nn = 8192, 256, 768
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(2, M // 2, K, generator=g)).to(torch.bfloat16)
    w = (torch.randn(K, Nn, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(Nn, generator=g).to(torch.bfloat16)
    go = torch.randn(2, M // 2, Nn, generator=g).to(torch.bfloat16)
    xg, wg, bg = (t.to(DEV).requires_grad_(True) for t in (x, w, b))
    y = T.linear(xg, wg, bg)
    y.backward(go.to(DEV))
    xc, wc, bc = (t.float().requires_grad_(True) for t in (x, w, b))
    yc = xc @ wc + bc
    yc.backward(go.float())
    _close(y, yc, 5e-2, 1e-2)
    _close(xg.grad, xc.grad, 5e-2, 1e-2)
    _close(wg.grad, wc.grad, 5e-1, 1e-2)
    _close(bg.grad, bc.grad, 5e-1, 1e-2)


@pytest.mark.parametrize("M", [8192, 4100])
def test_swiglu_linear_fused(M):
    """GEMM + SwiGLU node whose backward kernel also writes dY^T for the weight gradient."""
    K, H = 256, 192
    g = torch.Generator().manual_seed(5)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(K, 2 * H, generator=g) * 0.05).to(torch.bfloat16)
    go = torch.randn(M, H, generator=g).to(torch.bfloat16)
    xg, wg = (t.to(DEV).requires_grad_(True) for t in (x, w))
    a = T.swiglu_linear(xg, wg)
    a.backward(go.to(DEV))
    xc, wc = (t.float().requires_grad_(True) for t in (x, w))
    gu = xc @ wc
    ac = torch.nn.functional.silu(gu[:, :H]) * gu[:, H:]
    ac.backward(go.float())
    _close(a, ac, 3e-2, 1e-2)
    _close(xg.grad, xc.grad, 5e-2, 1e-2)
    _close(wg.grad, wc.grad, 5e-1, 1e-2)


@pytest.mark.parametrize("M,N,dt", [(4096, 15360, torch.bfloat16), (333, 520, torch.bfloat16), (64, 8, torch.float16),
                                    (2048, 1000, torch.float32), (8192, 22016, torch.bfloat16)])
def test_bias_grad_colsum_matches_fp32(M, N, dt):
    """Native bias-gradient column sum (norm.hip bias_grad_part_kernel + colsum) vs an fp32 sum; ragged column
    blocks and row chunks, and bitwise reproducible run to run."""
    from paddle2_amd.ops import torch_ops as T

    g = torch.Generator(device="cuda").manual_seed(7)
    dy = torch.randn(M, N, generator=g, device="cuda").to(dt)
    db = T.bias_grad(dy)
    ref = dy.float().sum(0)
    assert db.dtype == dt and db.shape == (N,)
    tol = 1e-4 if dt == torch.float32 else 1e-2
    assert (db.float() - ref).abs().max().item() <= tol * max(1.0, ref.abs().max().item())
    assert torch.equal(db, T.bias_grad(dy))
