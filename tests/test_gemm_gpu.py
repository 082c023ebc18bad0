"""Hand-written MFMA GEMM (csrc/kernels/gemm.hip) vs an fp32 PyTorch reference of the same op.

Covers the three Linear layouts (forward x@W, dgrad dy@W^T, wgrad x^T@dy into an fp32 main grad with
beta 0/1), the bias and SwiGLU epilogues, ragged edges (M, N not multiples of the 256 tile, K a
multiple of 8 but not of 64), and the 7B-width bench shapes at M = 32768 tokens.
"""
import pytest
import torch

from paddle2_amd.ops import gemm as G

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(params=[None, 0, 4, 5, 6, 7, 8, G.V7_SPREAD], ids=["per-pass", "v2", "v4", "v4spread", "v6", "v7", "v7b4", "v7spread"],
                autouse=True)
def schedule(request, monkeypatch):
    """Every test runs on each kernel schedule (None = the per-pass default routing)."""
    monkeypatch.setattr(G, "VARIANT", request.param)
    return request.param


def _rand(*shape, scale=1.0, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=dev) * scale).to(torch.bfloat16)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


SHAPES = [(256, 256, 64), (512, 768, 128), (300, 520, 72), (1000, 264, 1032), (64, 1024, 4096), (2048, 4096, 4096)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_fwd(M, N, K):
    x, w = _rand(M, K, seed=1), _rand(K, N, seed=2, scale=0.05)
    ref = x.float() @ w.float()
    assert _rel(G.mm_fwd(x, w), ref) < 8e-3


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_fwd_bias(M, N, K):
    x, w, b = _rand(M, K, seed=3), _rand(K, N, seed=4, scale=0.05), _rand(N, seed=5)
    ref = x.float() @ w.float() + b.float()
    assert _rel(G.mm_fwd(x, w, bias=b), ref) < 8e-3


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_dgrad(M, N, K):
    # dx[M, K] = dy[M, N] @ w[K, N]^T
    dy, w = _rand(M, N, seed=6), _rand(K, N, seed=7, scale=0.05)
    ref = dy.float() @ w.float().t()
    assert _rel(G.mm_dgrad(dy, w), ref) < 8e-3


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_wgrad_fp32_main_grad(M, N, K, beta):
    # out[K, N] = x[M, K]^T @ dy[M, N] + beta * out  (M is the reduction: tokens)
    x, dy = _rand(M, K, seed=8), _rand(M, N, seed=9)
    out0 = torch.randn(K, N, device=dev) if beta else torch.full((K, N), float("nan"), device=dev)
    ref = x.double().t() @ dy.double() + (beta * out0.double() if beta else 0)
    out = out0.clone()
    G.mm_wgrad(x, dy, out, beta=beta)
    assert torch.isfinite(out).all()
    assert _rel(out, ref) < 1e-5  # fp32 accumulation of exact bf16 products


def test_identity_asymmetric_catches_transpose():
    """A = I with an asymmetric B (guide §3): a row/col swap in the C write cannot pass."""
    n = 256
    eye = torch.eye(n, device=dev, dtype=torch.bfloat16)
    b = (torch.arange(n * n, device=dev, dtype=torch.float32).reshape(n, n) % 251 - 125).to(torch.bfloat16)
    assert torch.equal(G.mm_fwd(eye, b), b)
    assert torch.equal(G.mm_dgrad(eye, b.t().contiguous()), b)
    out = torch.empty(n, n, device=dev)
    G.mm_wgrad(eye, b, out)
    assert torch.equal(out, b.float())


@pytest.mark.parametrize("M,K,H", [(512, 256, 256), (300, 136, 96), (4096, 4096, 11008)])
def test_swiglu_epilogue(M, K, H):
    x, w = _rand(M, K, seed=10), _rand(K, 2 * H, seed=11, scale=0.05)
    a, gu = G.mm_swiglu(x, w)
    gu_ref = x.float() @ w.float()
    assert _rel(gu, gu_ref) < 1e-2  # bf16-rounded pre-activation
    g, u = gu.float()[:, :H], gu.float()[:, H:]
    a_ref = torch.nn.functional.silu(g) * u  # from the stored (rounded) pre-activation
    assert _rel(a, a_ref) < 8e-3


GELU_SHAPES = [(256, 256, 128), (300, 520, 72), (1000, 264, 1032), (2048, 5120, 5120)]


@pytest.mark.parametrize("M,N,K", GELU_SHAPES)
@pytest.mark.parametrize("approx", [True, False])
def test_gelu_epilogue(M, N, K, approx):
    """gelu(x @ W + b) and the stored pre-activation from one GEMM vs the fp32 reference."""
    x, w, b = _rand(M, K, seed=20), _rand(K, N, seed=21, scale=K ** -0.5), _rand(N, seed=22)
    a, h = G.mm_gelu(x, w, b, approximate=approx)
    h_ref = x.float() @ w.float() + b.float()
    assert _rel(h, h_ref) < 8e-3
    a_ref = torch.nn.functional.gelu(h.float(), approximate="tanh" if approx else "none")  # from the stored h
    assert _rel(a, a_ref) < 8e-3


@pytest.mark.parametrize("M,N,K", GELU_SHAPES)
@pytest.mark.parametrize("approx", [True, False])
def test_dgelu_epilogue(M, N, K, approx):
    """dh = (dy @ W^T) * gelu'(h) vs autograd through an fp32 gelu."""
    dy, w, h = _rand(M, N, seed=23), _rand(K, N, seed=24, scale=N ** -0.5), _rand(M, K, seed=25)
    hr = h.float().requires_grad_()
    torch.nn.functional.gelu(hr, approximate="tanh" if approx else "none").backward(dy.float() @ w.float().t())
    assert _rel(G.mm_dgrad_dgelu(dy, w, h, approximate=approx), hr.grad) < 8e-3


def test_gelu_mlp_node_matches_fp32(monkeypatch):
    """The fused GPT MLP node (torch_ops._GeluMLPFn, opt-in): output and every gradient vs the fp32 composition."""
    from paddle2_amd.ops import torch_ops as T

    monkeypatch.setattr(T, "_FUSED_GELU_MLP", True)
    M, H, F4 = 1024, 512, 2048
    x = _rand(M, H, seed=26)
    w1, b1 = _rand(H, F4, seed=27, scale=H ** -0.5), _rand(F4, seed=28, scale=0.1)
    w2, b2 = _rand(F4, H, seed=29, scale=F4 ** -0.5), _rand(H, seed=30, scale=0.1)
    dy = _rand(M, H, seed=31)
    ts = [t.clone().requires_grad_() for t in (x, w1, b1, w2, b2)]
    assert T.gelu_mlp_ok(*ts)
    y = T._GeluMLPFn.apply(*ts, True)
    y.backward(dy)
    rs = [t.float().requires_grad_() for t in (x, w1, b1, w2, b2)]
    yr = torch.nn.functional.gelu(rs[0] @ rs[1] + rs[2], approximate="tanh") @ rs[3] + rs[4]
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    for t, r in zip(ts, rs):
        assert _rel(t.grad, r.grad) < 1.5e-2


@pytest.mark.parametrize("N,K", [(12288, 4096), (4096, 4096), (4096, 11008)])
def test_llama7b_shapes_m32768(N, K):
    """bench shapes at M = 32768 tokens: fwd, dgrad, fp32 wgrad vs fp32 references (row-sampled)."""
    M = 32768
    x, w, dy = _rand(M, K, seed=12), _rand(K, N, seed=13, scale=0.02), _rand(M, N, seed=14)
    rows = torch.arange(0, M, 97, device=dev)
    y = G.mm_fwd(x, w)
    assert _rel(y[rows], x[rows].float() @ w.float()) < 8e-3
    dx = G.mm_dgrad(dy, w)
    assert _rel(dx[rows], dy[rows].float() @ w.float().t()) < 8e-3
    out = torch.empty(K, N, device=dev)
    G.mm_wgrad(x, dy, out)
    cols = torch.arange(0, N, 61, device=dev)
    ref = x.float().t() @ dy[:, cols].float()
    assert _rel(out[:, cols], ref) < 1e-4


@pytest.mark.parametrize("mode", ["native", "blas"])
def test_linear_node_passes(mode, monkeypatch):
    """ops.torch_ops.linear (the Llama Linear node) with every GEMM pass on the native kernel (or hipBLASLt)
    vs an fp32 reference of y = x W, dx = dy W^T, dW = x^T dy; plus the fp32 main-grad route."""
    from paddle2_amd.ops import torch_ops as T

    for k in ("fwd", "dgrad", "wgrad"):
        monkeypatch.setitem(T._GEMM_PASS, k, mode)
    M, K, N = 4096, 512, 768
    x = _rand(M, K, seed=20).requires_grad_()
    w = _rand(K, N, seed=21, scale=0.05).requires_grad_()
    dy = _rand(M, N, seed=22)
    y = T.linear(x, w)
    y.backward(dy)
    xf, wf, dyf = x.detach().float(), w.detach().float(), dy.float()
    assert _rel(y, xf @ wf) < 8e-3
    assert _rel(x.grad, dyf @ wf.t()) < 8e-3
    assert _rel(w.grad, xf.t() @ dyf) < 8e-3

    class Owner:
        def __init__(self):
            self.buf = torch.zeros(K, N, device=dev)
            self.done = 0

        def grad_target(self, i):
            return self.buf, 1

        def param_grad_done(self, i):
            self.done += 1

    o = Owner()
    w2 = w.detach().clone().requires_grad_()
    w2._p2_gt = (o, 0)
    T.linear(x.detach(), w2).backward(dy)
    T.linear(x.detach(), w2).backward(dy)  # accumulates (beta = 1)
    assert o.done == 2 and w2.grad is None
    assert _rel(o.buf, 2 * (xf.t() @ dyf)) < 1e-4


@pytest.mark.parametrize("mode", ["native", "blas"])
def test_swiglu_linear_node(mode, monkeypatch):
    from paddle2_amd.ops import torch_ops as T

    for k in ("fwd", "dgrad", "wgrad"):
        monkeypatch.setitem(T._GEMM_PASS, k, mode)
    M, K, H = 4096, 512, 384
    x = _rand(M, K, seed=23).requires_grad_()
    w = _rand(K, 2 * H, seed=24, scale=0.05).requires_grad_()
    da = _rand(M, H, seed=25)
    a = T.swiglu_linear(x, w)
    a.backward(da)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    gu = xf @ wf
    af = torch.nn.functional.silu(gu[:, :H]) * gu[:, H:]
    af.backward(da.float())
    assert _rel(a, af) < 1e-2
    assert _rel(x.grad, xf.grad) < 1e-2
    assert _rel(w.grad, wf.grad) < 1e-2


@pytest.mark.parametrize("M,N,K", [(2048, 4096, 4096), (300, 520, 72), (4096, 22016, 4096)])
def test_schedule_variants_bitwise_equal(M, N, K, monkeypatch, schedule):
    """v2 (8 waves), v4 (4 waves, AGPR accumulators), v6 (persistent) and v7 (TN schedule) accumulate the same
    products in the same order: their outputs must agree bit for bit (a staging race shows up here first)."""
    if schedule is not None:
        pytest.skip("compares the schedules itself")
    x, w, dy = _rand(M, K, seed=30), _rand(K, N, seed=31, scale=0.05), _rand(M, N, seed=32)
    monkeypatch.setattr(G, "SPLITK", False)   # tail split-K sums K-slices in another order (v2 / v4)
    outs = []
    swi = (N // 2) % 32 == 0
    for v in (0, 4, 5, 6, 7, 8, 9, 10, G.V7_SPREAD, 64 + 128, G.V7_MN):  # v5: v4 spread; v7 (TN) incl. spread
        monkeypatch.setattr(G, "VARIANT", v)
        o32 = torch.zeros(K, N, device=dev)
        G.mm_wgrad(x, dy, o32)
        outs.append((G.mm_fwd(x, w), G.mm_dgrad(dy, w), o32) + (G.mm_swiglu(x, w) if swi else ()))
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert torch.equal(a, b)


@pytest.mark.parametrize("M,N,K", [(4096, 22016, 32768), (11008, 4096, 32768), (1024, 1024, 8192),
                                   (304, 520, 2048)])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_tail_splitk_wgrad_and_fwd(M, N, K, beta, monkeypatch):
    """Shapes whose last wave per XCD is at most half full run their tail tiles as K-slices + a reduce:
    same result as the unsplit kernel up to summation order (fp32), and vs an fp64 reference."""
    # wgrad out[M, N] = x[K, M]^T @ dy[K, N] (K tokens); 4096x22016 = 1376 tiles, 11008x4096 = 688
    x, dy = _rand(K, M, seed=40), _rand(K, N, seed=41)
    out0 = torch.randn(M, N, device=dev)
    outs = []
    for split in (True, False):
        monkeypatch.setattr(G, "SPLITK", split)
        o = out0.clone()
        G.mm_wgrad(x, dy, o, beta=beta)
        outs.append(o)
    cols = torch.arange(0, N, 37, device=dev)
    ref = x.double().t() @ dy[:, cols].double() + (beta * out0[:, cols].double() if beta else 0)
    assert _rel(outs[0][:, cols], ref) < 1e-5
    assert _rel(outs[0], outs[1]) < 1e-6
    # bf16 epilogue (+bias) through the same path: forward y = a @ w
    monkeypatch.setattr(G, "SPLITK", True)
    a, w, b = _rand(M, K, seed=42), _rand(K, N, seed=43, scale=0.02), _rand(N, seed=44)
    rows = torch.arange(0, M, 53, device=dev)
    assert _rel(G.mm_fwd(a, w, bias=b)[rows], a[rows].float() @ w.float() + b.float()) < 8e-3


@pytest.mark.parametrize("B,S,nq,nkv", [(2, 256, 4, 2), (1, 512, 8, 8), (1, 200, 2, 1)])
def test_qkv_rope_linear_node(B, S, nq, nkv):
    """The QKV projection with RoPE in the GEMM epilogue (torch_ops._QKVRopeLinearFn): rotated q / k heads and the
    unrotated v vs the fp32 GEMM + rotate-half reference, and the input / weight gradients through RoPE^T."""
    from paddle2_amd.ops import torch_ops as T

    K, D = 512, 128
    Nn = (nq + 2 * nkv) * D
    x = _rand(B, S, K, seed=40)
    w = _rand(K, Nn, seed=41, scale=K ** -0.5)
    cos, sin = T.rope_tables(S, D, interleaved=False, device=dev)
    dy = _rand(B, S, Nn, seed=42)
    xi, wi = x.clone().requires_grad_(), w.clone().requires_grad_()
    y = T._QKVRopeLinearFn.apply(xi, wi, cos.contiguous(), sin.contiguous(), nq + nkv, S)
    y.backward(dy)
    xr, wr = x.float().requires_grad_(), w.float().requires_grad_()
    h = (xr @ wr).view(B, S, nq + 2 * nkv, D)
    c, s_ = cos[None, :, None, :], sin[None, :, None, :]
    qk = h[:, :, :nq + nkv]
    x1, x2 = qk[..., :D // 2], qk[..., D // 2:]
    rot = torch.cat([x1 * c[..., :D // 2] - x2 * s_[..., :D // 2], x2 * c[..., D // 2:] + x1 * s_[..., D // 2:]], -1)
    yr = torch.cat([rot, h[:, :, nq + nkv:]], 2).view(B, S, Nn)
    yr.backward(dy.float())
    assert _rel(y, yr) < 8e-3
    assert _rel(xi.grad, xr.grad) < 1e-2
    assert _rel(wi.grad, wr.grad) < 1e-2


@pytest.mark.parametrize("M,H,N", [(256, 256, 128), (1024, 640, 512), (4096, 1408, 1024)])
def test_dswiglu_epilogue(M, H, N):
    """d_gu = SwiGLU backward of (dy @ W^T) with the saved gate | up, from one GEMM epilogue, vs fp32 autograd."""
    if G._variant("dgrad") != G.V7_SPREAD:
        pytest.skip("spread TN schedule only")
    dy, w, gu = _rand(M, N, seed=50), _rand(H, N, seed=51, scale=N ** -0.5), _rand(M, 2 * H, seed=52)
    out = G.mm_dgrad_dswiglu(dy, w, gu)
    assert out is not None
    gr = gu.float().requires_grad_()
    g, u = gr[:, :H], gr[:, H:]
    (torch.nn.functional.silu(g) * u).backward(dy.float() @ w.float().t())
    assert _rel(out, gr.grad) < 1e-2


def test_swiglu_mlp_node_matches_fp32(monkeypatch):
    """The one-node Llama MLP (torch_ops._SwiGLUMLPFn): output and the input / weight gradients vs fp32."""
    from paddle2_amd.ops import torch_ops as T

    monkeypatch.setattr(T, "_SWIGLU_MLP_NODE", True)   # opt-in route

    M, K, H = 4096, 512, 1408
    x = _rand(M, K, seed=53)
    wgu, wd = _rand(K, 2 * H, seed=54, scale=K ** -0.5), _rand(H, K, seed=55, scale=H ** -0.5)
    dy = _rand(M, K, seed=56)
    if not T.swiglu_mlp_ok(x, wgu, wd):
        pytest.skip("MLP node not selected for this schedule")
    xi, a, b = (t.clone().requires_grad_() for t in (x, wgu, wd))
    y = T.swiglu_mlp(xi, a, b)
    y.backward(dy)
    xr, ar, br = (t.float().requires_grad_() for t in (x, wgu, wd))
    h = xr @ ar
    yr = (torch.nn.functional.silu(h[:, :H]) * h[:, H:]) @ br
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    for got, ref in ((xi.grad, xr.grad), (a.grad, ar.grad), (b.grad, br.grad)):
        assert _rel(got, ref) < 2e-2


@pytest.mark.parametrize("M,N,K", [(1024, 1536, 4096), (520, 776, 2048), (4096, 5120, 4096), (2048, 256, 8192),
                                   (256, 4096, 1024)])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_wgrad_v7_mn_matches_v5_and_fp64(M, N, K, beta, schedule, monkeypatch):
    """The weight gradient on the persistent spread kernel with both operands MN-major (gemm7.hip SCHED bit 15): the
    same products in the same order as v4's spread wgrad (bit-identical without the tail split-K; beta 1 adds by
    one fp32 atomic per element = the read-modify-write's rounding), and vs fp64 with the split, incl. ragged tiles
    (M, N not multiples of 256) and the bf16 epilogue."""
    if schedule is not None:
        pytest.skip("compares two fixed schedules")
    # out[M, N] = x[K, M]^T @ dy[K, N] (K tokens)
    x, dy = _rand(K, M, seed=60), _rand(K, N, seed=61)
    out0 = torch.randn(M, N, device=dev)
    ref = x.double().t() @ dy.double() + (beta * out0.double() if beta else 0)
    res = {}
    for split in (False, True):
        monkeypatch.setattr(G, "SPLITK", split)
        for v in (5, G.V7_MN):
            monkeypatch.setattr(G, "VARIANT", v)
            o = out0.clone()
            G.mm_wgrad(x, dy, o, beta=beta)
            res[(split, v)] = o
    assert torch.equal(res[(False, 5)], res[(False, G.V7_MN)])
    assert _rel(res[(True, G.V7_MN)], ref) < 1e-5
    assert _rel(res[(True, G.V7_MN)], res[(False, G.V7_MN)]) < 1e-6
    monkeypatch.setattr(G, "VARIANT", G.V7_MN)
    ob = G.mm_wgrad_bf16(x, dy)
    assert _rel(ob, x.float().t() @ dy.float()) < 8e-3


@pytest.mark.parametrize("M,N,K", [(4096, 5120, 5120), (1000, 1000, 2048), (256, 15360, 5120), (8192, 4096, 4096),
                                   (512, 22016, 1024)])
def test_fwd_nn_small_m_matches_tn(M, N, K, schedule, monkeypatch):
    """Short token batches run the forward on W as stored (spread schedule, B N-major, no W^T pass; v4's kernel or the
    persistent v7 one): the same products in the same order as the TN route on W^T, so bit-identical without the tail
    split-K, and vs fp32 with it."""
    if schedule is not None:
        pytest.skip("per-pass routing only")
    x, w, b = _rand(M, K, seed=50), _rand(K, N, seed=51, scale=K ** -0.5), _rand(N, seed=52, scale=0.5)
    assert G._fwd_nn(M)
    ref = x.float() @ w.float() + b.float()
    ys = {}
    for split in (True, False):
        monkeypatch.setattr(G, "SPLITK", split)
        monkeypatch.setattr(G, "V7_TAILK", split)
        for v in (5, G.V7_NNF):   # v4's spread kernel / the persistent v7 kernel with W N-major
            monkeypatch.setitem(G.PASS_VARIANT, "fwd_nn", v)
            monkeypatch.setitem(G.PASS_VARIANT, "fwd_nn_wide", v)
            ys[(split, v)] = G.mm_fwd(x, w, b)
            assert _rel(ys[(split, v)], ref) < 8e-3
    monkeypatch.setattr(G, "FWD_NN_MAX_M", 0)
    assert not G._fwd_nn(M)
    y_tn = G.mm_fwd(x, w, b)
    assert torch.equal(ys[(False, 5)], y_tn)
    assert torch.equal(ys[(False, G.V7_NNF)], y_tn)


@pytest.mark.parametrize("M,N,K,bias", [(4096, 5120, 5120, False), (4096, 5120, 5120, True), (1000, 1000, 2048, True),
                                        (640, 4096, 1024, False)])
def test_v7_tail_splitk_matches_fp32(M, N, K, bias, monkeypatch):
    """Spread TN schedule with the tail split-K (a partial last wave of <= CUs / 2 tiles as K-slices + fp32 fix-up;
    gemm7.hip SCHED bit 12): forward (+ bias) and dgrad vs fp32, and vs the same GEMM without the split."""
    x, w, dy = _rand(M, K, seed=40), _rand(K, N, seed=41, scale=K ** -0.5), _rand(M, N, seed=42)
    b = _rand(N, seed=43, scale=0.5) if bias else None
    ref = x.float() @ w.float() + (b.float() if bias else 0.0)
    y = G.mm_fwd(x, w, b)
    assert _rel(y, ref) < 8e-3
    dx = G.mm_dgrad(dy, w)
    assert _rel(dx, dy.float() @ w.float().t()) < 8e-3
    monkeypatch.setattr(G, "V7_TAILK", False)
    y0 = G.mm_fwd(x, w, b)
    assert _rel(y, y0) < 8e-3


@pytest.mark.parametrize("M,V,H", [(1024, 2048, 512), (777, 4096, 256)])
def test_tied_logits_native_matches_fp32(M, V, H):
    """GPT's tied output layer h @ E^T on the native TN GEMM (E as stored): forward and both gradients vs fp32."""
    from paddle2_amd.ops import torch_ops as T

    torch.manual_seed(0)
    h = (torch.randn(M, H, device="cuda") * 0.5).bfloat16().requires_grad_()
    E = (torch.randn(V, H, device="cuda") * 0.5).bfloat16().requires_grad_()
    y = T.tied_logits(h, E)
    fn, names = y.grad_fn, []
    while fn is not None:
        names.append(type(fn).__name__)
        fn = fn.next_functions[0][0] if fn.next_functions else None
    assert any(n.startswith("_TiedLogitsFn") for n in names), names
    g = torch.randn(M, V, device="cuda").bfloat16()
    y.backward(g)
    hf, Ef = h.detach().float().requires_grad_(), E.detach().float().requires_grad_()
    yf = hf @ Ef.t()
    yf.backward(g.float())
    assert _rel(y, yf) < 1e-2
    assert _rel(h.grad, hf.grad) < 1e-2
    assert _rel(E.grad, Ef.grad) < 1e-2
