"""FP8 cast kernels and fp8 linear on the MI355X vs torch references."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("fmt", [torch.float8_e4m3fn, torch.float8_e5m2])
@pytest.mark.parametrize("shape", [(64, 128), (130, 72), (1000, 24), (136, 264), (4096, 5120)])
def test_fp8_cast_transpose_amax(fmt, shape):
    from paddle2_amd.ops import fp8

    x = torch.randn(shape, device=DEV, dtype=torch.bfloat16) * 3
    meta = fp8.FP8TensorMeta(fmt, device=torch.device(DEV))
    meta.scale.fill_(7.0)
    meta.initialized = True  # use this fixed scale (skip the first-use just-in-time scaling)
    q, qT = fp8.cast(x, meta, transpose=True)
    ref = (x.float() * 7.0).clamp(-fp8._MAX[fmt], fp8._MAX[fmt]).to(fmt)
    assert torch.equal(q.view(torch.uint8), ref.view(torch.uint8))
    assert torch.equal(qT.view(torch.uint8), ref.t().contiguous().view(torch.uint8))
    assert float(meta.amax.max()) == pytest.approx(float(x.float().abs().max()))   # sharded slots
    meta.amax.zero_()
    q2, _ = fp8.cast(x, meta, transpose=False)
    assert torch.equal(q2.view(torch.uint8), ref.view(torch.uint8))
    assert float(meta.amax.max()) == pytest.approx(float(x.float().abs().max()))


def test_fp8_delayed_scaling_update():
    from paddle2_amd.ops import fp8

    m = fp8.FP8TensorMeta(torch.float8_e4m3fn, history_len=4, device=torch.device(DEV))
    m.amax.fill_(1.0)
    m.amax[17] = 2.0   # the slots fold by max
    m.update()
    assert float(m.scale) == pytest.approx(448.0 / 2.0)
    assert float(m.inv_scale) == pytest.approx(2.0 / 448.0)
    assert float(m.amax.abs().max()) == 0.0


@pytest.mark.parametrize("shape", [(64, 128), (136, 264), (1000, 24), (4096, 5120)])
def test_fp8_cast_fused_column_sums(shape):
    """cast(..., colsum=True): the dY cast also returns per-64-row-block column sums (the fp8 linear's bias
    gradient without a second read of dY); the casts are unchanged, and the folded sums match fp32 (incl. R % 64)."""
    from paddle2_amd.ops import _native as N
    from paddle2_amd.ops import fp8

    R, C = shape
    x = torch.randn(shape, device=DEV, dtype=torch.bfloat16) * 3
    meta = fp8.FP8TensorMeta(torch.float8_e5m2, device=torch.device(DEV))
    meta.scale.fill_(5.0)
    meta.initialized = True
    q, qT, part = fp8.cast(x, meta, transpose=True, colsum=True)
    ref = (x.float() * 5.0).clamp(-57344.0, 57344.0).to(torch.float8_e5m2)
    assert torch.equal(q.view(torch.uint8), ref.view(torch.uint8))
    assert torch.equal(qT.view(torch.uint8), ref.t().contiguous().view(torch.uint8))
    assert part is not None and part.shape == ((R + 63) // 64, C)
    blocks = torch.nn.functional.pad(x.float(), (0, 0, 0, part.shape[0] * 64 - R)).reshape(-1, 64, C).sum(1)
    torch.testing.assert_close(part, blocks, rtol=1e-5, atol=1e-3)
    db = torch.empty(C, dtype=torch.float32, device=DEV)
    N.native().colsum(0, part.data_ptr(), db.data_ptr(), part.shape[0], C, N.stream())
    torch.testing.assert_close(db, x.float().sum(0), rtol=1e-5, atol=1e-2)


def test_fp8_linear_bias_grad_from_fused_sums():
    """The fp8 linear's bias gradient (from the dY cast's column sums) equals dY summed over tokens in fp32."""
    import paddle2_amd as paddle
    from paddle2_amd.incubate.fp8 import Float8Linear

    paddle.set_device("gpu:0")
    paddle.seed(1)
    lin = Float8Linear(256, 512)
    lin.to(dtype="bfloat16")
    x = paddle.randn([3, 48, 256]).astype("bfloat16")   # 144 tokens: a partial 64-row block
    y = lin(x)
    g = torch.randn(y.shape, device=DEV, dtype=torch.bfloat16)
    y._t.backward(g)
    db = lin.bias.grad._t.float()
    torch.testing.assert_close(db, g.float().reshape(-1, 512).sum(0), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("hlen", [1, 4, 16, 64, 70])
def test_fp8_update_scale_matches_cpu_recipe(hlen):
    """The one-wave update kernel (slot fold, history roll, history max; serial beyond 64 entries) against the CPU
    path of FP8TensorMeta.update over several steps, including steps whose amax is zero."""
    from paddle2_amd.ops import fp8

    g = torch.Generator().manual_seed(hlen)
    gpu = fp8.FP8TensorMeta(torch.float8_e5m2, history_len=hlen, margin=1, device=torch.device(DEV))
    cpu = fp8.FP8TensorMeta(torch.float8_e5m2, history_len=hlen, margin=1)
    for step in range(hlen + 5):
        a = torch.rand(fp8.AMAX_SLOTS, generator=g) * (0 if step % 3 == 2 else 10.0 ** (step % 4))
        gpu.amax.copy_(a)
        cpu.amax.copy_(a)
        gpu.update()
        cpu.update()
        assert torch.equal(gpu.history.cpu(), cpu.history), step
        assert float(gpu.scale) == pytest.approx(float(cpu.scale), rel=1e-6)
        assert float(gpu.inv_scale) == pytest.approx(float(cpu.inv_scale), rel=1e-6)
        assert float(gpu.amax.abs().max()) == 0.0


def test_fp8_linear_matches_bf16():
    import paddle2_amd as paddle
    from paddle2_amd.incubate.fp8 import Float8Linear

    paddle.set_device("gpu:0")
    paddle.seed(0)
    lin = Float8Linear(256, 512)
    lin.to(dtype="bfloat16")
    x = paddle.randn([4, 64, 256]).astype("bfloat16")
    x.stop_gradient = False
    for _ in range(2):  # second pass uses history-derived scales
        y = lin(x)
    ref = torch.matmul(x._t.float(), lin.weight._t.float()) + lin.bias._t.float()
    rel = float((y._t.float() - ref).norm() / ref.norm())
    assert rel < 0.08, rel
    y.sum().backward()
    gw_ref = x._t.float().reshape(-1, 256).t() @ torch.ones(256, 512, device=DEV)
    relg = float((lin.weight.grad._t.float() - gw_ref).norm() / gw_ref.norm())
    assert relg < 0.1, relg


def test_gpt_fp8_trains_on_gpu():
    import paddle2_amd as paddle
    from paddle2_amd.models import GPTConfig, GPTForCausalLM

    paddle.set_device("gpu:0")
    paddle.seed(1)
    m = GPTForCausalLM(GPTConfig.tiny(use_fp8=True, hidden_size=256, intermediate_size=1024))
    o = paddle.optimizer.AdamW(1e-3, parameters=m.parameters(), multi_precision=True)
    ids = paddle.randint(0, 512, [4, 129])
    losses = []
    for _ in range(6):
        loss = m(ids[:, :-1], labels=ids[:, 1:])
        loss.backward()
        o.step()
        o.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0], losses


class _Slot:
    """A stand-in sharding unit: one fp32 main-grad slot per weight (grad_target / param_grad_done)."""

    def __init__(self, shape):
        self.buf = torch.full(shape, 0.25, device=DEV, dtype=torch.float32)
        self.done = 0

    def grad_target(self, i):
        return self.buf, 1   # accumulate onto the existing value (beta 1)

    def param_grad_done(self, i):
        self.done += 1


def test_fp8_wgrad_into_fp32_main_grad_slot(monkeypatch):
    """PADDLE2_AMD_FP8_WGRAD_MAIN: the native fp8 weight-gradient GEMM writes fp32 straight into the unit's slot
    (C = dW + 1 * C) — equal, up to the bf16 rounding the other path applies, to the bf16 dW + conversion."""
    from paddle2_amd.ops import fp8

    torch.manual_seed(0)
    K, Nn, M = 512, 768, 1024
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(K, Nn, device=DEV) * 0.05).bfloat16()
    g = torch.randn(M, Nn, device=DEV, dtype=torch.bfloat16)
    metas = [fp8.FP8TensorMeta(f, device=torch.device(DEV)) for f in (fp8.E4M3, fp8.E4M3, fp8.E5M2)]

    def run(main):
        monkeypatch.setattr(fp8, "WGRAD_MAIN", main)
        for m in metas:   # same scales for both runs
            m.initialized = False
            m.history.zero_()
            m.amax.zero_()
        wl = w.clone().requires_grad_()
        slot = _Slot((K, Nn))
        if main:
            wl._p2_gt = (slot, 0)
        y = fp8.fp8_linear(x, wl, None, *metas)
        y.backward(g)
        return wl.grad, slot

    gw_bf16, _ = run(False)
    gw_none, slot = run(True)
    assert gw_none is None and slot.done == 1
    ref = gw_bf16.float() + 0.25
    rel = float((slot.buf - ref).norm() / ref.norm())
    assert rel < 1e-2, rel
    exact = (x.float().t() @ g.float()) + 0.25
    assert float((slot.buf - exact).norm() / exact.norm()) < 0.08


def test_fp8_deferred_scale_updates_match_immediate(monkeypatch):
    """PADDLE2_AMD_FP8_DEFER: the per-linear delayed-scaling updates queued and launched 16 roles at a time (or when a
    queued role is cast again, or its state is read) give bit-identical outputs, gradients and scaling state to one
    update launch per linear.  8 chained linears = 24 roles per step, so both flush triggers fire."""
    from paddle2_amd.ops import fp8

    torch.manual_seed(3)
    L, K, M = 8, 256, 512
    ws = [(torch.randn(K, K, device=DEV) * 0.06).bfloat16() for _ in range(L)]
    xs = [torch.randn(M, K, device=DEV, dtype=torch.bfloat16) for _ in range(3)]

    def run(defer):
        monkeypatch.setattr(fp8, "DEFER_UPDATES", defer)
        metas = [[fp8.FP8TensorMeta(f, device=torch.device(DEV)) for f in (fp8.E4M3, fp8.E4M3, fp8.E5M2)]
                 for _ in range(L)]
        outs, grads = [], []
        for x in xs:
            wl = [w.clone().requires_grad_() for w in ws]
            h = x
            for w, m in zip(wl, metas):
                h = fp8.fp8_linear(h, w, None, *m)
            h.float().square().mean().backward()
            outs.append(h.detach())
            grads.append([w.grad for w in wl])
        fp8.flush_updates()
        state = [torch.cat([m.history, m.scale, m.inv_scale]) for ms in metas for m in ms]
        return outs, grads, state

    o1, g1, s1 = run(False)
    o2, g2, s2 = run(True)
    assert not fp8._PENDING
    for a, b in zip(o1, o2):
        assert torch.equal(a, b)
    for ga, gb in zip(g1, g2):
        for a, b in zip(ga, gb):
            assert torch.equal(a, b)
    for a, b in zip(s1, s2):
        assert torch.equal(a, b)


def test_fp8_scale_updates_captured_in_hip_graph():
    """Inside a HIP-graph capture the delayed-scaling updates are not queued: they are captured with the linear,
    so every replay rolls the history (a queue flushed after the capture would run once, eagerly)."""
    from paddle2_amd.ops import fp8

    torch.manual_seed(4)
    x = torch.randn(256, 256, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(256, 256, device=DEV) * 0.05).bfloat16()
    metas = [fp8.FP8TensorMeta(f, device=torch.device(DEV)) for f in (fp8.E4M3, fp8.E4M3, fp8.E5M2)]
    with torch.no_grad():
        for _ in range(2):   # warm-up: first-use init and the per-shape GEMM route outside the capture
            fp8.fp8_linear(x, w, None, *metas)
        fp8.flush_updates()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y = fp8.fp8_linear(x, w, None, *metas)
        assert not fp8._PENDING
        h = metas[0].history.clone()
        assert int((h > 0).sum()) == 2
        for k in range(3):
            g.replay()
            torch.cuda.synchronize()
            assert int((metas[0].history > 0).sum()) == 3 + k
    ref = x.float() @ w.float()
    assert float((y.float() - ref).norm() / ref.norm()) < 0.08


def test_fp8_capture_without_manual_flush_advances_once_per_replay():
    """eager warm-up steps leave deferred updates queued; paddle's CUDAGraph.capture_begin settles
    them first, so the captured graph holds only the capture's own update and each replay rolls the history once.
    A raw torch capture with updates still queued raises instead of recording the stale update."""
    from paddle2_amd.device import CUDAGraph
    from paddle2_amd.ops import fp8

    torch.manual_seed(5)
    x = torch.randn(256, 256, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(256, 256, device=DEV) * 0.05).bfloat16()
    metas = [fp8.FP8TensorMeta(f, device=torch.device(DEV)) for f in (fp8.E4M3, fp8.E4M3, fp8.E5M2)]
    with torch.no_grad():
        for _ in range(2):
            fp8.fp8_linear(x, w, None, *metas)
        assert fp8._PENDING, "the eager warm-up should leave its updates queued"
        g = CUDAGraph()
        g.capture_begin()
        y = fp8.fp8_linear(x, w, None, *metas)
        g.capture_end()
        assert not fp8._PENDING
        torch.cuda.synchronize()
        n0 = int((metas[0].history > 0).sum())
        assert n0 == 2
        for k in range(3):
            g.replay()
            torch.cuda.synchronize()
            assert int((metas[0].history > 0).sum()) == n0 + 1 + k
        # raw capture with a queue left by eager steps: refused
        fp8.fp8_linear(x, w, None, *metas)
        assert fp8._PENDING
        g2 = torch.cuda.CUDAGraph()
        with pytest.raises(RuntimeError, match="before_capture"):
            with torch.cuda.graph(g2):
                fp8.fp8_linear(x, w, None, *metas)
        fp8._PENDING.clear()
        fp8._PENDING_IDS.clear()
    ref = x.float() @ w.float()
    assert float((y.float() - ref).norm() / ref.norm()) < 0.08
