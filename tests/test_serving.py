"""Serving runtime: decode attention (paged / MMHA layouts), block attention, fused multi-transformer,
and KV-cached generation == full-recompute greedy decoding (reference tests:
test/legacy_test/test_masked_multihead_attention_op.py, test_block_multihead_attention.py,
test_fused_multi_transformer_op.py).  Runs on CPU (reference paths) and, marked gpu, on the MI355X
through the HIP kernels."""
import math

import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd import serving

DEVS = ["cpu"] + (["cuda"] if torch.cuda.is_available() else [])


def _dense(q, K, V, scale):
    # q [Hq, D], K/V [L, Hk, D]
    Hq, Hk = q.shape[0], K.shape[1]
    G = Hq // Hk
    k = K.float().repeat_interleave(G, 1)
    v = V.float().repeat_interleave(G, 1)
    s = torch.einsum("hd,lhd->hl", q.float(), k) * scale
    return torch.einsum("hl,lhd->hd", torch.softmax(s, -1), v)


def _decode_case(dev, dtype, D, Hq, Hk, lens, bs=16):
    g = torch.Generator().manual_seed(0)
    B = len(lens)
    maxb = (max(lens) + bs - 1) // bs
    nblk = B * maxb + 3
    kc = torch.randn(nblk, bs, Hk, D, generator=g).to(dev, dtype)
    vc = torch.randn(nblk, bs, Hk, D, generator=g).to(dev, dtype)
    perm = torch.randperm(nblk, generator=g)[: B * maxb].reshape(B, maxb).to(dev, torch.int32)
    q = torch.randn(B, Hq, D, generator=g).to(dev, dtype)
    out = serving.decode_attention(q, kc, vc, torch.tensor(lens, dtype=torch.int32, device=dev), perm)
    for b, L in enumerate(lens):
        idx = torch.arange(L, device=dev)
        blocks = perm[b, idx // bs].long()
        K = kc[blocks, idx % bs]
        V = vc[blocks, idx % bs]
        ref = _dense(q[b], K, V, 1 / math.sqrt(D))
        torch.testing.assert_close(out[b].float(), ref, atol=2e-2, rtol=2e-2)


def test_decode_attention_paged_cpu():
    _decode_case("cpu", torch.float32, 64, 8, 2, [5, 37, 64])


@pytest.mark.gpu
@pytest.mark.parametrize("D,Hq,Hk", [(128, 32, 32), (128, 32, 8), (64, 16, 4), (128, 8, 1)])
@pytest.mark.parametrize("lens", [[1, 300, 4097], [64, 65]])
def test_decode_attention_paged_gpu(D, Hq, Hk, lens):
    _decode_case("cuda", torch.bfloat16, D, Hq, Hk, lens)


@pytest.mark.parametrize("dev", DEVS)
def test_masked_multihead_attention_cache(dev):
    if dev == "cuda":
        pytest.skip("covered by the gpu-marked variant")
    _mmha(dev, torch.float32)


@pytest.mark.gpu
def test_masked_multihead_attention_gpu():
    _mmha("cuda", torch.bfloat16)


def _mmha(dev, dt):
    b, nh, hd, max_s = 2, 4, 64, 32
    g = torch.Generator().manual_seed(1)
    cache = torch.zeros(2, b, nh, max_s, hd, dtype=dt, device=dev)
    ks, vs = [], []
    for t in range(5):
        x = torch.randn(b, 3 * nh * hd, generator=g).to(dev, dt)
        lens = torch.full((b, 1), t, dtype=torch.int32, device=dev)
        out, _ = serving.masked_multihead_attention(paddle.Tensor._wrap(x), paddle.Tensor._wrap(cache),
                                                    sequence_lengths=paddle.Tensor._wrap(lens))
        qkv = x.reshape(b, 3, nh, hd)
        ks.append(qkv[:, 1])
        vs.append(qkv[:, 2])
        K, V = torch.stack(ks, 1), torch.stack(vs, 1)  # [b, t+1, nh, hd]
        for bb in range(b):
            ref = _dense(qkv[bb, 0], K[bb], V[bb], 1 / math.sqrt(hd))
            torch.testing.assert_close(out._t[bb].reshape(nh, hd).float(), ref, atol=3e-2, rtol=3e-2)


def _tiny_llama(dev):
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    paddle.seed(3)
    cfg = LlamaConfig.tiny(num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                           dtype="bfloat16" if dev == "cuda" else "float32")
    m = LlamaForCausalLM(cfg)
    if dev == "cuda":
        m.to(device="gpu:0")
    m.eval()
    return m


def test_generation_matches_full_recompute_cpu():
    from paddle2_amd.serving.generation import LlamaGenerator, greedy_reference

    m = _tiny_llama("cpu")
    gen = LlamaGenerator(m, max_batch=2, max_seq_len=64, block_size=8, use_graph=False)
    prompts = [[1, 5, 9, 3], [7, 2]]
    outs = gen.generate(prompts, max_new_tokens=6)
    for p, o in zip(prompts, outs):
        assert o == greedy_reference(m, p, 6)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_packed_prefill_matches_per_prompt(dev):
    """prefill_batch (all prompts as one packed token batch, varlen attention, per-token RoPE positions) gives the
    per-prompt prefill's last-token logits and fills the same KV cache rows."""
    from paddle2_amd.serving.generation import LlamaGenerator

    if dev == "cuda":
        paddle.set_device("gpu:0")
    m = _tiny_llama(dev)
    prompts = [[1, 5, 9, 3, 11, 4, 2], [7, 2, 8], [4, 4, 1, 9, 13]]
    a = LlamaGenerator(m, max_batch=3, max_seq_len=64, block_size=8, use_graph=False)
    b = LlamaGenerator(m, max_batch=3, max_seq_len=64, block_size=8, use_graph=False)
    packed = a.prefill_batch([0, 1, 2], prompts)
    seq = torch.stack([b.prefill(i, torch.as_tensor(p)) for i, p in enumerate(prompts)])
    tol = dict(atol=2e-2, rtol=2e-2) if dev == "cuda" else dict(atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(packed.float(), seq.float(), **tol)
    assert torch.equal(a.cache.seq_lens[:3].cpu(), b.cache.seq_lens[:3].cpu())
    for li in range(len(a.cache.k)):
        for i, p in enumerate(prompts):
            for t in range(len(p)):
                blk_a = a.cache.block_table[i, t // 8]
                blk_b = b.cache.block_table[i, t // 8]
                torch.testing.assert_close(a.cache.k[li][blk_a, t % 8].float(), b.cache.k[li][blk_b, t % 8].float(),
                                           **tol)


def test_generation_transposed_weight_layout_cpu():
    """weight_layout="nk" (the GPU default: cached W^T per projection) generates the same tokens, and the
    cache follows in-place weight updates (version bump)."""
    from paddle2_amd.serving.generation import LlamaGenerator, greedy_reference

    m = _tiny_llama("cpu")
    gen = LlamaGenerator(m, max_batch=2, max_seq_len=64, block_size=8, use_graph=False, weight_layout="nk")
    prompts = [[1, 5, 9, 3], [7, 2]]
    assert gen.generate(prompts, max_new_tokens=6) == [greedy_reference(m, p, 6) for p in prompts]
    assert len(gen._wt) > 0
    w = m.lm_head.weight
    with torch.no_grad():
        w._t.mul_(-1.0)
    gen2 = LlamaGenerator(m, max_batch=2, max_seq_len=64, block_size=8, use_graph=False, weight_layout="nk")
    gen2._wt = gen._wt
    assert gen2.generate(prompts[:1], max_new_tokens=4) == [greedy_reference(m, prompts[0], 4)]


@pytest.mark.gpu
def test_generation_hip_graph_gpu():
    from paddle2_amd.serving.generation import LlamaGenerator, greedy_reference

    paddle.set_device("gpu:0")
    m = _tiny_llama("cuda")
    prompts = [[1, 5, 9, 3, 11, 4], [7, 2, 8]]
    eager = LlamaGenerator(m, max_batch=2, max_seq_len=128, block_size=16, use_graph=False).generate(prompts, 8)
    graph = LlamaGenerator(m, max_batch=2, max_seq_len=128, block_size=16, use_graph=True).generate(prompts, 8)
    assert eager == graph
    # bf16 rounding can flip near-ties late in the sequence: require the first tokens to agree
    for p, o in zip(prompts, eager):
        ref = greedy_reference(m, p, 8)
        assert o[:3] == ref[:3], (o, ref)


@pytest.mark.gpu
def test_generation_graph_follows_weight_update_gpu():
    """A captured decode graph reads the cached W^T buffers; an in-place weight update between two generate()
    calls is re-transposed into those same buffers, so the replayed graph uses the new weights (no stale /
    freed W^T)."""
    from paddle2_amd.serving.generation import LlamaGenerator, greedy_reference

    paddle.set_device("gpu:0")
    m = _tiny_llama("cuda")
    prompts = [[1, 5, 9, 3, 11, 4], [7, 2, 8]]
    gen = LlamaGenerator(m, max_batch=2, max_seq_len=128, block_size=16, use_graph=True, weight_layout="nk")
    gen.generate(prompts, 6)
    assert gen._graph is not None
    bufs = {k: v[2].data_ptr() for k, v in gen._wt.items()}
    with torch.no_grad():
        m.lm_head.weight._t.mul_(-1.0)
        m.llama.layers[0].mlp.down_proj.weight._t.mul_(0.5)
    out = gen.generate(prompts, 6)
    assert {k: v[2].data_ptr() for k, v in gen._wt.items()} == bufs   # updated in place, same addresses
    eager = LlamaGenerator(m, max_batch=2, max_seq_len=128, block_size=16, use_graph=False,
                           weight_layout="nk").generate(prompts, 6)   # same GEMM kernels, fresh W^T copies
    assert out == eager
    for p, o in zip(prompts, out):
        assert o[:3] == greedy_reference(m, p, 6)[:3]


@pytest.mark.gpu
def test_decode_step_runs_the_native_decode_gemm_gpu(monkeypatch):
    """The decode step's [B, 1, K] hidden states (and a short prompt's rows) reach the native weight-streaming GEMM
    flattened to [rows, K], and the tokens match the hipBLASLt ("kn") layout."""
    from paddle2_amd.ops import weight_only as WO
    from paddle2_amd.serving.generation import LlamaGenerator

    paddle.set_device("gpu:0")
    m = _tiny_llama("cuda")
    prompts = [[1, 5, 9, 3, 11, 4], [7, 2, 8]]
    monkeypatch.setattr(WO, "DECODE_GEMM", "native")
    native_calls = []
    real = WO.decode_matmul

    def counting(x, wt, bias=None):
        if WO.decode_ok(x, wt):
            native_calls.append(tuple(x.shape))
        return real(x, wt, bias)

    monkeypatch.setattr(WO, "decode_matmul", counting)
    out = LlamaGenerator(m, max_batch=2, max_seq_len=128, block_size=16, use_graph=False,
                         weight_layout="nk").generate(prompts, 6)
    assert (2, 256) in native_calls   # the B = 2 decode rows
    eager = LlamaGenerator(m, max_batch=2, max_seq_len=128, block_size=16, use_graph=False,
                           weight_layout="kn").generate(prompts, 6)
    for a, b in zip(out, eager):
        assert a[:3] == b[:3]


def test_static_mm_cache_lives_on_the_weight():
    """fused_multi_transformer's W^T copies hang off the weight tensor (no module-global cache pinning weights)
    and follow in-place updates; clear_static_weight_cache drops them."""
    import gc
    import weakref

    from paddle2_amd.serving import _static_mm, clear_static_weight_cache

    if not torch.cuda.is_available():
        w = torch.randn(8, 4)
        x = torch.randn(3, 8)
        torch.testing.assert_close(_static_mm(x, w), x @ w)   # CPU: plain matmul, nothing attached
        assert not hasattr(w, "_pd_wt")
        return
    w = torch.randn(64, 32, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(5, 64, device="cuda", dtype=torch.bfloat16)
    torch.testing.assert_close(_static_mm(x, w).float(), (x.float() @ w.float()), atol=5e-2, rtol=2e-2)
    buf = w._pd_wt[1].data_ptr()
    with torch.no_grad():
        w.mul_(2.0)
    torch.testing.assert_close(_static_mm(x, w).float(), (x.float() @ w.float()), atol=1e-1, rtol=2e-2)
    assert w._pd_wt[1].data_ptr() == buf
    ref = weakref.ref(w)
    del w
    gc.collect()
    assert ref() is None   # nothing global kept the weight alive
    w2 = torch.randn(64, 32, device="cuda", dtype=torch.bfloat16)
    _static_mm(x, w2)
    clear_static_weight_cache(w2)
    assert not hasattr(w2, "_pd_wt")


@pytest.mark.gpu
def test_fused_multi_transformer_gpu_matches_cpu():
    """The GPU fused_multi_transformer (cached W^T projections, native decode kernels) matches the CPU op."""
    from paddle2_amd.incubate.nn import FusedMultiTransformer

    prev = paddle.get_device()
    try:
        paddle.set_device("cpu")    # the reference pass on the CPU op (the default device on a GPU box is gpu:0)
        paddle.seed(0)
        layer = FusedMultiTransformer(128, 4, 256, num_layers=2, activation="gelu")
        b, s, nh, hd = 2, 6, 4, 32
        x = paddle.randn([b, s, 128])
        caches = [paddle.zeros([2, b, nh, 16, hd]) for _ in range(2)]
        ref, _ = layer(x, caches=caches)
        assert ref._t.device.type == "cpu"
        paddle.set_device("gpu:0")
        layer.to(device="gpu:0")
        xg = paddle.to_tensor(x._t.cuda())
        cg = [paddle.zeros([2, b, nh, 16, hd]) for _ in range(2)]
        out, _ = layer(xg, caches=cg)
        assert out._t.is_cuda
    finally:
        paddle.set_device(prev)
    torch.testing.assert_close(out._t.float().cpu(), ref._t.float(), atol=2e-3, rtol=2e-3)


def test_fused_multi_transformer_decode_matches_context():
    from paddle2_amd.incubate.nn import FusedMultiTransformer

    paddle.seed(0)
    layer = FusedMultiTransformer(64, 4, 128, num_layers=2, activation="gelu")
    b, s, nh, hd = 2, 6, 4, 16
    x = paddle.randn([b, s, 64])
    caches = [paddle.zeros([2, b, nh, 16, hd]) for _ in range(2)]
    full, _ = layer(x, caches=caches)  # context phase over all s tokens
    caches2 = [paddle.zeros([2, b, nh, 16, hd]) for _ in range(2)]
    ctx, _ = layer(x[:, : s - 1], caches=caches2)
    last, _ = layer(x[:, s - 1:], caches=caches2, time_step=s - 1)
    torch.testing.assert_close(last._t[:, 0], full._t[:, -1], atol=1e-4, rtol=1e-4)


def test_tensor_parallel_fused_inference_ops_match_single_rank():
    """ring_id all-reduce in fused_multi_transformer (context + decode), fused_feedforward and
    fused_multi_head_attention: 2 gloo ranks with head / ffn shards == 1 rank with the full weights."""
    from _dist import run_workers

    for r in run_workers("tp_infer_worker.py", 2):
        assert r["fmt_diff"] < 1e-4 and r["ffn_diff"] < 1e-4 and r["mha_diff"] < 1e-4, r
        assert r["bad_ring"] == "raised", r


@pytest.mark.gpu
@pytest.mark.parametrize("impl", [1, 2])
@pytest.mark.parametrize("D,Hq,Hk", [(128, 32, 32), (128, 32, 8), (128, 8, 1), (128, 32, 2)])
def test_decode_attention_kernels_gpu(impl, D, Hq, Hk, monkeypatch):
    """vector (1) and MFMA (2) decode kernels, forced, vs fp32 (lens straddle the 32-key tiles and the splits)."""
    monkeypatch.setattr(serving, "_DECODE_IMPL", impl)
    _decode_case("cuda", torch.bfloat16, D, Hq, Hk, [1, 31, 33, 300, 4097])


@pytest.mark.gpu
def test_decode_step_folds_swiglu_into_down_gemm_gpu(monkeypatch):
    """Decode rows (<= 16) run the down projection on the SwiGLU-staged decode GEMM (no separate SwiGLU pass);
    tokens match the unfused path."""
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM
    from paddle2_amd.ops import weight_only as WO
    from paddle2_amd.serving.generation import LlamaGenerator

    paddle.set_device("gpu:0")
    paddle.seed(3)
    cfg = LlamaConfig.tiny(num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, intermediate_size=704,
                           dtype="bfloat16")
    m = LlamaForCausalLM(cfg)
    m.to(device="gpu:0")
    m.eval()
    prompts = [[1, 5, 9, 3, 11, 4], [7, 2, 8]]
    calls = []
    real, real_part = WO.decode_glu_matmul, WO.decode_glu_partials

    def counting(gu, wt):
        calls.append(tuple(gu.shape))
        return real(gu, wt)

    def counting_part(gu, wt, shape):
        calls.append(tuple(gu.shape))
        return real_part(gu, wt, shape)

    monkeypatch.setattr(WO, "decode_glu_matmul", counting)
    monkeypatch.setattr(WO, "decode_glu_partials", counting_part)
    fused = LlamaGenerator(m, max_batch=2, max_seq_len=128, block_size=16, use_graph=False,
                           weight_layout="nk").generate(prompts, 6)
    assert (2, 2 * 704) in calls
    graph = LlamaGenerator(m, max_batch=2, max_seq_len=128, block_size=16, use_graph=True,
                           weight_layout="nk").generate(prompts, 6)
    assert graph == fused   # the captured decode step replays the fused kernel
    monkeypatch.setattr(WO, "decode_glu_ok", lambda gu, wt: False)
    plain = LlamaGenerator(m, max_batch=2, max_seq_len=128, block_size=16, use_graph=False,
                           weight_layout="nk").generate(prompts, 6)
    for a, b in zip(fused, plain):
        assert a[:3] == b[:3]


@pytest.mark.gpu
def test_decode_partials_handoff_bit_identical_gpu(monkeypatch):
    """Decode rows' o / down projections hand their split-K partials to the residual-add + RMSNorm that consumes them
    (no reduce launch): the decode logits are bit-identical to the path with the reduce launch, eager and graphed,
    and the norm sums them exactly like the reduce kernel (rms_norm_partials vs reduce + rms_norm)."""
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM
    from paddle2_amd.ops import torch_ops as T
    from paddle2_amd.ops import weight_only as WO
    from paddle2_amd.serving.generation import LlamaGenerator

    paddle.set_device("gpu:0")
    paddle.seed(5)
    cfg = LlamaConfig.tiny(num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, intermediate_size=704,
                           dtype="bfloat16")
    m = LlamaForCausalLM(cfg)
    m.to(device="gpu:0")
    m.eval()
    toks = torch.tensor([3, 9], device="cuda")
    pos = torch.tensor([5, 2], dtype=torch.int32, device="cuda")
    logits = {}
    for graph in (False, True):
        for on in (True, False):
            monkeypatch.setattr(WO, "PARTIALS", on)
            gen = LlamaGenerator(m, max_batch=2, max_seq_len=64, block_size=16, use_graph=graph, weight_layout="nk")
            for i in range(2):
                gen.cache.allocate(i, 16)
            logits[(graph, on)] = gen.decode_step(toks, pos).clone()
    for graph in (False, True):
        assert torch.equal(logits[(graph, True)], logits[(graph, False)])
    # the op on its own: random partials of 1..16 rows, bf16 and fp32 norm weights
    g = torch.Generator(device="cuda").manual_seed(0)
    for M, Nn, S, wdt in ((1, 4096, 4, torch.bfloat16), (16, 4096, 3, torch.float32), (5, 1024, 1, torch.bfloat16)):
        ws = torch.randn(S * M * Nn, device="cuda", generator=g)
        p = WO.DecodePartials(ws, S, M, Nn, (M, 1, Nn), torch.bfloat16)
        res = torch.randn(M, 1, Nn, device="cuda", generator=g).to(torch.bfloat16)
        w = torch.rand(Nn, device="cuda", generator=g).to(wdt)
        y, h = T.rms_norm_partials(p, w, 1e-5, res)
        y2, h2 = T.rms_norm(p.materialize(), w, 1e-5, res)
        assert torch.equal(h, h2) and torch.equal(y, y2)
