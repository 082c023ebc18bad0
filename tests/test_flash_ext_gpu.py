"""Varlen (cu_seqlens) and FlashMask variants of the MFMA flash-attention kernels vs. fp32 references.

Reference behaviour: flash_attn_unpadded (python/paddle/nn/functional/flash_attention.py:652) and
flashmask_attention (:1098, mask semantics of its flashmask_to_densemask docstring)."""
import pytest
import torch

from paddle2_amd.ops import torch_ops as T

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _close(a, b, atol, rtol, what=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"{what}: max abs err {err} > {tol}"


def _rand(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g).to(torch.bfloat16).float()


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("lens_q,lens_k,Hq,Hk", [([100, 300, 1, 513], None, 4, 2),
                                                  ([64, 256, 17], [128, 256, 40], 2, 2)])
def test_flash_varlen(causal, D, lens_q, lens_k, Hq, Hk):
    lens_k = lens_k or lens_q
    cu_q = torch.tensor([0] + list(torch.tensor(lens_q).cumsum(0)), dtype=torch.int32)
    cu_k = torch.tensor([0] + list(torch.tensor(lens_k).cumsum(0)), dtype=torch.int32)
    tq, tk = int(cu_q[-1]), int(cu_k[-1])
    q, k, v = _rand((tq, Hq, D), 1), _rand((tk, Hk, D), 2), _rand((tk, Hk, D), 3)
    go = _rand((tq, Hq, D), 4)
    qg, kg, vg = (t.to(DEV, torch.bfloat16).requires_grad_(True) for t in (q, k, v))
    og, lg = T.flash_attention_varlen(qg, kg, vg, cu_q.to(DEV), cu_k.to(DEV), max(lens_q), max(lens_k), causal)
    og.backward(go.to(DEV, torch.bfloat16))
    # per-sequence fp32 reference
    for i in range(len(lens_q)):
        a, b, c, d = int(cu_q[i]), int(cu_q[i + 1]), int(cu_k[i]), int(cu_k[i + 1])
        qc, kc, vc = (t.clone().requires_grad_(True) for t in (q[a:b], k[c:d], v[c:d]))
        oc, lc = T._attn_reference(qc[None], kc[None], vc[None], causal, D ** -0.5)
        oc.backward(go[a:b][None])
        _close(og[a:b], oc[0], 2e-2, 2e-2, f"out seq {i}")
        fin = torch.isfinite(lc[0])
        _close(lg[:, a:b].cpu()[fin], lc[0][fin], 1e-2, 1e-3, f"lse seq {i}")
        _close(qg.grad[a:b], qc.grad, 5e-2, 3e-2, f"dq seq {i}")
        _close(kg.grad[c:d], kc.grad, 5e-2, 3e-2, f"dk seq {i}")
        _close(vg.grad[c:d], vc.grad, 5e-2, 3e-2, f"dv seq {i}")


def _doc_mask(B, S, Hm, causal, n, seed):
    """Random document / sliding / global masks in startend_row_indices form."""
    g = torch.Generator().manual_seed(seed)
    j = torch.arange(S)
    if causal and n == 1:       # causal document mask: key j masked from the end of its document down
        bounds = torch.sort(torch.randint(1, S, (B, Hm, 3), generator=g), -1).values
        ends = torch.cat([bounds, torch.full((B, Hm, 1), S)], -1)
        idx = torch.gather(ends, -1, torch.searchsorted(ends, j.expand(B, Hm, S).contiguous(), right=True))
        return idx[..., None]
    if causal and n == 2:       # causal blockwise: [LTS, LTE)
        lts = (j + torch.randint(1, S // 2, (B, Hm, 1), generator=g)).clamp(max=S)
        lte = (lts + torch.randint(0, S, (B, Hm, S), generator=g)).clamp(max=S)
        return torch.stack([lts, lte], -1)
    if not causal and n == 2:   # sliding window both sides: LTS, UTE
        w = int(torch.randint(8, S // 2, (1,), generator=g))
        lts = (j + w + 1).clamp(max=S).expand(B, Hm, S)
        ute = (j - w).clamp(min=0).expand(B, Hm, S)
        return torch.stack([lts, ute], -1)
    lts = (j + torch.randint(16, S, (B, Hm, 1), generator=g)).clamp(max=S)     # global + window, 4 bounds
    lte = torch.full((B, Hm, S), S)
    uts = torch.randint(0, S // 4, (B, Hm, S), generator=g)
    ute = (uts + torch.randint(0, S // 2, (B, Hm, S), generator=g)).clamp(max=S)
    return torch.stack([lts, lte, uts, ute], -1)


@pytest.mark.parametrize("causal,n", [(True, 1), (True, 2), (False, 2), (False, 4)])
@pytest.mark.parametrize("D,S,Hq,Hk,Hm", [(128, 640, 4, 2, 1), (64, 333, 2, 2, 2), (128, 1024, 2, 1, 2)])
def test_flashmask(causal, n, D, S, Hq, Hk, Hm):
    B = 2
    q, k, v = _rand((B, S, Hq, D), 5), _rand((B, S, Hk, D), 6), _rand((B, S, Hk, D), 7)
    go = _rand((B, S, Hq, D), 8)
    idx = _doc_mask(B, S, Hm, causal, n, seed=S + n).to(torch.int32)
    qg, kg, vg = (t.to(DEV, torch.bfloat16).requires_grad_(True) for t in (q, k, v))
    og, lg = T.flash_attention_mask(qg, kg, vg, idx.to(DEV), causal)
    og.backward(go.to(DEV, torch.bfloat16))
    qc, kc, vc = (t.clone().requires_grad_(True) for t in (q, k, v))
    fm = T.flashmask_intervals(idx, causal)
    oc, lc = T._attn_reference_masked(qc, kc, vc, causal, D ** -0.5, fm)
    oc.backward(go)
    _close(og, oc, 2e-2, 2e-2, "out")
    fin = torch.isfinite(lc)
    _close(lg.cpu()[fin], lc[fin], 1e-2, 1e-3, "lse")
    _close(qg.grad, qc.grad, 5e-2, 3e-2, "dq")
    _close(kg.grad, kc.grad, 5e-2, 3e-2, "dk")
    _close(vg.grad, vc.grad, 5e-2, 3e-2, "dv")


def test_flashmask_window_api():
    """paddle.nn.functional.flashmask_attention(window_size=...) lowers to row ranges (reference :1698-1722)."""
    import paddle2_amd as paddle
    import paddle2_amd.nn.functional as F

    paddle.set_device("gpu:0")
    B, S, H, D = 1, 512, 2, 128
    q, k, v = (paddle.Tensor._wrap(_rand((B, S, H, D), s).to(DEV, torch.bfloat16)) for s in (9, 10, 11))
    out = F.flashmask_attention(q, k, v, window_size=64, causal=True)
    i = torch.arange(S)
    dense = (i[None, :] > i[:, None]) | (i[None, :] < i[:, None] - 64)  # masked where key outside [i-64, i]
    bias = torch.zeros(S, S).masked_fill(dense, float("-inf"))
    ref = torch.nn.functional.scaled_dot_product_attention(
        q._t.float().cpu().transpose(1, 2), k._t.float().cpu().transpose(1, 2), v._t.float().cpu().transpose(1, 2),
        attn_mask=bias).transpose(1, 2)
    _close(out._t, ref, 2e-2, 2e-2, "window")


@pytest.mark.parametrize("P", [2, 4])
def test_ring_attention_block_algebra(P):
    """The zigzag ring schedule of context_parallel.ring_flash_attention, simulated for P virtual ranks in one
    process on the native block primitives (flash fwd with lse merge; flash bwd with the final out / lse)."""
    from paddle2_amd.distributed.fleet.meta_parallel import context_parallel as CP

    B, S, Hq, Hk, D = 1, 256 * P, 4, 2, 128
    q, k, v = _rand((B, S, Hq, D), 20), _rand((B, S, Hk, D), 21), _rand((B, S, Hk, D), 22)
    go = _rand((B, S, Hq, D), 23)
    qc, kc, vc = (t.clone().requires_grad_(True) for t in (q, k, v))
    oc, _ = T._attn_reference(qc, kc, vc, True, D ** -0.5)
    oc.backward(go)
    dev = lambda t: t.to(DEV, torch.bfloat16)  # noqa: E731
    sh = [[CP.zigzag_shard(dev(t), P, r) for r in range(P)] for t in (q, k, v, go)]
    c = S // P // 2
    outs, lses = [], []
    for r in range(P):
        ql = sh[0][r]
        out = torch.zeros(ql.shape, dtype=torch.float32, device=DEV)
        lse = torch.full((B, Hq, ql.shape[1]), float("-inf"), device=DEV)
        for i in range(P):
            src = (r - i) % P
            kk, vv = sh[1][src], sh[2][src]
            kind = CP._step_kind(i, r, P)
            if kind == 0:
                CP._merge(out, lse, *T.attn_block_fwd(ql, kk, vv, True, D ** -0.5))
            elif kind == 1:
                CP._merge(out, lse, *T.attn_block_fwd(ql, kk[:, :c], vv[:, :c], False, D ** -0.5))
            else:
                CP._merge(out, lse, *T.attn_block_fwd(ql[:, c:], kk, vv, False, D ** -0.5), slice(c, 2 * c))
        outs.append(out.to(torch.bfloat16))
        lses.append(lse)
    _close(CP.zigzag_unshard(outs), oc, 2e-2, 2e-2, "ring out")
    dq = [torch.zeros(sh[0][r].shape, device=DEV) for r in range(P)]
    dk = [torch.zeros(sh[1][r].shape, device=DEV) for r in range(P)]
    dv = [torch.zeros(sh[2][r].shape, device=DEV) for r in range(P)]
    for r in range(P):
        ql, o, do, l = sh[0][r], outs[r], sh[3][r], lses[r]
        for i in range(P):
            src = (r - i) % P
            kk, vv = sh[1][src], sh[2][src]
            kind = CP._step_kind(i, r, P)
            if kind == 0:
                a, b, e = T.attn_block_bwd(ql, kk, vv, o, do, l, True, D ** -0.5)
                dq[r] += a.float(); dk[src] += b.float(); dv[src] += e.float()  # noqa: E702
            elif kind == 1:
                a, b, e = T.attn_block_bwd(ql, kk[:, :c], vv[:, :c], o, do, l, False, D ** -0.5)
                dq[r] += a.float(); dk[src][:, :c] += b.float(); dv[src][:, :c] += e.float()  # noqa: E702
            else:
                a, b, e = T.attn_block_bwd(ql[:, c:], kk, vv, o[:, c:], do[:, c:], l[:, :, c:].contiguous(), False,
                                           D ** -0.5)
                dq[r][:, c:] += a.float(); dk[src] += b.float(); dv[src] += e.float()  # noqa: E702
    _close(CP.zigzag_unshard(dq), qc.grad, 5e-2, 3e-2, "ring dq")
    _close(CP.zigzag_unshard(dk), kc.grad, 5e-2, 3e-2, "ring dk")
    _close(CP.zigzag_unshard(dv), vc.grad, 5e-2, 3e-2, "ring dv")


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D,Hq,Hk,Sq,Sk", [(128, 4, 2, 300, 300), (64, 2, 2, 200, 333)])
def test_flash_dropout_dense(causal, D, Hq, Hk, Sq, Sk):
    """In-kernel dropout (DROP variant) vs. an fp32 reference that applies the bit-identical host mask."""
    B, p, seed = 2, 0.2, 0x1234ABCD
    q, k, v = _rand((B, Sq, Hq, D), 11), _rand((B, Sk, Hk, D), 12), _rand((B, Sk, Hk, D), 13)
    go = _rand((B, Sq, Hq, D), 14)
    qg, kg, vg = (t.to(DEV, torch.bfloat16).requires_grad_(True) for t in (q, k, v))
    og, lg = T.flash_attention_dropout(qg, kg, vg, p, causal, seed32=seed)
    og.backward(go.to(DEV, torch.bfloat16))
    keep = T.attn_dropout_mask(seed, B, Hq, Sq, Sk, p)
    assert abs(1.0 - keep.float().mean().item() - p) < 0.01
    qc, kc, vc = (t.clone().requires_grad_(True) for t in (q, k, v))
    oc, lc = T._attn_reference_dropout(qc, kc, vc, causal, D ** -0.5, keep, p)
    oc.backward(go)
    _close(og, oc, 2e-2, 2e-2, "out")
    _close(lg.cpu(), lc, 1e-2, 1e-3, "lse (undropped row sums)")
    _close(qg.grad, qc.grad, 5e-2, 3e-2, "dq")
    _close(kg.grad, kc.grad, 5e-2, 3e-2, "dk")
    _close(vg.grad, vc.grad, 5e-2, 3e-2, "dv")
    # same seed => same output (mask regenerated, not drawn from a stream)
    o2, _ = T.flash_attention_dropout(qg.detach(), kg.detach(), vg.detach(), p, causal, seed32=seed)
    assert torch.equal(o2, og.detach())


def test_flash_dropout_varlen():
    D, Hq, p, seed = 128, 2, 0.3, 99
    lens = [70, 257, 130]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    tot = int(cu[-1])
    q, k, v, go = (_rand((tot, Hq, D), 20 + i) for i in range(4))
    qg, kg, vg = (t.to(DEV, torch.bfloat16).requires_grad_(True) for t in (q, k, v))
    og, _ = T.flash_attention_varlen(qg, kg, vg, cu.to(DEV), cu.to(DEV), max(lens), max(lens), True, dropout=p,
                                     seed32=seed)
    og.backward(go.to(DEV, torch.bfloat16))
    qc, kc, vc = (t.clone().requires_grad_(True) for t in (q, k, v))
    oc, _ = T.flash_attention_varlen(qc, kc, vc, cu, cu, max(lens), max(lens), True, dropout=p, seed32=seed)
    oc.backward(go)
    _close(og, oc, 2e-2, 2e-2, "out")
    _close(qg.grad, qc.grad, 5e-2, 3e-2, "dq")
    _close(kg.grad, kc.grad, 5e-2, 3e-2, "dk")
    _close(vg.grad, vc.grad, 5e-2, 3e-2, "dv")


@pytest.mark.parametrize("causal", [False, True])
def test_flash_running_max_jumps(causal):
    """Late keys with much larger scores force the deferred-max rescale branch (running max jumps mid-row)."""
    B, S, H, D = 1, 512, 2, 128
    q, k, v, go = (_rand((B, S, H, D), 30 + i) for i in range(4))
    k[:, 300:310] *= 12.0  # score spike past the first key tiles
    k[:, 450] *= 20.0
    qg, kg, vg = (t.to(DEV, torch.bfloat16).requires_grad_(True) for t in (q, k, v))
    og, lg = T.flash_attention(qg, kg, vg, causal)
    og.backward(go.to(DEV, torch.bfloat16))
    qc, kc, vc = (t.clone().requires_grad_(True) for t in (q, k, v))
    oc, lc = T._attn_reference(qc, kc, vc, causal, D ** -0.5)
    oc.backward(go)
    _close(og, oc, 2e-2, 2e-2, "out")
    _close(lg.cpu(), lc, 5e-2, 1e-3, "lse")
    _close(qg.grad, qc.grad, 1e-1, 3e-2, "dq")
    _close(kg.grad, kc.grad, 1e-1, 3e-2, "dk")
    _close(vg.grad, vc.grad, 5e-2, 3e-2, "dv")
