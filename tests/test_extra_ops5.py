"""Long-tail ops batch 5 vs plain fp32 loop references written from the reference kernels' semantics
(rank_attention.cu.h, qkv_unpack_mha_kernel.cu, match_matrix_tensor_kernel.cc, the fusion/cpu LoD fusions,
fused_scale_bias_relu_conv_bn_kernel.cu); parity with the reference binaries is unpinned (none run here)."""
import torch

import paddle2_amd as paddle
from paddle2_amd.ops import extra_ops as E
from paddle2_amd.ops import op_schema as S


def _lod(t, lens):
    x = paddle.to_tensor(t)
    off = [0]
    for n in lens:
        off.append(off[-1] + n)
    x._lod = [off]
    return x


def test_rank_attention_matches_loop():
    torch.manual_seed(0)
    N, D, P, R = 5, 3, 4, 3
    x = torch.randn(N, D)
    rp = torch.randn(R * R * D, P)
    ro = torch.zeros(N, 2 * R + 1, dtype=torch.int32)
    for i in range(N):
        ro[i, 0] = (i % R) + 1
        for k in range(R):
            if (i + k) % 4 != 3:
                ro[i, 2 * k + 1] = ((i + k) % R) + 1
                ro[i, 2 * k + 2] = (i * 2 + k) % N
    h, out, ins = E.rank_attention(paddle.to_tensor(x), paddle.to_tensor(ro), paddle.to_tensor(rp), max_rank=R)
    ref = torch.zeros(N, P)
    for i in range(N):
        for k in range(R):
            lo, pe = int(ro[i, 0]) - 1, int(ro[i, 2 * k + 1]) - 1
            if lo < 0 or pe < 0:
                continue
            blk = rp[(lo * R + pe) * D:(lo * R + pe + 1) * D]
            ref[i] += x[int(ro[i, 2 * k + 2])] @ blk
    assert torch.allclose(out._t, ref, atol=1e-5)
    assert ins._t.reshape(-1).tolist() == ro[:, 0].float().tolist() and h._t.shape == (N, R * D)


def test_qkv_unpack_mha_gqa_with_mask():
    torch.manual_seed(1)
    B, S_, Hq, Hk, D = 2, 7, 4, 2, 8
    q, k, v = torch.randn(B, 1, Hq, D), torch.randn(B, S_, Hk, D), torch.randn(B, S_, Hk, D)
    mask = torch.zeros(B, 1, 1, S_)
    mask[1, ..., 5:] = -1e9
    out = E.qkv_unpack_mha(paddle.to_tensor(q), paddle.to_tensor(k), paddle.to_tensor(v), paddle.to_tensor(mask))
    for b in range(B):
        for h in range(Hq):
            s = (k[b, :, h // 2] @ q[b, 0, h]) / D ** 0.5 + mask[b, 0, 0]
            ref = torch.softmax(s, 0) @ v[b, :, h // 2]
            assert torch.allclose(out._t[b, 0, h], ref, atol=1e-5)


def test_match_matrix_tensor():
    torch.manual_seed(2)
    D, T = 3, 2
    x = _lod(torch.randn(5, D), [2, 3])
    y = _lod(torch.randn(4, D), [3, 1])
    w = torch.randn(D, T, D)
    out, tmp = E.match_matrix_tensor(x, y, paddle.to_tensor(w), dim_t=T)
    ref = []
    for (a, b), (c, d) in (((0, 2), (0, 3)), ((2, 5), (3, 4))):
        for t in range(T):
            ref.append((x._t[a:b] @ w[:, t] @ y._t[c:d].t()).reshape(-1))
    assert torch.allclose(out._t.reshape(-1), torch.cat(ref), atol=1e-5)
    assert out._lod == [[0, 12, 18]]


def test_seqconv_eltadd_relu_and_seqexpand_concat_fc():
    torch.manual_seed(3)
    x = _lod(torch.randn(5, 2), [2, 3])
    filt, bias = torch.randn(3 * 2, 4), torch.randn(4)
    out, cols = E.fusion_seqconv_eltadd_relu(x, paddle.to_tensor(filt), paddle.to_tensor(bias), 3, -1)
    ref = torch.zeros(5, 4)
    for a, b in ((0, 2), (2, 5)):
        for t in range(a, b):
            win = [x._t[t + s] if a <= t + s < b else torch.zeros(2) for s in (-1, 0, 1)]
            ref[t] = torch.relu(torch.cat(win) @ filt + bias)
    assert torch.allclose(out._t, ref, atol=1e-5)
    x1 = torch.randn(2, 3)
    w = torch.randn(5, 4)
    o2, _ = E.fusion_seqexpand_concat_fc([x, paddle.to_tensor(x1)], paddle.to_tensor(w), None, "relu")
    rep = torch.cat([x1[0:1].expand(2, 3), x1[1:2].expand(3, 3)])
    assert torch.allclose(o2._t, torch.relu(torch.cat([x._t, rep], 1) @ w), atol=1e-5)


def test_fused_embedding_fc_lstm_equals_fusion_lstm_on_projected_rows():
    torch.manual_seed(4)
    V, H = 6, 3
    emb = torch.randn(V, 4 * H)
    ids = _lod(torch.tensor([[1], [4], [2], [0]]), [2, 2])
    wh, b = torch.randn(H, 4 * H), torch.randn(1, 4 * H)
    h, c = E.fused_embedding_fc_lstm(ids, paddle.to_tensor(emb), paddle.to_tensor(wh), paddle.to_tensor(b))
    proj = _lod(emb[ids._t.reshape(-1)], [2, 2])
    h2, _ = E.fusion_lstm(proj, paddle.to_tensor(torch.eye(4 * H)), paddle.to_tensor(wh), paddle.to_tensor(b))
    assert torch.allclose(h._t, h2._t, atol=1e-6) and h._t.shape == (4, H)


def test_attention_lstm_runs_and_is_bounded():
    torch.manual_seed(5)
    M, D = 3, 2
    x = _lod(torch.randn(4, M), [1, 3])
    h, c = E.attention_lstm(x, paddle.to_tensor(torch.zeros(2, D)), None, paddle.to_tensor(torch.randn(M + D, 1)),
                            None, None, None, paddle.to_tensor(torch.randn(M + D, 4 * D)),
                            paddle.to_tensor(torch.randn(1, 4 * D)))
    assert h._t.shape == (4, D) and bool((h._t.abs() < 1).all())
    # a one-step sequence attends only to itself: pooled == x row
    lw, lb = torch.randn(M + D, 4 * D), torch.randn(1, 4 * D)
    x1 = _lod(torch.randn(1, M), [1])
    h1, c1 = E.attention_lstm(x1, paddle.to_tensor(torch.zeros(1, D)), None,
                              paddle.to_tensor(torch.randn(M + D, 1)), None, None, None, paddle.to_tensor(lw),
                              paddle.to_tensor(lb))
    gf, gi, go, gc = (torch.cat([x1._t[0], torch.zeros(D)]) @ lw + lb[0]).chunk(4)
    cref = torch.sigmoid(gi) * torch.tanh(gc)
    assert torch.allclose(c1._t[0], cref, atol=1e-5)
    assert torch.allclose(h1._t[0], torch.sigmoid(go) * torch.tanh(cref), atol=1e-5)


def test_fused_scale_bias_relu_conv_bn():
    torch.manual_seed(6)
    x = torch.randn(2, 5, 5, 3)
    w = torch.randn(4, 3, 3, 3)   # OHWI
    sc, bi = torch.rand(3) + 0.5, torch.randn(3)
    g, bb = torch.rand(4) + 0.5, torch.randn(4)
    outs = E.fused_scale_bias_relu_conv_bn(*(paddle.to_tensor(t) for t in (x, w, sc, bi, g, bb, torch.zeros(4),
                                                                          torch.ones(4))), paddings=(1, 1))
    y = torch.nn.functional.conv2d(torch.relu(x * sc + bi).permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), padding=1)
    assert torch.allclose(outs[0]._t, y.permute(0, 2, 3, 1), atol=1e-4)
    bn = torch.nn.functional.batch_norm(y, None, None, g, bb, training=True, eps=1e-5)
    folded = y * outs[5]._t[None, :, None, None] + outs[6]._t[None, :, None, None]
    assert torch.allclose(folded, bn, atol=1e-4)


def test_yolo_box_post_shapes_and_alias():
    torch.manual_seed(7)
    C = 2
    heads = [paddle.to_tensor(torch.randn(1, 3 * (5 + C), s, s)) for s in (2, 4, 8)]
    out, num = E.yolo_box_post(*heads, paddle.to_tensor([[64, 64]]), paddle.to_tensor([[1.0, 1.0]]),
                               [10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119], [10, 13, 16, 30, 33, 23], C,
                               0.01, 32, 16, 8, True, 1.0, 0.45)
    assert out._t.shape[1] == 6 and int(num._t[0]) == out._t.shape[0] > 0
    assert set(out._t[:, 0].tolist()) <= {0.0, 1.0}
    for n in ("rank_attention", "qkv_unpack_mha", "yolo_box_post", "p_send_array", "attention_lstm"):
        assert S.resolve(n) is not None


def test_p_send_recv_array_two_ranks():
    from _dist import run_workers

    res = run_workers("p2p_array_worker.py", 2)
    assert res[1]["a"] == [[[0.0, 1.0, 2.0], [3.0, 4.0, 5.0]], [[1.0] * 3] * 2]
    assert res[1]["b_shapes"] == [[4], [2, 2, 2]] and res[1]["b_sum"] == [6.0, 24.0]
