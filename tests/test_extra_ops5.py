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


def test_tdm_sampler_structure():
    # tree: layer 1 nodes 1..2, layer 2 nodes 3..6; travel rows are per-item positive paths
    travel = torch.tensor([[1, 3], [2, 6], [1, 0]])
    layer = torch.tensor([1, 2, 3, 4, 5, 6])
    out, lab, msk = E.tdm_sampler(paddle.to_tensor(torch.tensor([0, 1, 2])), paddle.to_tensor(travel),
                                  paddle.to_tensor(layer), True, [1, 2], [0, 2, 6], seed=3)
    o, l, m = out._t.tolist(), lab._t.tolist(), msk._t.tolist()
    assert o[0][0] == 1 and l[0][:2] == [1, 0] and o[0][1] == 2
    assert o[0][2] == 3 and set(o[0][3:]) <= {4, 5, 6} and len(set(o[0][3:])) == 2
    assert o[2][2:] == [0, 0, 0] and m[2][2:] == [0, 0, 0] and m[1] == [1] * 5


def test_detection_map_perfect_and_half():
    gt = _lod(torch.tensor([[1, 0, .1, .1, .4, .4], [1, 0, .5, .5, .9, .9]]), [2])
    det = _lod(torch.tensor([[1, .9, .1, .1, .4, .4], [1, .8, .5, .5, .9, .9]]), [2])
    *_, m = E.detection_map(det, gt, class_num=2)
    assert abs(float(m._t[0]) - 1.0) < 1e-6
    det2 = _lod(torch.tensor([[1, .9, .1, .1, .4, .4], [1, .8, .0, .6, .1, .7]]), [2])
    pc, tp, fp, m2 = E.detection_map(det2, gt, class_num=2)
    assert abs(float(m2._t[0]) - 0.5) < 1e-6 and pc._t.reshape(-1).tolist() == [0, 2]
    # accumulated state: the second batch equals the first -> same AP
    *_, m3 = E.detection_map(det2, gt, paddle.to_tensor([1]), pc, tp, fp, class_num=2)
    assert abs(float(m3._t[0]) - 0.5) < 1e-6
    *_, m4 = E.detection_map(det2, gt, class_num=2, ap_type="11point")
    assert abs(float(m4._t[0]) - 6 / 11) < 1e-6


def test_faster_tokenizer_wordpiece():
    voc = {t: i for i, t in enumerate(["[PAD]", "[UNK]", "[CLS]", "[SEP]", "hello", "world", "un", "##aff",
                                       "##able", ",", "!"])}
    ids, seg = E.faster_tokenizer(voc, ["Hello, unaffable world!"], ["hello"], do_lower_case=True,
                                  max_seq_len=12, pad_to_max_seq_len=True)
    assert ids._t.tolist()[0] == [2, 4, 9, 6, 7, 8, 5, 10, 3, 4, 3, 0]
    assert seg._t.tolist()[0] == [0] * 9 + [1, 1, 0]
    ids2, _ = E.faster_tokenizer(voc, ["xyz hello"])
    assert ids2._t.tolist()[0] == [2, 1, 4, 3]


def test_fusion_group_and_pyramid_hash_and_lamb_init():
    E.register_fusion_group("fg_axpy", lambda a, b: (a * 2 + b, torch.relu(a - b)))
    a, b = torch.randn(4), torch.randn(4)
    o1, o2 = E.fusion_group([paddle.to_tensor(a), paddle.to_tensor(b)], [0, 2], func_name="fg_axpy")
    assert torch.allclose(o1._t, a * 2 + b) and o2._t.dtype == torch.bfloat16
    x = _lod(torch.tensor([[3], [5], [7], [1]], dtype=torch.int32), [3, 1])
    w = torch.randn(64 + 4)
    out, drop, _ = E.pyramid_hash(x, paddle.to_tensor(w), num_emb=8, space_len=64, pyramid_layer=3, rand_len=4,
                                  use_filter=False)
    assert out._t.shape == (4, 8) and out._lod == [[0, 3, 4]] and drop._t.tolist() == [1, 1, 1, 0]
    out2, *_ = E.pyramid_hash(x, paddle.to_tensor(w), num_emb=8, space_len=64, pyramid_layer=3, rand_len=4,
                              use_filter=False)
    assert torch.equal(out._t, out2._t)   # deterministic hashing
    ps = [paddle.to_tensor(torch.randn(3, 5)), paddle.to_tensor(torch.randn(7).half())]
    gs = [paddle.to_tensor(torch.randn(3, 5)), paddle.to_tensor(torch.randn(7).half())]
    res = E.distributed_fused_lamb_init(ps, gs, alignment=8, rank=0, nranks=2)
    assert len(res) == 18 and torch.equal(res[13][0]._t, ps[0]._t) and torch.equal(res[14][1]._t, ps[1]._t.float())
    assert res[0]._t.numel() == 16 + 8 and res[4]._t.numel() == 8 + 4


def test_fused_dconv_drelu_dbn_matches_autograd_reference():
    torch.manual_seed(8)
    x = torch.randn(2, 4, 4, 3)
    mean, var = x.mean((0, 1, 2)), x.var((0, 1, 2), unbiased=False)
    inv = torch.rsqrt(var + 1e-5)
    g, b = torch.rand(3) + 0.5, torch.randn(3)
    w = torch.randn(5, 3, 3, 3)
    dy = torch.randn(2, 4, 4, 5)
    outs = E.fused_dconv_drelu_dbn(*(paddle.to_tensor(t) for t in (dy, w)), bn1_mean=paddle.to_tensor(mean),
                                   bn1_inv_std=paddle.to_tensor(inv), bn1_gamma=paddle.to_tensor(g),
                                   bn1_beta=paddle.to_tensor(b), bn1_input=paddle.to_tensor(x), paddings=(1, 1))
    xr, wr, gr, br = (t.clone().requires_grad_(True) for t in (x, w, g, b))
    a = torch.relu((xr - mean) * inv * gr + br)
    y = torch.nn.functional.conv2d(a.permute(0, 3, 1, 2), wr.permute(0, 3, 1, 2), padding=1)
    y.backward(dy.permute(0, 3, 1, 2))
    for o, r in zip(outs[:4], (wr.grad, xr.grad, gr.grad, br.grad)):
        assert torch.allclose(o._t, r, atol=1e-4)
    assert outs[4] is None
