"""Long-tail reference ops (paddle2_amd/ops/extra_ops.py) through _C_ops: functional optimizer steps against the
optimizer classes, MoE routing helpers, fused inference ops against their composite definitions."""
import numpy as np
import torch

import paddle2_amd as paddle

C = paddle._C_ops


def _cls_steps(cls, p0, grads, **kw):
    lin = paddle.create_parameter([len(p0)], "float32")
    lin._t.data.copy_(torch.tensor(p0))
    opt = cls(parameters=[lin], **kw)
    for g in grads:
        lin._t.grad = torch.tensor(g)
        opt.step()
    return lin.numpy()


def _data(n=3):
    rs = np.random.RandomState(0)
    return rs.randn(6).astype("float32"), [rs.randn(6).astype("float32") for _ in range(n)]


def test_coverage_rises():
    from paddle2_amd.ops import op_schema as S

    cov = S.coverage()
    assert cov["implemented"] / cov["reference_ops"] >= 0.89, cov["missing"]


def test_nadam_radam_asgd_rprop_match_classes():
    p0, gs = _data(8)
    p = paddle.to_tensor(p0.copy())
    mdp, b2p, mup = paddle.to_tensor([1.0]), paddle.to_tensor([1.0]), paddle.to_tensor([1.0])
    m1, m2 = paddle.zeros([6]), paddle.zeros([6])
    for g in gs[:3]:
        C.nadam_(p, paddle.to_tensor(g), paddle.to_tensor([0.01]), mdp, b2p, mup, m1, m2, None)
    np.testing.assert_allclose(p.numpy(), _cls_steps(paddle.optimizer.NAdam, p0, gs[:3], learning_rate=0.01),
                               rtol=1e-5, atol=1e-6)
    p = paddle.to_tensor(p0.copy())
    b1p, b2p, rho = paddle.to_tensor([1.0]), paddle.to_tensor([1.0]), paddle.to_tensor([0.0])
    m1, m2 = paddle.zeros([6]), paddle.zeros([6])
    for g in gs:  # rho_t crosses 5 after a few steps: both branches run
        C.radam_(p, paddle.to_tensor(g), paddle.to_tensor([0.01]), b1p, b2p, rho, m1, m2, None)
    np.testing.assert_allclose(p.numpy(), _cls_steps(paddle.optimizer.RAdam, p0, gs, learning_rate=0.01),
                               rtol=1e-5, atol=1e-6)
    p, d, y = paddle.to_tensor(p0.copy()), paddle.zeros([6]), paddle.zeros([6])
    for g in gs[:2]:
        C.asgd_(p, paddle.to_tensor(g), paddle.to_tensor([0.1]), d, y, paddle.to_tensor([1.0]), None)
    np.testing.assert_allclose(p.numpy(), _cls_steps(paddle.optimizer.ASGD, p0, gs[:2], learning_rate=0.1),
                               rtol=1e-5, atol=1e-6)
    p, prev, lrs = paddle.to_tensor(p0.copy()), paddle.zeros([6]), paddle.full([6], 0.01)
    for g in gs[:3]:
        C.rprop_(p, paddle.to_tensor(g), prev, lrs, None, (1e-5, 50.0), (0.5, 1.2))
    np.testing.assert_allclose(p.numpy(), _cls_steps(paddle.optimizer.Rprop, p0, gs[:3], learning_rate=0.01),
                               rtol=1e-5, atol=1e-6)


def test_ftrl_lars_decayed_adagrad():
    p0, gs = _data(1)
    p, n, z = paddle.to_tensor(p0.copy()), paddle.zeros([6]), paddle.zeros([6])
    C.ftrl(p, n, z, paddle.to_tensor(gs[0]), paddle.to_tensor([0.1]), 1e6, 0.0)
    assert np.all(p.numpy() == 0)  # huge l1: every coordinate shrinks to zero
    p, v = paddle.to_tensor(p0.copy()), paddle.zeros([6])
    C.lars_momentum_(p, paddle.to_tensor(gs[0]), v, paddle.to_tensor([0.1]), None, 0.9, 0.001, [0.0])
    local = 0.001 * np.linalg.norm(p0) / np.linalg.norm(gs[0])
    np.testing.assert_allclose(p.numpy(), p0 - 0.1 * local * gs[0], rtol=1e-5)
    p, m = paddle.to_tensor(p0.copy()), paddle.zeros([6])
    C.decayed_adagrad(p, paddle.to_tensor(gs[0]), m, paddle.to_tensor([0.1]), 0.95, 1e-6)
    np.testing.assert_allclose(p.numpy(), p0 - 0.1 * gs[0] / (np.sqrt(0.05 * gs[0] ** 2) + 1e-6), rtol=1e-5)


def test_moe_routing_helpers():
    gate = paddle.to_tensor(np.array([2, 0, 2, 1, -1, 2], "int64"))
    cnt = C.number_count(gate, 3)
    assert cnt.numpy().tolist() == [1, 1, 3]
    pos = C.assign_pos(gate, paddle.to_tensor(np.cumsum([1, 1, 3])), 5)
    assert pos.numpy().tolist() == [1, 3, 0, 2, 5]
    lim = C.limit_by_capacity(paddle.to_tensor(np.array([2, 1, 3, 2, 2, 2], "int64")),
                              paddle.to_tensor(np.array([3, 2, 4], "int64")), 2)
    assert lim.numpy().tolist() == [2, 1, 3, 1, 1, 1]
    pruned = C.prune_gate_by_capacity(gate, paddle.to_tensor(np.array([1, 1, 2], "int64")), 3, 1)
    assert pruned.numpy().tolist() == [2, 0, 2, 1, -1, -1]


def test_fused_inference_ops_match_composites():
    rs = np.random.RandomState(1)
    x, w, y = rs.randn(4, 8).astype("float32"), rs.randn(8, 6).astype("float32"), rs.randn(4, 6).astype("float32")
    b0, sc, b1 = rs.randn(6).astype("float32"), rs.rand(6).astype("float32"), rs.randn(6).astype("float32")
    out = C.fused_fc_elementwise_layernorm(paddle.to_tensor(x), paddle.to_tensor(w), paddle.to_tensor(y),
                                           paddle.to_tensor(b0), paddle.to_tensor(sc), paddle.to_tensor(b1),
                                           1, "relu")
    h = np.maximum(x @ w + b0, 0) + y
    ref = (h - h.mean(1, keepdims=True)) / np.sqrt(h.var(1, keepdims=True) + 1e-5) * sc + b1
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-4, atol=1e-5)
    a, b = paddle.to_tensor(x), paddle.to_tensor(rs.randn(4, 8).astype("float32"))
    o = C.fused_elemwise_activation(a, b, ["elementwise_add", "relu"])
    np.testing.assert_allclose(o.numpy(), x + np.maximum(b.numpy(), 0), rtol=1e-6)
    o = C.fused_elemwise_activation(a, b, ["relu", "elementwise_mul"])
    np.testing.assert_allclose(o.numpy(), np.maximum(x * b.numpy(), 0), rtol=1e-6)
    pc = C.partial_concat([a, b], 2, 3)
    np.testing.assert_allclose(pc.numpy(), np.concatenate([x[:, 2:5], b.numpy()[:, 2:5]], 1))
    ps = C.partial_sum([a, b], 1, 2)
    np.testing.assert_allclose(ps.numpy(), x[:, 1:3] + b.numpy()[:, 1:3], rtol=1e-6)
    outs, buf = C.coalesce_tensor([a, b], None, True)
    assert buf.shape[0] >= 64 and np.allclose(outs[1].numpy(), b.numpy())
    outs[0]._t.add_(1.0)  # views of the fused buffer
    assert np.allclose(buf.numpy()[:32], (x + 1).reshape(-1))
    q = C.quant_linear(paddle.to_tensor(x), paddle.to_tensor(np.round(w * 20).astype("float32")), None, 1, "",
                       False, 1.0 / np.abs(x).max(), [1.0 / 20] * 6)
    np.testing.assert_allclose(q.numpy(), x @ w, atol=0.05 * np.abs(x @ w).max())


def test_rnn_op_and_beam_search():
    rs = np.random.RandomState(2)
    lstm = torch.nn.LSTM(4, 5)
    ws = [lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0]
    x = torch.tensor(rs.randn(3, 2, 4).astype("float32"))
    h0, c0 = torch.zeros(1, 2, 5), torch.zeros(1, 2, 5)
    out, _, states, _ = C.rnn(paddle.Tensor._wrap(x), [paddle.Tensor._wrap(h0), paddle.Tensor._wrap(c0)],
                              [paddle.Tensor._wrap(w.detach()) for w in ws], None, 0.0, False, 4, 5, 1, "LSTM")
    ref, (hn, cn) = lstm(x, (h0, c0))
    np.testing.assert_allclose(out.numpy(), ref.detach().numpy(), rtol=1e-5, atol=1e-6)
    # beam search: 1 sentence, beam 2, 3 candidates each
    pre_ids = paddle.to_tensor(np.array([[1], [2]], "int64"))
    pre_sc = paddle.to_tensor(np.array([[0.0], [0.0]], "float32"))
    ids = paddle.to_tensor(np.array([[5, 6, 7], [8, 9, 4]], "int64"))
    sc = paddle.to_tensor(np.array([[0.1, 0.9, 0.2], [0.8, 0.3, 0.4]], "float32"))
    sel, ssc, parent = C.beam_search(pre_ids, pre_sc, ids, sc, 0, 2, 0)
    assert sel.numpy().reshape(-1).tolist() == [6, 8]
    assert parent.numpy().tolist() == [0, 1]


def test_sequence_and_detection_ops():
    out, olen = C.ctc_align(paddle.to_tensor(np.array([[0, 1, 1, 0, 2, 2, 3, 0]], "int64")),
                            paddle.to_tensor(np.array([8], "int64")), 0)
    assert olen.numpy().tolist() == [[3]] and out.numpy()[0, :3].tolist() == [1, 2, 3]
    # CRF Viterbi vs brute force over all 3^4 paths
    rs = np.random.RandomState(3)
    em, tr = rs.randn(1, 4, 3).astype("float32"), rs.randn(5, 3).astype("float32")
    path = C.crf_decoding(paddle.to_tensor(em), paddle.to_tensor(tr)).numpy()[0].tolist()
    import itertools

    def score(p):
        s = tr[0, p[0]] + em[0, 0, p[0]] + tr[1, p[-1]]
        for t in range(1, 4):
            s += tr[2 + p[t - 1], p[t]] + em[0, t, p[t]]
        return s

    best = max(itertools.product(range(3), repeat=4), key=score)
    assert path == list(best)
    # IOB chunks: tags type*2 + (0=B, 1=I); label has chunks (0,1,t0) and (3,3,t1)
    lab = np.array([[0, 1, 4, 2, 4]], "int64")
    inf = np.array([[0, 1, 4, 2, 3]], "int64")
    p, r, f, ni, nl, nc = C.chunk_eval(paddle.to_tensor(inf), paddle.to_tensor(lab), "IOB", 2)
    assert int(nl.numpy()[0]) == 2 and int(ni.numpy()[0]) == 2 and int(nc.numpy()[0]) == 1
    # AUC of a perfect ranking
    sp, sn = paddle.zeros([4096], "int64"), paddle.zeros([4096], "int64")
    a, _, _ = C.auc(paddle.to_tensor(np.array([0.9, 0.8, 0.2, 0.1], "float32")),
                    paddle.to_tensor(np.array([1, 1, 0, 0], "int64")), sp, sn)
    assert abs(float(a.numpy()[0]) - 1.0) < 1e-6
    idx, dist = C.bipartite_match(paddle.to_tensor(np.array([[0.9, 0.2], [0.8, 0.7]], "float32")))
    assert idx.numpy().tolist() == [[0, 1]]
    anchors, var = C.anchor_generator(paddle.zeros([1, 8, 2, 3]), [32.0], [1.0], [0.1, 0.1, 0.2, 0.2], [16.0, 16.0])
    assert list(anchors.shape) == [2, 3, 1, 4]
    a0 = anchors.numpy()[0, 0, 0]
    assert abs((a0[2] - a0[0]) - 31.0) < 1e-4  # 32-px square anchor (x2 - x1 = w - 1)
    boxes = np.array([[[0, 0, 10, 10], [1, 1, 10, 10], [20, 20, 30, 30]]], "float32")
    scores = np.array([[[0.0, 0.0, 0.0], [0.9, 0.8, 0.7]]], "float32")
    out, index, cnt = C.multiclass_nms3(paddle.to_tensor(boxes), paddle.to_tensor(scores), None, 0.1, 10, 10, 0.5,
                                        False)
    assert cnt.numpy().tolist() == [2] and out.numpy()[:, 1].tolist() == [np.float32(0.9), np.float32(0.7)]
    seq = C.im2sequence(paddle.ones([2, 3, 4, 4]), None, [2, 2], [2, 2])
    assert list(seq.shape) == [8, 12]
    x = paddle.to_tensor(rs.randn(1, 2, 5, 5).astype("float32"))
    corr = C.correlation(x, x, 1, 1, 1)
    assert list(corr.shape) == [1, 9, 5, 5]
    np.testing.assert_allclose(corr.numpy()[0, 4], (x.numpy()[0] ** 2).mean(0), rtol=1e-5)


def test_fused_long_tail_batch3():
    rs = np.random.RandomState(4)
    x = rs.randn(2, 4, 4, 8).astype("float32")
    res = rs.randn(2, 4, 4, 8).astype("float32")
    sc, bi = rs.rand(8).astype("float32"), rs.randn(8).astype("float32")
    y, h, _, _ = C.add_group_norm_silu(paddle.to_tensor(x), paddle.to_tensor(res), paddle.to_tensor(sc),
                                       paddle.to_tensor(bi), 1e-5, 4)
    ref = torch.nn.functional.silu(torch.nn.functional.group_norm(torch.tensor(x + res).permute(0, 3, 1, 2), 4,
                                                                  torch.tensor(sc), torch.tensor(bi))).permute(0, 2, 3, 1)
    np.testing.assert_allclose(y.numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)
    a, b = rs.randn(3, 5).astype("float32"), rs.randn(5, 4).astype("float32")
    *_, out = C.fusion_squared_mat_sub(paddle.to_tensor(a), paddle.to_tensor(b), 0.5)
    np.testing.assert_allclose(out.numpy(), 0.5 * ((a @ b) ** 2 - (a * a) @ (b * b)), rtol=1e-4, atol=1e-5)
    B, S, H, nh = 2, 5, 8, 2
    inp, w, bias = rs.randn(B, S, H).astype("float32"), rs.randn(H, 3, H).astype("float32"), rs.randn(3 * H).astype(
        "float32")
    o = C.multihead_matmul(paddle.to_tensor(inp), paddle.to_tensor(w), paddle.to_tensor(bias), None, False, True,
                           False, 0.5, nh)
    qkv = (inp @ w.reshape(H, 3 * H) + bias).reshape(B, S, 3, nh, H // nh)
    q, k, v = (np.transpose(qkv[:, :, i], (0, 2, 1, 3)) for i in range(3))
    s = 0.5 * q @ np.swapaxes(k, -1, -2)
    p = np.exp(s - s.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    np.testing.assert_allclose(o.numpy(), np.transpose(p @ v, (0, 2, 1, 3)).reshape(B, S, H), rtol=1e-4, atol=1e-5)
    # resnet_unit (NCHW, no shortcut) == conv -> BN(eval) -> relu
    xc = rs.randn(1, 3, 6, 6).astype("float32")
    f = rs.randn(4, 3, 3, 3).astype("float32")
    m, vv, g, bb = rs.randn(4).astype("float32"), rs.rand(4).astype("float32") + 0.5, rs.rand(4).astype(
        "float32"), rs.randn(4).astype("float32")
    T = paddle.to_tensor
    u = C.resnet_unit(T(xc), T(f), T(g), T(bb), T(m), T(vv), None, None, None, None, None, None, 1, 1, 1,
                      data_format="NCHW")
    ref = torch.relu(torch.nn.functional.batch_norm(torch.nn.functional.conv2d(torch.tensor(xc), torch.tensor(f),
                                                                               padding=1),
                                                    torch.tensor(m), torch.tensor(vv), torch.tensor(g),
                                                    torch.tensor(bb), False, 0.0, 1e-5))
    np.testing.assert_allclose(u.numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)
    # reduced attention scores: every query row's probabilities sum to 1 -> the per-key sums add up to Sq
    q4, k4 = rs.randn(1, 6, 2, 8).astype("float32"), rs.randn(1, 6, 2, 8).astype("float32")
    s4 = np.einsum("bqhd,bkhd->bhqk", q4, k4) / np.sqrt(8)
    lse = np.log(np.exp(s4).sum(-1))
    red = C.calc_reduced_attn_scores(T(q4), T(k4), T(lse.astype("float32")))
    np.testing.assert_allclose(red.numpy().sum(-1), np.full((1, 2, 1), 6.0), rtol=1e-4)


def test_batch4_dgc_lod_misc():
    T = paddle.to_tensor
    x = T(np.array([3.0, 4.0], "float32"))
    np.testing.assert_allclose(C.dgc_clip_by_norm(x, T([5.0]), 1.0, 1.0).numpy(), [0.6, 0.8], rtol=1e-6)
    np.testing.assert_allclose(C.dgc_clip_by_norm(x, T([0.0]), 1.0, 1.0).numpy(), [3.0, 4.0])
    g = T(np.array([0.1, -5.0, 0.2, 3.0], "float32"))
    u, v = paddle.zeros([4]), paddle.zeros([4])
    _, _, enc, dense, k, _ = C.dgc(u, v, g, None, T([1.0]), None, 0.9, False, [0.5])
    assert int(k.numpy()[0]) == 2
    np.testing.assert_allclose(dense.numpy(), [0.0, -5.0, 0.0, 3.0])
    np.testing.assert_allclose(v.numpy(), [0.1, 0.0, 0.2, 0.0], rtol=1e-6)   # sent entries cleared
    rois, n = C.collect_fpn_proposals([T(np.ones((2, 4), "float32")), T(np.zeros((3, 4), "float32"))],
                                      [T(np.array([0.5, 0.9], "float32")), T(np.array([0.1, 0.95, 0.2], "float32"))],
                                      None, 3)
    assert int(n.numpy()[0]) == 3 and rois.numpy()[0].tolist() == [0, 0, 0, 0]   # 0.95 first
    a = T(np.arange(8, dtype="float32").reshape(4, 2))
    a.set_recursive_sequence_lengths([[1, 3]])
    b = T(np.ones((3, 2), "float32"))
    b.set_recursive_sequence_lengths([[2, 1]])
    cat = C.fusion_seqpool_concat([a, b], "SUM", 1)
    np.testing.assert_allclose(cat.numpy(), [[0, 1, 2, 2], [12, 15, 1, 1]])
    attn = T(np.random.RandomState(5).rand(1, 2, 4, 4).astype("float32"))
    xs = T(np.arange(12, dtype="float32").reshape(1, 4, 3))
    out, idx = C.fused_token_prune(attn, xs, None, T(np.zeros((1, 1, 2, 2), "float32")), True, True)
    assert idx.numpy()[0, 0] == 0 and list(out.shape) == [1, 2, 3]
    info = T(np.array([[0, 0, 0, 1, 2], [0, 1, 0, 3, 0], [7, 1, 0, 0, 0], [9, 2, 1, 0, 0]], "int64"))
    ch, leaf = C.tdm_child(T(np.array([0, 1], "int64")), info, 2)
    assert ch.numpy().tolist() == [[1, 2], [3, 0]] and leaf.numpy().tolist() == [[0, 1], [1, 0]]
    # LoD LSTM == torch LSTM on each sequence (gate order i, f, c, o == torch's i, f, g, o)
    rs = np.random.RandomState(6)
    D, H = 3, 4
    wx, wh, bias = rs.randn(D, 4 * H).astype("float32"), rs.randn(H, 4 * H).astype("float32"), rs.randn(
        1, 4 * H).astype("float32")
    xv = rs.randn(5, D).astype("float32")
    xt = T(xv)
    xt.set_recursive_sequence_lengths([[2, 3]])
    hs, _ = C.fusion_lstm(xt, T(wx), T(wh), T(bias))
    lstm = torch.nn.LSTM(D, H)
    with torch.no_grad():
        lstm.weight_ih_l0.copy_(torch.tensor(wx).t())
        lstm.weight_hh_l0.copy_(torch.tensor(wh).t())
        lstm.bias_ih_l0.copy_(torch.tensor(bias[0]))
        lstm.bias_hh_l0.zero_()
    for a0, b0 in ((0, 2), (2, 5)):
        ref, _ = lstm(torch.tensor(xv[a0:b0])[:, None])
        np.testing.assert_allclose(hs.numpy()[a0:b0], ref[:, 0].detach().numpy(), rtol=1e-4, atol=1e-5)
