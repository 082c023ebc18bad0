"""nn components added in round 2: RNN / BiRNN / RNNCellBase wrappers, LPPool1D/2D, MaxUnPool1D/3D,
FractionalMaxPool2D/3D, HSigmoidLoss, RNNTLoss (references: python/paddle/nn/layer/rnn.py,
nn/functional/pooling.py, nn/functional/loss.py; parity vs PyTorch / brute-force definitions)."""
import itertools
import math

import pytest
import torch

import paddle2_amd as paddle

P = paddle.to_tensor


def test_rnn_wrapper_matches_fused_lstm():
    torch.manual_seed(0)
    cell = paddle.nn.LSTMCell(5, 7)
    x = torch.randn(3, 6, 5)
    ref = torch.nn.LSTM(5, 7, batch_first=True)
    with torch.no_grad():
        ref.weight_ih_l0.copy_(cell.weight_ih._t)
        ref.weight_hh_l0.copy_(cell.weight_hh._t)
        ref.bias_ih_l0.copy_(cell.bias_ih._t)
        ref.bias_hh_l0.copy_(cell.bias_hh._t)
    out, (h, c) = paddle.nn.RNN(cell)(P(x))
    ro, (rh, rc) = ref(x)
    torch.testing.assert_close(out._t, ro, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(h._t, rh[0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(c._t, rc[0], rtol=1e-5, atol=1e-5)
    assert isinstance(cell, paddle.nn.RNNCellBase) and cell.state_shape == ((7,), (7,))


def test_rnn_sequence_length_freezes_states_and_reverse():
    torch.manual_seed(1)
    cell = paddle.nn.GRUCell(4, 3)
    x = torch.randn(2, 5, 4)
    lens = torch.tensor([5, 2])
    out, h = paddle.nn.RNN(cell)(P(x), sequence_length=P(lens))
    out2, h2 = paddle.nn.RNN(cell)(P(x[1:2, :2]))
    torch.testing.assert_close(h._t[1], h2._t[0], rtol=1e-5, atol=1e-6)  # state frozen after step 2
    torch.testing.assert_close(out._t[1, :2], out2._t[0], rtol=1e-5, atol=1e-6)
    # reverse == forward over the flipped sequence
    o_r, h_r = paddle.nn.RNN(cell, is_reverse=True)(P(x))
    o_f, h_f = paddle.nn.RNN(cell)(P(x.flip(1)))
    torch.testing.assert_close(o_r._t, o_f._t.flip(1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(h_r._t, h_f._t, rtol=1e-5, atol=1e-6)


def test_birnn_time_major():
    torch.manual_seed(2)
    fw, bw = paddle.nn.SimpleRNNCell(3, 4), paddle.nn.SimpleRNNCell(3, 4)
    x = torch.randn(6, 2, 3)  # time major
    out, (sf, sb) = paddle.nn.BiRNN(fw, bw, time_major=True)(P(x))
    assert tuple(out.shape) == (6, 2, 8)
    of, _ = paddle.nn.RNN(fw, time_major=True)(P(x))
    ob, _ = paddle.nn.RNN(bw, time_major=True, is_reverse=True)(P(x))
    torch.testing.assert_close(out._t, torch.cat([of._t, ob._t], -1))


def test_pool_variants():
    torch.manual_seed(3)
    x = torch.randn(2, 3, 12)
    torch.testing.assert_close(paddle.nn.LPPool1D(2, 3, 3)(P(x))._t, torch.nn.functional.lp_pool1d(x, 2, 3, 3))
    x2 = torch.randn(2, 3, 8, 8).abs()  # odd p on negatives is NaN in both
    torch.testing.assert_close(paddle.nn.LPPool2D(3, 2)(P(x2))._t, torch.nn.functional.lp_pool2d(x2, 3, 2))
    y, idx = torch.nn.functional.max_pool1d(x, 2, return_indices=True)
    torch.testing.assert_close(paddle.nn.MaxUnPool1D(2)(P(y), P(idx))._t, torch.nn.functional.max_unpool1d(y, idx, 2))
    x3 = torch.randn(1, 2, 4, 4, 4)
    y3, i3 = torch.nn.functional.max_pool3d(x3, 2, return_indices=True)
    torch.testing.assert_close(paddle.nn.MaxUnPool3D(2)(P(y3), P(i3))._t,
                               torch.nn.functional.max_unpool3d(y3, i3, 2))
    a, m = paddle.nn.FractionalMaxPool2D(output_size=5, kernel_size=2, random_u=0.3, return_mask=True)(P(x2))
    b = paddle.nn.functional.fractional_max_pool2d(P(x2), output_size=5, kernel_size=2, random_u=0.3)
    assert tuple(a.shape) == (2, 3, 5, 5) and torch.equal(a._t, b._t)  # random_u makes it reproducible
    assert torch.equal(x2.flatten(2).gather(2, m._t.flatten(2)).reshape(a.shape), a._t)
    c = paddle.nn.FractionalMaxPool3D(output_size=3, random_u=0.5)(P(x3))
    assert tuple(c.shape) == (1, 2, 3, 3, 3)


def test_hsigmoid_loss_default_tree():
    torch.manual_seed(4)
    N, D, C = 5, 6, 7
    x = torch.randn(N, D)
    lab = torch.randint(0, C, (N,))
    layer = paddle.nn.HSigmoidLoss(D, C)
    out = layer(P(x), P(lab))._t
    W, b = layer.weight._t, layer.bias._t.reshape(-1)
    ref = []
    for n in range(N):
        c = int(lab[n]) + C
        s = 0.0
        for j in range(int(math.log2(c))):
            node = (c >> (j + 1)) - 1
            bit = (c >> j) & 1
            z = float((x[n] @ W[node] + b[node]).detach())
            s += math.log1p(math.exp(z)) - bit * z
        ref.append([s])
    torch.testing.assert_close(out, torch.tensor(ref), rtol=1e-5, atol=1e-5)


def test_rnnt_loss_matches_path_enumeration():
    """-log sum over all monotone alignments (T blanks interleaved with U labels) of the path probability."""
    torch.manual_seed(5)
    B, T, U, V = 2, 3, 2, 4
    logits = torch.randn(B, T, U + 1, V)
    labels = torch.randint(1, V, (B, U))
    xl = P(logits)
    xl.stop_gradient = False
    lossp = paddle.nn.RNNTLoss(blank=0, fastemit_lambda=0.0, reduction="none")(
        xl, P(labels), P(torch.full((B,), T)), P(torch.full((B,), U)))
    loss = lossp._t.detach()
    lp = torch.log_softmax(logits.detach(), -1)
    for bi in range(B):
        tot = []
        # a path: sequence of T blanks and U emits ending with a blank at t = T-1
        for pos in itertools.combinations(range(T + U - 1), U):
            t = u = 0
            s = 0.0
            for k in range(T + U - 1):
                if k in pos:
                    s += float(lp[bi, t, u, labels[bi, u]])
                    u += 1
                else:
                    s += float(lp[bi, t, u, 0])
                    t += 1
            s += float(lp[bi, T - 1, U, 0])
            tot.append(s)
        ref = -torch.logsumexp(torch.tensor(tot), 0)
        torch.testing.assert_close(loss[bi], ref, rtol=1e-5, atol=1e-5)
    lossp.sum().backward()
    g = xl.grad._t
    assert torch.isfinite(g).all()
    torch.testing.assert_close(g.sum(-1), torch.zeros(B, T, U + 1), atol=1e-5, rtol=0)  # log-softmax grads


def test_beam_search_decoder_finds_exhaustive_best():
    """Bigram 'cell' (logits = table[prev token]); with beam >= V^(L-1) beam search is exact, so the top
    beam must equal the best of all V^L sequences; gather_tree back-traces parents."""
    torch.manual_seed(6)
    V, L, start, end = 4, 3, 0, 3
    table = torch.randn(V, V)
    table[:, end] = -30.0  # never emitted: decoding runs to max_step_num

    class Bigram(paddle.nn.RNNCellBase):
        def forward(self, inputs, states):
            return paddle.to_tensor(table[inputs._t]), states

    dec = paddle.nn.BeamSearchDecoder(Bigram(), start, end, beam_size=V ** (L - 1))
    ids, _, lens = paddle.nn.dynamic_decode(dec, inits=P(torch.zeros(2, 1)), max_step_num=L - 1, return_length=True)
    assert tuple(ids.shape) == (2, L, V ** (L - 1))
    lp = torch.log_softmax(table, -1)
    best, best_s = None, -1e9
    for seq in itertools.product(range(V - 1), repeat=L):
        s, prev = 0.0, start
        for tkn in seq:
            s += float(lp[prev, tkn])
            prev = tkn
        if s > best_s:
            best, best_s = seq, s
    assert tuple(ids._t[0, :, 0].tolist()) == best and tuple(ids._t[1, :, 0].tolist()) == best
    assert (lens._t == L).all()


def test_gather_tree():
    ids = torch.tensor([[[2, 2], [6, 1]], [[3, 9], [6, 1]], [[0, 1], [9, 0]]])
    parents = torch.tensor([[[0, 0], [1, 1]], [[1, 0], [1, 0]], [[0, 0], [0, 1]]])
    out = paddle.nn.functional.gather_tree(P(ids), P(parents))._t
    # reference docstring example (python/paddle/nn/functional/extension.py gather_tree)
    assert out.tolist() == [[[2, 2], [1, 6]], [[3, 3], [6, 1]], [[0, 1], [9, 0]]]
