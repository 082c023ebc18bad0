"""paddle.audio / geometric / text / hub / onnx (reference tests: test/legacy_test/test_audio_functions.py,
test_graph_send_recv_op.py, test_segment_ops.py, test_graph_reindex.py, test_graph_sample_neighbors.py,
test_viterbi_decode_op.py, test_hub.py).  Numerics are checked against NumPy references written here."""
import itertools
import math
import os

import numpy as np
import pytest
import torch

import paddle2_amd as paddle


# ----------------------------------------------------------------------------- audio
def _np_mel_fbank(sr, n_fft, n_mels, fmin, fmax):
    def hz2mel(f):
        f = np.asarray(f, dtype=np.float64)
        lin = f / (200.0 / 3)
        log = 15.0 + np.log(f / 1000.0 + 1e-10) / (np.log(6.4) / 27.0)
        return np.where(f >= 1000.0, log, lin)

    def mel2hz(m):
        lin = m * (200.0 / 3)
        log = 1000.0 * np.exp((np.log(6.4) / 27.0) * (m - 15.0))
        return np.where(m >= 15.0, log, lin)

    fft = np.linspace(0, sr / 2, n_fft // 2 + 1)
    pts = mel2hz(np.linspace(hz2mel(fmin), hz2mel(fmax), n_mels + 2))
    w = np.zeros((n_mels, len(fft)))
    for i in range(n_mels):
        lo, c, hi = pts[i], pts[i + 1], pts[i + 2]
        w[i] = np.maximum(0, np.minimum((fft - lo) / (c - lo), (hi - fft) / (hi - c)))
        w[i] *= 2.0 / (hi - lo)
    return w


def test_mel_fbank_matches_numpy():
    fb = paddle.audio.functional.compute_fbank_matrix(16000, 512, 40, 50.0, 8000.0, dtype="float64").numpy()
    np.testing.assert_allclose(fb, _np_mel_fbank(16000, 512, 40, 50.0, 8000.0), rtol=1e-6, atol=1e-9)


def test_hz_mel_roundtrip_and_htk():
    f = paddle.to_tensor([20.0, 440.0, 1000.0, 3000.0, 8000.0], dtype="float64")
    for htk in (False, True):
        back = paddle.audio.functional.mel_to_hz(paddle.audio.functional.hz_to_mel(f, htk), htk)
        np.testing.assert_allclose(back.numpy(), f.numpy(), rtol=1e-6)
    assert abs(paddle.audio.functional.hz_to_mel(1000.0, htk=True) - 2595 * math.log10(1 + 1000 / 700)) < 1e-9


def test_dct_orthonormal():
    d = paddle.audio.functional.create_dct(20, 20, dtype="float64").numpy()
    np.testing.assert_allclose(d.T @ d, np.eye(20), atol=1e-10)


def test_power_to_db_and_features():
    x = paddle.to_tensor([1.0, 10.0, 100.0, 1e-12])
    np.testing.assert_allclose(paddle.audio.functional.power_to_db(x, top_db=None).numpy(), [0, 10, 20, -100],
                               atol=1e-4)
    np.testing.assert_allclose(paddle.audio.functional.power_to_db(x, top_db=30.0).numpy(), [0, 10, 20, -10],
                               atol=1e-4)
    wav = paddle.to_tensor(np.random.RandomState(0).randn(2, 4000).astype("float32"))
    spec = paddle.audio.features.Spectrogram(n_fft=256, hop_length=64, power=2.0)(wav)
    ref = torch.stft(wav._t, 256, 64, 256, torch.hann_window(256, periodic=True, dtype=torch.float32),
                     return_complex=True).abs() ** 2
    np.testing.assert_allclose(spec.numpy(), ref.numpy(), rtol=1e-4, atol=1e-3)
    mel = paddle.audio.features.MelSpectrogram(sr=16000, n_fft=256, hop_length=64, n_mels=32)(wav)
    assert mel.shape == [2, 32, spec.shape[2]]
    mfcc = paddle.audio.features.MFCC(sr=16000, n_mfcc=13, n_fft=256, n_mels=32)(wav)
    assert mfcc.shape[:2] == [2, 13]


def test_wave_backend_roundtrip(tmp_path):
    sig = np.sin(np.linspace(0, 100, 1600)).astype("float32")[None] * 0.5
    p = str(tmp_path / "a.wav")
    paddle.audio.save(p, paddle.to_tensor(sig), 16000)
    wav, sr = paddle.audio.load(p)
    assert sr == 16000 and wav.shape == [1, 1600]
    np.testing.assert_allclose(wav.numpy(), sig, atol=1e-4)
    assert paddle.audio.info(p).num_frames == 1600


# ----------------------------------------------------------------------------- geometric
def _np_send_recv(x, src, dst, op, rows):
    out = np.zeros((rows,) + x.shape[1:], dtype=x.dtype)
    buckets = {}
    for s, d in zip(src, dst):
        buckets.setdefault(d, []).append(x[s])
    for d, vals in buckets.items():
        v = np.stack(vals)
        out[d] = {"sum": v.sum(0), "mean": v.mean(0), "max": v.max(0), "min": v.min(0)}[op]
    return out


@pytest.mark.parametrize("op", ["sum", "mean", "max", "min"])
def test_send_u_recv(op):
    rs = np.random.RandomState(1)
    x = rs.randn(6, 3).astype("float32")
    src, dst = rs.randint(0, 6, 12), rs.randint(0, 5, 12)
    out = paddle.geometric.send_u_recv(paddle.to_tensor(x), paddle.to_tensor(src), paddle.to_tensor(dst), op)
    np.testing.assert_allclose(out.numpy(), _np_send_recv(x, src, dst, op, 6), rtol=1e-6)


def test_send_ue_recv_send_uv_segment():
    rs = np.random.RandomState(2)
    x, e = rs.randn(5, 4).astype("float32"), rs.randn(9, 4).astype("float32")
    src, dst = rs.randint(0, 5, 9), rs.randint(0, 5, 9)
    out = paddle.geometric.send_ue_recv(paddle.to_tensor(x), paddle.to_tensor(e), paddle.to_tensor(src),
                                        paddle.to_tensor(dst), "mul", "sum", out_size=5)
    ref = np.zeros((5, 4), "float32")
    for i, (s, d) in enumerate(zip(src, dst)):
        ref[d] += x[s] * e[i]
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-5, atol=1e-6)
    uv = paddle.geometric.send_uv(paddle.to_tensor(x), paddle.to_tensor(x), paddle.to_tensor(src),
                                  paddle.to_tensor(dst), "sub")
    np.testing.assert_allclose(uv.numpy(), x[src] - x[dst], rtol=1e-6)
    ids = np.array([0, 0, 1, 3, 3])
    np.testing.assert_allclose(paddle.geometric.segment_mean(paddle.to_tensor(x), paddle.to_tensor(ids)).numpy(),
                               np.stack([x[:2].mean(0), x[2], np.zeros(4), x[3:].mean(0)]), rtol=1e-6)


def test_send_u_recv_grad():
    x = paddle.to_tensor(np.random.RandomState(3).randn(4, 2).astype("float32"), stop_gradient=False)
    out = paddle.geometric.send_u_recv(x, paddle.to_tensor([0, 1, 1, 3]), paddle.to_tensor([1, 0, 2, 2]))
    out.sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), np.array([[1, 1], [2, 2], [0, 0], [1, 1]], "float32"))


def test_reindex_and_sampling():
    s, d, o = paddle.geometric.reindex_graph(paddle.to_tensor([0, 1, 2]), paddle.to_tensor([8, 9, 0, 4, 7, 6, 7]),
                                             paddle.to_tensor([2, 3, 2], dtype="int32"))
    assert s.numpy().tolist() == [3, 4, 0, 5, 6, 7, 6]
    assert d.numpy().tolist() == [0, 0, 1, 1, 1, 2, 2]
    assert o.numpy().tolist() == [0, 1, 2, 8, 9, 4, 7, 6]
    # CSC graph: node i's in-neighbours are row[colptr[i]:colptr[i+1]]
    row = paddle.to_tensor([3, 7, 0, 9, 1, 4, 2, 9, 3, 9, 1, 9, 7])
    colptr = paddle.to_tensor([0, 2, 4, 5, 6, 7, 9, 11, 11, 13, 13])
    nodes = paddle.to_tensor([0, 8, 1, 2])
    nb, cnt = paddle.geometric.sample_neighbors(row, colptr, nodes, sample_size=2)
    assert cnt.numpy().tolist() == [2, 2, 2, 1]
    r, cp = row.numpy(), colptr.numpy()
    off = 0
    for n, c in zip(nodes.numpy(), cnt.numpy()):
        assert set(nb.numpy()[off:off + c]) <= set(r[cp[n]:cp[n + 1]])
        off += c
    nb2, cnt2, eids = paddle.geometric.sample_neighbors(row, colptr, nodes, -1, eids=paddle.to_tensor(np.arange(13)),
                                                        return_eids=True)
    assert cnt2.numpy().tolist() == [2, 2, 2, 1] and (r[eids.numpy()] == nb2.numpy()).all()


# ----------------------------------------------------------------------------- text
def _brute_viterbi(pot, trans, length, tag):
    n = pot.shape[1]
    best, path = -np.inf, None
    for seq in itertools.product(range(n), repeat=length):
        s = pot[0, seq[0]] + (trans[-1, seq[0]] if tag else 0)
        for t in range(1, length):
            s += trans[seq[t - 1], seq[t]] + pot[t, seq[t]]
        if tag:
            s += trans[-2, seq[-1]]
        if s > best:
            best, path = s, seq
    return best, list(path)


@pytest.mark.parametrize("tag", [False, True])
def test_viterbi_decode_bruteforce(tag):
    rs = np.random.RandomState(4)
    pot = rs.rand(3, 4, 3).astype("float64")
    trans = rs.rand(3, 3).astype("float64")
    lens = np.array([4, 2, 3])
    scores, paths = paddle.text.viterbi_decode(paddle.to_tensor(pot), paddle.to_tensor(trans),
                                               paddle.to_tensor(lens), tag)
    for b in range(3):
        s, p = _brute_viterbi(pot[b], trans, lens[b], tag)
        assert abs(scores.numpy()[b] - s) < 1e-9
        assert paths.numpy()[b, :lens[b]].tolist() == p
        assert (paths.numpy()[b, lens[b]:] == 0).all()


def test_uci_housing(tmp_path):
    data = np.random.RandomState(5).rand(50, 14)
    p = tmp_path / "housing.data"
    p.write_text("\n".join(" ".join(f"{v:.6f}" for v in r) for r in data))
    tr, te = paddle.text.UCIHousing(str(p), "train"), paddle.text.UCIHousing(str(p), "test")
    assert len(tr) == 40 and len(te) == 10
    x, y = tr[0]
    assert x.shape == (13,) and y.shape == (1,)
    with pytest.raises(FileNotFoundError):
        paddle.text.UCIHousing(None)


# ----------------------------------------------------------------------------- hub / onnx
def test_hub_local(tmp_path):
    (tmp_path / "hubconf.py").write_text(
        "dependencies = ['numpy']\n"
        "import paddle2_amd as paddle\n"
        "def tiny_mlp(hidden=8):\n"
        "    '''A tiny MLP.'''\n"
        "    return paddle.nn.Sequential(paddle.nn.Linear(4, hidden), paddle.nn.ReLU())\n")
    assert "tiny_mlp" in paddle.hub.list(str(tmp_path), source="local")
    assert "tiny MLP" in paddle.hub.help(str(tmp_path), "tiny_mlp", source="local")
    m = paddle.hub.load(str(tmp_path), "tiny_mlp", source="local", hidden=5)
    assert m(paddle.randn([2, 4])).shape == [2, 5]
    with pytest.raises(RuntimeError):
        paddle.hub.load("someone/repo:main", "x", source="github")


def test_onnx_export_without_onnx_package(tmp_path):
    """The exporter writes ModelProto bytes itself (onnx/exporter.py): no onnx package needed."""
    paddle.onnx.export(paddle.nn.Linear(2, 2), str(tmp_path / "m"),
                       input_spec=[paddle.static.InputSpec([None, 2], "float32")])
    assert os.path.exists(tmp_path / "m.onnx")
