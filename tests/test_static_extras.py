"""LoD sequence ops (static.nn.sequence_*) and the remaining paddle.static API (reference tests:
test/legacy_test/test_sequence_pool.py, test_sequence_softmax_op.py, test_sequence_expand.py, test_ema.py)."""
import numpy as np
import pytest

import paddle2_amd as paddle

SN = paddle.static.nn


def _lod_tensor(arr, lens):
    t = paddle.to_tensor(arr)
    t.set_recursive_sequence_lengths([lens])
    return t


def test_sequence_pool_all_types():
    x = np.arange(12, dtype="float32").reshape(6, 2)
    t = _lod_tensor(x, [2, 0, 4])
    assert t.lod() == [[0, 2, 2, 6]] and t.recursive_sequence_lengths() == [[2, 0, 4]]
    segs = [x[0:2], None, x[2:6]]
    for pt, f in (("sum", lambda s: s.sum(0)), ("average", lambda s: s.mean(0)),
                  ("sqrt", lambda s: s.sum(0) / np.sqrt(len(s))), ("max", lambda s: s.max(0)),
                  ("min", lambda s: s.min(0)), ("first", lambda s: s[0]), ("last", lambda s: s[-1])):
        out = SN.sequence_pool(t, pt, pad_value=-1.0).numpy()
        ref = np.stack([f(s) if s is not None else np.full(2, -1.0, "float32") for s in segs])
        np.testing.assert_allclose(out, ref, rtol=1e-6, err_msg=pt)
    np.testing.assert_allclose(SN.sequence_last_step(t).numpy()[2], x[5])


def test_sequence_softmax_expand_conv():
    x = np.array([1.0, 2.0, 3.0, 0.5, 0.5], "float32").reshape(5, 1)
    t = _lod_tensor(x, [3, 2])
    sm = SN.sequence_softmax(t).numpy().reshape(-1)
    e = np.exp(x[:3, 0] - x[:3, 0].max())
    np.testing.assert_allclose(sm[:3], e / e.sum(), rtol=1e-6)
    np.testing.assert_allclose(sm[3:], [0.5, 0.5], rtol=1e-6)
    a = _lod_tensor(np.array([[1.0], [2.0]], "float32"), [1, 1])
    y = _lod_tensor(np.zeros((5, 1), "float32"), [2, 3])
    ex = SN.sequence_expand(a, y)
    assert ex.numpy().reshape(-1).tolist() == [1.0, 1.0, 2.0, 2.0, 2.0] and ex.lod() == [[0, 1, 2, 3, 4, 5]]
    paddle.seed(0)
    xs = _lod_tensor(np.random.RandomState(0).randn(5, 3).astype("float32"), [3, 2])
    out = SN.sequence_conv(xs, 4, filter_size=3, bias_attr=False)
    assert list(out.shape) == [5, 4] and out.lod() == [[0, 3, 5]]
    # row 2 (last of sequence 1) must not see row 3 (first of sequence 2): zero the other rows and compare
    xs2 = _lod_tensor(np.concatenate([xs.numpy()[:3], np.zeros((2, 3), "float32")]), [3, 2])
    paddle.seed(0)
    out2 = SN.sequence_conv(xs2, 4, filter_size=3, bias_attr=False)
    np.testing.assert_allclose(out.numpy()[:3], out2.numpy()[:3], rtol=1e-5, atol=1e-6)


def test_static_extras():
    w = paddle.create_parameter([3], "float32")
    w._t.data.copy_(paddle.to_tensor([1.0, 2.0, 3.0])._t)
    ema = paddle.static.ExponentialMovingAverage(0.5, parameters=[w])
    ema.update()
    w._t.data.add_(2.0)
    ema.update()
    with ema.apply():
        np.testing.assert_allclose(w.numpy(), [2.0, 3.0, 4.0])   # 0.5 * old + 0.5 * new
    np.testing.assert_allclose(w.numpy(), [3.0, 4.0, 5.0])       # restored
    attr = paddle.static.WeightNormParamAttr(dim=0, name="wn")
    assert attr.dim == 0 and attr.name == "wn"
    sq, ab, ps, qs, pos, ins = paddle.static.ctr_metric_bundle(paddle.to_tensor([0.9, 0.2]), paddle.to_tensor([1.0, 0.0]))
    assert abs(float(sq.numpy()[0]) - (0.01 + 0.04)) < 1e-6 and float(ins.numpy()[0]) == 2
    a, _, _ = paddle.static.auc(paddle.to_tensor(np.array([[0.1, 0.9], [0.8, 0.2]], "float32")),
                                paddle.to_tensor(np.array([1, 0], "int64")))
    assert abs(float(a.numpy()[0]) - 1.0) < 1e-6
    assert paddle.static.xpu_places() == []
    with pytest.raises(RuntimeError):
        paddle.static.IpuStrategy()
