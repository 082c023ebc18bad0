"""Tensor API semantics vs NumPy (reference test strategy: test/legacy_test/test_*_op.py OpTest
compares each op against a NumPy reference)."""
import numpy as np
import pytest

import paddle2_amd as paddle


def npt(x):
    return x.numpy()


def test_creation():
    assert paddle.zeros([2, 3]).shape == [2, 3]
    assert paddle.ones([2], dtype="int64").dtype == paddle.int64
    np.testing.assert_array_equal(npt(paddle.arange(0, 10, 2)), np.arange(0, 10, 2))
    np.testing.assert_allclose(npt(paddle.linspace(0, 1, 5)), np.linspace(0, 1, 5), rtol=1e-6)
    np.testing.assert_array_equal(npt(paddle.full([2, 2], 7.0)), np.full([2, 2], 7.0, np.float32))
    np.testing.assert_array_equal(npt(paddle.eye(3)), np.eye(3, dtype=np.float32))
    x = paddle.to_tensor([[1, 2], [3, 4]])
    assert x.dtype == paddle.int64
    assert paddle.to_tensor([1.0, 2.0]).dtype == paddle.float32
    np.testing.assert_array_equal(npt(paddle.zeros_like(x)), np.zeros((2, 2)))
    np.testing.assert_array_equal(npt(paddle.tril(paddle.ones([3, 3]))), np.tril(np.ones((3, 3))))
    assert paddle.empty([4, 5]).shape == [4, 5]


def test_math_broadcast_and_reductions():
    a = np.random.rand(3, 4).astype("float32")
    b = np.random.rand(4).astype("float32")
    x, y = paddle.to_tensor(a), paddle.to_tensor(b)
    np.testing.assert_allclose(npt(x + y), a + b, rtol=1e-6)
    np.testing.assert_allclose(npt(paddle.add(x, y)), a + b, rtol=1e-6)
    np.testing.assert_allclose(npt(x * 2 - 1), a * 2 - 1, rtol=1e-6)
    np.testing.assert_allclose(npt(paddle.sum(x, axis=1)), a.sum(1), rtol=1e-5)
    np.testing.assert_allclose(npt(x.mean(axis=0, keepdim=True)), a.mean(0, keepdims=True), rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.max(x, axis=-1)), a.max(-1))
    np.testing.assert_array_equal(npt(paddle.argmax(x, axis=1)), a.argmax(1))
    np.testing.assert_allclose(npt(paddle.exp(x)), np.exp(a), rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.pow(x, 2)), a ** 2, rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.clip(x, 0.2, 0.5)), np.clip(a, 0.2, 0.5))
    np.testing.assert_allclose(npt(paddle.cumsum(x, axis=1)), np.cumsum(a, 1), rtol=1e-5)
    np.testing.assert_allclose(float(paddle.std(x)), a.std(ddof=1), rtol=1e-4)
    np.testing.assert_allclose(npt(paddle.logsumexp(x, axis=1)), np.log(np.exp(a).sum(1)), rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.prod(x, axis=0)), a.prod(0), rtol=1e-5)


def test_matmul_and_linalg():
    a = np.random.rand(2, 3, 4).astype("float32")
    b = np.random.rand(4, 5).astype("float32")
    np.testing.assert_allclose(npt(paddle.matmul(paddle.to_tensor(a), paddle.to_tensor(b))), a @ b, rtol=1e-5)
    np.testing.assert_allclose(
        npt(paddle.matmul(paddle.to_tensor(b), paddle.to_tensor(b), transpose_x=True)), b.T @ b, rtol=1e-5)
    m = np.random.rand(3, 3).astype("float32") + 3 * np.eye(3, dtype="float32")
    np.testing.assert_allclose(npt(paddle.linalg.inv(paddle.to_tensor(m))), np.linalg.inv(m), rtol=1e-4)
    np.testing.assert_allclose(float(paddle.linalg.norm(paddle.to_tensor(m))), np.linalg.norm(m), rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.bmm(paddle.to_tensor(a), paddle.to_tensor(a).transpose([0, 2, 1]))),
                               a @ a.transpose(0, 2, 1), rtol=1e-5)


def test_manipulation():
    a = np.arange(24).reshape(2, 3, 4).astype("float32")
    x = paddle.to_tensor(a)
    assert paddle.reshape(x, [4, -1]).shape == [4, 6]
    np.testing.assert_array_equal(npt(paddle.transpose(x, [2, 0, 1])), a.transpose(2, 0, 1))
    np.testing.assert_array_equal(npt(paddle.concat([x, x], axis=1)), np.concatenate([a, a], 1))
    np.testing.assert_array_equal(npt(paddle.stack([x, x], axis=0)), np.stack([a, a], 0))
    parts = paddle.split(x, [1, 3], axis=2)
    assert [p.shape for p in parts] == [[2, 3, 1], [2, 3, 3]]
    parts = paddle.split(x, 2, axis=2)
    np.testing.assert_array_equal(npt(parts[1]), a[:, :, 2:])
    assert paddle.unsqueeze(x, [0, 2]).shape == [1, 2, 1, 3, 4]
    assert paddle.squeeze(paddle.ones([1, 3, 1]), axis=0).shape == [3, 1]
    assert paddle.flatten(x, 1).shape == [2, 12]
    np.testing.assert_array_equal(npt(paddle.flip(x, [0])), a[::-1])
    np.testing.assert_array_equal(npt(paddle.tile(paddle.to_tensor([1, 2]), [2])), [1, 2, 1, 2])
    np.testing.assert_array_equal(npt(paddle.gather(x, paddle.to_tensor([1, 0]))), a[[1, 0]])
    idx = np.array([[0, 1], [1, 2]])
    np.testing.assert_array_equal(npt(paddle.gather_nd(x, paddle.to_tensor(idx))), a[idx[:, 0], idx[:, 1]])
    np.testing.assert_array_equal(npt(x.expand([2, 2, 3, 4])), np.broadcast_to(a, (2, 2, 3, 4)))
    np.testing.assert_array_equal(npt(paddle.slice(x, axes=[1], starts=[1], ends=[3])), a[:, 1:3])
    np.testing.assert_array_equal(npt(x[:, 1, ::2]), a[:, 1, ::2])
    np.testing.assert_array_equal(npt(paddle.roll(x, 1, axis=2)), np.roll(a, 1, 2))
    np.testing.assert_array_equal(npt(paddle.where(x > 10, x, paddle.zeros_like(x))), np.where(a > 10, a, 0))


def test_setitem_and_inplace():
    x = paddle.zeros([3, 4])
    x[1] = 5.0
    x[:, 2] = paddle.ones([3])
    ref = np.zeros((3, 4), np.float32)
    ref[1] = 5
    ref[:, 2] = 1
    np.testing.assert_array_equal(npt(x), ref)
    y = paddle.ones([2])
    y.add_(paddle.ones([2]))
    np.testing.assert_array_equal(npt(y), [2, 2])
    y.scale_(3.0)
    np.testing.assert_array_equal(npt(y), [6, 6])


def test_search_sort_logic():
    a = np.array([[3, 1, 2], [9, 7, 8]], dtype="float32")
    x = paddle.to_tensor(a)
    v, i = paddle.topk(x, 2, axis=1)
    np.testing.assert_array_equal(npt(v), [[3, 2], [9, 8]])
    np.testing.assert_array_equal(npt(i), [[0, 2], [0, 2]])
    np.testing.assert_array_equal(npt(paddle.sort(x, axis=1)), np.sort(a, 1))
    np.testing.assert_array_equal(npt(paddle.argsort(x, axis=1, descending=True)), np.argsort(-a, 1))
    assert bool(paddle.all(x > 0))
    assert bool(paddle.any(x > 8.5))
    np.testing.assert_array_equal(npt(paddle.nonzero(x > 7)), np.argwhere(a > 7))
    np.testing.assert_array_equal(npt(paddle.masked_select(x, x > 7)), a[a > 7])
    assert paddle.equal_all(x, paddle.to_tensor(a))
    np.testing.assert_array_equal(npt(paddle.unique(paddle.to_tensor([3, 1, 3, 2]))), [1, 2, 3])
    assert paddle.allclose(x, x + 1e-9)


def test_dtype_cast_and_bf16_numpy():
    x = paddle.to_tensor([1.5, 2.25])
    xb = x.astype("bfloat16")
    assert xb.dtype == paddle.bfloat16
    assert x.cast("float16").dtype == paddle.float16
    assert np.allclose(xb.astype("float32").numpy(), [1.5, 2.25])
    # Paddle exposes bf16 numpy as uint16 bit patterns
    raw = xb.numpy()
    assert raw.dtype == np.uint16


def test_random_seeded():
    paddle.seed(123)
    a = paddle.randn([4]).numpy()
    paddle.seed(123)
    b = paddle.randn([4]).numpy()
    np.testing.assert_array_equal(a, b)
    r = paddle.randint(0, 5, [100])
    assert int(r.min()) >= 0 and int(r.max()) < 5
    u = paddle.uniform([1000], min=-1, max=1)
    assert -1 <= float(u.min()) and float(u.max()) <= 1
    p = paddle.randperm(10).numpy()
    assert sorted(p.tolist()) == list(range(10))


def test_tensor_methods_and_props():
    x = paddle.to_tensor([[1.0, 2.0], [3.0, 4.0]], stop_gradient=False)
    assert x.ndim == 2 and x.size == 4 and x.shape == [2, 2]
    assert not x.stop_gradient
    y = (x * x).sum()
    y.backward()
    np.testing.assert_allclose(x.grad.numpy(), 2 * x.numpy())
    assert x.detach().stop_gradient
    assert x.t().shape == [2, 2]
    assert x.reshape([4]).tolist() == [1.0, 2.0, 3.0, 4.0]
    assert float(x.norm()) == pytest.approx(np.sqrt(30.0), rel=1e-5)
    assert x.place.is_cpu_place()
