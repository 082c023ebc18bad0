"""Every name of the reference ``paddle.__all__`` (python/paddle/__init__.py) exists, and the in-place twins /
late additions behave like their reference definitions."""
import ast
import os

import numpy as np
import pytest

import paddle2_amd as paddle

REF = "/root/reference/python/paddle/__init__.py"


@pytest.mark.skipif(not os.path.exists(REF), reason="reference tree not present")
def test_reference_all_names_exist():
    src = open(REF).read()
    i = src.index("__all__")
    j = src.index("[", i)
    depth = 0
    for k in range(j, len(src)):
        depth += {"[": 1, "]": -1}.get(src[k], 0)
        if depth == 0:
            break
    names = ast.literal_eval(src[j:k + 1])
    assert len(names) > 400
    assert [n for n in names if not hasattr(paddle, n)] == []


def test_inplace_twins():
    x = paddle.to_tensor([1.0, 2.0, 3.0])
    out = paddle.equal_(x, paddle.to_tensor([1.0, 0.0, 3.0]))
    assert out is x and x.numpy().tolist() == [1.0, 0.0, 1.0]
    a = paddle.to_tensor([12, 18], dtype="int64")
    a.gcd_(paddle.to_tensor([8, 12], dtype="int64"))
    assert a.numpy().tolist() == [4, 6]
    m = paddle.ones([3, 3])
    paddle.triu_(m)
    assert np.array_equal(m.numpy(), np.triu(np.ones((3, 3))))
    y = paddle.to_tensor([[1.0, 2.0], [3.0, 4.0]])
    paddle.t_(y)
    assert y.numpy().tolist() == [[1.0, 3.0], [2.0, 4.0]]
    with pytest.raises(ValueError):
        paddle.addmm_(paddle.ones([1, 2]), paddle.ones([3, 4]), paddle.ones([4, 2]))   # result [3, 2] != x


def test_new_functions():
    m, e = paddle.frexp(paddle.to_tensor([8.0, -3.0, 0.0]))
    assert m.numpy().tolist() == [0.5, -0.75, 0.0] and e.numpy().tolist() == [4.0, 2.0, 0.0]
    assert paddle.reduce_as(paddle.ones([2, 3, 4]), paddle.ones([3, 1])).numpy().ravel().tolist() == [8.0] * 3
    np.testing.assert_allclose(paddle.histogram_bin_edges(paddle.to_tensor([0.0, 1, 2, 3]), bins=4).numpy(),
                               [0, 0.75, 1.5, 2.25, 3])
    h, edges = paddle.histogramdd(paddle.to_tensor([[0.0, 0], [1, 1], [2, 2]]), bins=2)
    assert h.numpy().tolist() == [[1.0, 0.0], [0.0, 2.0]] and len(edges) == 2
    assert list(paddle.block_diag([paddle.ones([1, 1]), paddle.ones([2, 2])]).shape) == [3, 3]
    assert [list(t.shape) for t in paddle.dsplit(paddle.ones([2, 2, 6]), 3)] == [[2, 2, 2]] * 3
    assert list(paddle.pdist(paddle.ones([4, 3])).shape) == [6]
    np.testing.assert_allclose(paddle.gammainc(paddle.to_tensor([1.0]), paddle.to_tensor([2.0])).numpy(),
                               [1 - np.exp(-2.0)], rtol=1e-6)
    np.testing.assert_allclose((paddle.gammainc(paddle.to_tensor([2.5]), paddle.to_tensor([1.5])) +
                                paddle.gammaincc(paddle.to_tensor([2.5]), paddle.to_tensor([1.5]))).numpy(), [1.0],
                               rtol=1e-6)
    assert paddle.reverse(paddle.to_tensor([1, 2, 3]), 0).numpy().tolist() == [3, 2, 1]
    paddle.seed(3)
    s = paddle.log_normal(0.0, 0.25, shape=[4000])
    assert abs(float(np.log(s.numpy()).mean())) < 0.03 and (s.numpy() > 0).all()
    with paddle.LazyGuard():
        lin = paddle.nn.Linear(2, 2)
    assert list(lin.weight.shape) == [2, 2]
