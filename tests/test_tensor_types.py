"""SelectedRows (sparse embedding gradients + row-wise optimizer updates), TensorArray ops, StringTensor kernels
(reference tests: test/legacy_test/test_selected_rows.py, test_lookup_table_v2_op.py (is_sparse), test_sgd_op.py
(SelectedRows), test_adam_op.py (lazy_mode), test_array_read_write_op.py, test_tensor_array_to_tensor.py,
test/cpp/phi/kernels/test_strings_lower_upper_dev_api.cc)."""
import numpy as np
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.framework.tensor_types import SelectedRows, StringTensor, strings_lower, strings_upper


def test_selected_rows_merge_and_dense():
    sr = SelectedRows([3, 1, 3], height=5, value=torch.tensor([[1.0, 2.0], [3.0, 4.0], [5.0, 6.0]]))
    assert sr.shape == [5, 2] and sr.height() == 5 and sr.rows() == [3, 1, 3]
    assert sr.has_key(1) and not sr.has_key(0) and sr.index(3) == 0
    m = sr.merge_add()
    assert m.rows() == [1, 3]
    np.testing.assert_allclose(m._value.numpy(), [[3, 4], [6, 8]])
    dense = sr.to_dense().numpy()
    np.testing.assert_allclose(dense[3], [6, 8])
    np.testing.assert_allclose(dense[0], [0, 0])
    np.testing.assert_allclose(sr.to_torch_sparse().to_dense().numpy(), dense)


def _emb_pair(sparse, opt_cls, **kw):
    paddle.seed(7)
    emb = paddle.nn.Embedding(10, 4, sparse=sparse)
    opt = opt_cls(parameters=emb.parameters(), **kw)
    return emb, opt


@pytest.mark.parametrize("opt_cls,kw", [
    (paddle.optimizer.SGD, {"learning_rate": 0.5}),
    (paddle.optimizer.Adam, {"learning_rate": 0.1}),
    (paddle.optimizer.Momentum, {"learning_rate": 0.1, "momentum": 0.9}),
])
def test_sparse_embedding_matches_dense(opt_cls, kw):
    ids = [paddle.to_tensor(np.array([[1, 3, 3], [7, 1, 0]], "int64")),
           paddle.to_tensor(np.array([[2, 3, 9], [9, 9, 4]], "int64"))]
    (e1, o1), (e2, o2) = _emb_pair(False, opt_cls, **kw), _emb_pair(True, opt_cls, **kw)
    np.testing.assert_allclose(e1.weight.numpy(), e2.weight.numpy())
    for step in range(4):
        x = ids[step % 2]
        for e, o in ((e1, o1), (e2, o2)):
            (e(x) * paddle.to_tensor(np.arange(4, dtype="float32"))).sum().backward()
            o.step()
            o.clear_grad()
    np.testing.assert_allclose(e2.weight.numpy(), e1.weight.numpy(), rtol=1e-5, atol=1e-6)


def test_sparse_grad_is_row_sparse():
    emb = paddle.nn.Embedding(10, 4, sparse=True)
    emb(paddle.to_tensor(np.array([1, 5], "int64"))).sum().backward()
    g = emb.weight._t.grad
    assert g.is_sparse
    sr = SelectedRows.from_torch_sparse(g)
    assert sorted(sr.rows()) == [1, 5] and sr.height() == 10


def test_adam_lazy_mode_touches_only_looked_up_rows():
    paddle.seed(3)
    emb = paddle.nn.Embedding(8, 3, sparse=True)
    opt = paddle.optimizer.Adam(learning_rate=0.1, parameters=emb.parameters(), lazy_mode=True)
    w0 = emb.weight.numpy().copy()
    emb(paddle.to_tensor(np.array([2, 6], "int64"))).sum().backward()
    opt.step()
    opt.clear_grad()
    w1 = emb.weight.numpy()
    changed = np.where(np.abs(w1 - w0).sum(1) > 0)[0].tolist()
    assert changed == [2, 6]
    # second step on row 2 only: row 6's moments must stay untouched (lazy), so row 6 does not move
    emb(paddle.to_tensor(np.array([2], "int64"))).sum().backward()
    opt.step()
    np.testing.assert_allclose(emb.weight.numpy()[6], w1[6])
    # the same two steps in non-lazy dense Adam move row 6 again on step 2 (momentum)
    paddle.seed(3)
    emb2 = paddle.nn.Embedding(8, 3)
    opt2 = paddle.optimizer.Adam(learning_rate=0.1, parameters=emb2.parameters())
    for ids in ([2, 6], [2]):
        emb2(paddle.to_tensor(np.array(ids, "int64"))).sum().backward()
        opt2.step()
        opt2.clear_grad()
    assert np.abs(emb2.weight.numpy()[6] - w1[6]).sum() > 0


def test_sparse_grad_with_global_clip():
    paddle.seed(5)
    e1 = paddle.nn.Embedding(6, 2)
    paddle.seed(5)
    e2 = paddle.nn.Embedding(6, 2, sparse=True)
    clip = paddle.nn.ClipGradByGlobalNorm(0.1)
    o1 = paddle.optimizer.SGD(1.0, parameters=e1.parameters(), grad_clip=clip)
    o2 = paddle.optimizer.SGD(1.0, parameters=e2.parameters(), grad_clip=clip)
    x = paddle.to_tensor(np.array([0, 3, 3], "int64"))
    for e, o in ((e1, o1), (e2, o2)):
        e(x).sum().backward()
        o.step()
    np.testing.assert_allclose(e2.weight.numpy(), e1.weight.numpy(), rtol=1e-6)


def test_tensor_array_ops():
    arr = paddle.tensor.create_array("float32")
    x = paddle.full([1, 3], 5.0)
    i = paddle.zeros([1], "int64")
    arr = paddle.tensor.array_write(x, i, array=arr)
    np.testing.assert_allclose(paddle.tensor.array_read(arr, i).numpy(), [[5, 5, 5]])
    arr = paddle.tensor.array_write(paddle.full([1, 3], 7.0), paddle.ones([1], "int64"), array=arr)
    assert paddle.tensor.array_length(arr) == 2
    # overwrite in place
    paddle.tensor.array_write(paddle.full([1, 3], 1.0), i, array=arr)
    np.testing.assert_allclose(arr[0].numpy(), [[1, 1, 1]])
    with pytest.raises(IndexError):
        paddle.tensor.array_write(x, paddle.full([1], 5, "int64"), array=arr)
    out, sizes = paddle.tensor.tensor_array_to_tensor(arr, axis=0)
    assert list(out.shape) == [2, 3] and sizes.numpy().tolist() == [1, 1]
    out, sizes = paddle.tensor.tensor_array_to_tensor(arr, axis=1, use_stack=True)
    assert list(out.shape) == [1, 2, 3]
    init = paddle.tensor.create_array("float32", [x, x])
    assert len(init) == 2
    with pytest.raises(TypeError):
        paddle.tensor.create_array("float32", [1.0])


def test_tensor_array_in_recorded_loop():
    """A to_static function accumulating into a TensorArray with a Python loop records and replays."""
    def f(x):
        arr = paddle.tensor.create_array("float32")
        for k in range(3):
            arr = paddle.tensor.array_write(x * float(k + 1), paddle.full([1], k, "int64"), array=arr)
        out, _ = paddle.tensor.tensor_array_to_tensor(arr, axis=0)
        return out

    sf = paddle.jit.to_static(f)
    x = paddle.to_tensor(np.array([[1.0, 2.0]], "float32"))
    np.testing.assert_allclose(sf(x).numpy(), f(x).numpy())


def test_string_tensor_kernels():
    s = StringTensor([["Hello", "WORLD"], ["ÀÉÎ straße", "MiXeD 123"]])
    assert s.shape == [2, 2] and s.numel() == 4
    assert strings_lower(s).tolist() == [["hello", "world"], ["àéî straße", "mixed 123"]]
    assert strings_upper(s, use_utf8_encoding=False).tolist() == [["HELLO", "WORLD"], ["ÀÉÎ STRAßE", "MIXED 123"]]
    assert strings_upper(s).tolist()[1][0] == "ÀÉÎ STRASSE"
    e = paddle.framework.tensor_types.strings_empty([2, 3])
    assert e.shape == [2, 3] and e.tolist() == [[""] * 3] * 2
    assert s[0, 1] == "WORLD" and s == StringTensor(s.tolist())
