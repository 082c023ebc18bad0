"""paddle.incubate.autograd (vjp / jvp / Jacobian / Hessian / forward_grad / grad) against torch.autograd.functional
and closed forms; paddle.incubate.asp n:m masks, pruning and the sparsity-preserving optimizer (reference tests:
test/autograd/test_autograd_functional_dynamic.py, test/asp/test_asp_utils.py, test_asp_pruning_dynamic.py)."""
import numpy as np
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.incubate import asp
from paddle2_amd.incubate import autograd as IA


def _f(x, y):
    return x * y.sum() + paddle.sin(x)


def test_vjp_jvp_match_torch():
    x = paddle.to_tensor(np.array([0.5, -1.0, 2.0], "float64"))
    y = paddle.to_tensor(np.array([1.5, 0.25], "float64"))
    v = paddle.to_tensor(np.array([1.0, 2.0, -1.0], "float64"))
    out, (gx, gy) = IA.vjp(_f, [x, y], v)
    tf = lambda a, b: a * b.sum() + torch.sin(a)  # noqa: E731
    _, (rx, ry) = torch.autograd.functional.vjp(tf, (x._t, y._t), v._t)
    np.testing.assert_allclose(gx.numpy(), rx.numpy())
    np.testing.assert_allclose(gy.numpy(), ry.numpy())
    u = [paddle.to_tensor(np.array([1.0, 0.0, 1.0])), paddle.to_tensor(np.array([0.5, 0.5]))]
    _, jv = IA.jvp(_f, [x, y], u)
    _, rjv = torch.autograd.functional.jvp(tf, (x._t, y._t), (u[0]._t, u[1]._t))
    np.testing.assert_allclose(jv.numpy(), rjv.numpy(), rtol=1e-12)


def test_jacobian_lazy_rows_and_batched():
    def f(x):
        return paddle.matmul(x, x.T) if False else x * x * 3

    x = paddle.to_tensor(np.array([[1.0, 2.0], [3.0, 4.0]], "float64"))
    J = IA.Jacobian(f, x)
    assert J.shape == [4, 4]
    np.testing.assert_allclose(J[:].numpy(), np.diag(6 * x.numpy().reshape(-1)))
    np.testing.assert_allclose(J[1, :].numpy(), [0, 12, 0, 0])
    assert len(J._jacobian._rows) == 4
    Jb = IA.Jacobian(f, x, is_batched=True)
    assert Jb.shape == [2, 2, 2]
    np.testing.assert_allclose(Jb[:].numpy(), np.stack([np.diag(6 * r) for r in x.numpy()]))
    np.testing.assert_allclose(Jb[:, 1, 1].numpy(), [12.0, 24.0])


def test_hessian_quadratic():
    A = np.array([[2.0, 1.0], [1.0, 3.0]])
    At = paddle.to_tensor(A)

    def f(x):
        return 0.5 * (x * paddle.matmul(At, x)).sum()

    H = IA.Hessian(f, paddle.to_tensor(np.array([0.3, -0.7])))
    np.testing.assert_allclose(H[:].numpy(), A)


def test_forward_grad_and_grad_of_computed_outputs():
    x = paddle.to_tensor(np.array([1.0, 2.0, 3.0]), stop_gradient=False)
    y = x * x
    fg = IA.forward_grad(y, x, paddle.to_tensor(np.array([1.0, 0.0, 2.0])))
    np.testing.assert_allclose(fg.numpy(), [2.0, 0.0, 12.0])
    g = IA.grad(y, x)
    np.testing.assert_allclose(g.numpy(), [2.0, 4.0, 6.0])
    IA.enable_prim()
    assert IA.prim_enabled()
    IA.disable_prim()
    assert not IA.prim_enabled()


def test_asp_masks_numpy_api():
    mat = np.array([[2, 8, 9, 9], [9, 1, 3, 9], [5, 6, 3, 9], [2, 4, 6, 9]], "float32")
    m1 = asp.create_mask(mat, asp.MaskAlgo.MASK_1D, 2, 4)
    np.testing.assert_array_equal(m1, [[0, 0, 1, 1], [1, 0, 0, 1], [0, 1, 0, 1], [0, 0, 1, 1]])
    assert asp.check_mask_1d(mat * m1, 2, 4) and not asp.check_mask_1d(mat, 2, 4)
    for algo in (asp.MaskAlgo.MASK_2D_GREEDY, asp.MaskAlgo.MASK_2D_BEST):
        m2 = asp.create_mask(mat, algo, 2, 4)
        assert asp.check_mask_2d(mat * m2, 2, 4)
        assert asp.check_sparsity(mat * m2, asp.CheckMethod.CHECK_2D, 2, 4)
    best = (mat * asp.get_mask_2d_best(mat, 2, 4)).sum()
    greedy = (mat * asp.get_mask_2d_greedy(mat, 2, 4)).sum()
    assert best >= greedy
    assert asp.calculate_density(mat * m1) == 0.5


def test_asp_prune_model_and_decorated_training():
    paddle.seed(0)
    net = paddle.nn.Sequential(paddle.nn.Linear(16, 8), paddle.nn.ReLU(), paddle.nn.Linear(8, 4),
                               paddle.nn.Linear(4, 2))
    asp.reset_excluded_layers()
    asp.set_excluded_layers([net[3].weight.name])
    opt = asp.decorate(paddle.optimizer.SGD(0.1, parameters=net.parameters()))
    masks = asp.prune_model(net, n=2, m=4)
    assert net[0].weight.name in masks and net[3].weight.name not in masks
    for _ in range(3):
        x = paddle.to_tensor(np.random.RandomState(0).randn(5, 16).astype("float32"))
        net(x).sum().backward()
        opt.step()
        opt.clear_grad()
    for lin in (net[0], net[2]):
        w = lin.weight.numpy()               # [in, out]: 2:4 along `in` for every output column
        assert asp.check_mask_1d(w.T, 2, 4)
        assert abs(asp.calculate_density(w) - 0.5) < 1e-6
    assert asp.calculate_density(net[3].weight.numpy()) == 1.0
    conv = paddle.nn.Conv2D(8, 4, 3)
    asp.prune_model(conv, mask_algo="mask_2d_greedy")
    w = conv.weight.numpy()                  # [out, in, kh, kw]: along the input channels
    assert asp.calculate_density(w) <= 0.5 + 1e-6
    asp.reset_excluded_layers()
