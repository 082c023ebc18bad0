"""LBFGS and ASGD (CPU): convergence on analytic problems and the reference ASGD recurrence."""
import numpy as np
import torch

import paddle2_amd as paddle


def _rosen(x):
    return (1 - x[0]) ** 2 + 100 * (x[1] - x[0] ** 2) ** 2


def test_lbfgs_strong_wolfe_rosenbrock():
    paddle.set_device("cpu")
    x = paddle.create_parameter([2], "float64", default_initializer=paddle.nn.initializer.Assign(np.array([-1.5, 2.0])))
    opt = paddle.optimizer.LBFGS(learning_rate=1.0, max_iter=200, history_size=20, line_search_fn="strong_wolfe",
                                 parameters=[x], tolerance_grad=1e-12, tolerance_change=1e-14)

    def closure():
        opt.clear_grad()
        loss = _rosen(x)
        loss.backward()
        return loss

    for _ in range(5):
        opt.step(closure)
    np.testing.assert_allclose(x.numpy(), [1.0, 1.0], atol=1e-5)


def test_lbfgs_quadratic_no_line_search():
    paddle.set_device("cpu")
    rng = np.random.default_rng(0)
    A = rng.standard_normal((8, 8))
    A = A @ A.T + 8 * np.eye(8)
    b = rng.standard_normal(8)
    At, bt = torch.tensor(A), torch.tensor(b)
    x = paddle.create_parameter([8], "float64", default_initializer=paddle.nn.initializer.Constant(0.0))
    opt = paddle.optimizer.LBFGS(learning_rate=1.0, max_iter=100, parameters=[x], tolerance_grad=1e-10,
                                 tolerance_change=1e-16)

    def closure():
        opt.clear_grad()
        xt = x._t
        loss = 0.5 * xt @ At @ xt - bt @ xt
        loss.backward()
        return loss

    opt.step(closure)
    np.testing.assert_allclose(x.numpy(), np.linalg.solve(A, b), rtol=1e-5, atol=1e-6)


def test_asgd_matches_reference_recurrence():
    paddle.set_device("cpu")
    n, lr = 3, 0.1
    w0 = np.random.default_rng(1).standard_normal(5).astype(np.float32)
    w = paddle.create_parameter([5], "float32", default_initializer=paddle.nn.initializer.Assign(w0))
    opt = paddle.optimizer.ASGD(learning_rate=lr, batch_num=n, parameters=[w])
    ref, d, ys, m = w0.copy(), np.zeros(5, np.float32), np.zeros((n, 5), np.float32), 0
    for step in range(7):
        g = np.random.default_rng(step + 10).standard_normal(5).astype(np.float32)
        opt.clear_grad()
        (w * paddle.to_tensor(g)).sum().backward()
        opt.step()
        idx = m % n
        m += 1
        d = d - ys[idx] + g
        ys[idx] = g
        ref = ref - lr / min(m, n) * d
        np.testing.assert_allclose(w.numpy(), ref, rtol=1e-5, atol=1e-6)
