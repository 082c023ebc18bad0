"""paddle.incubate.optimizer: LookAhead, ModelAverage, GradientMergeOptimizer, RecomputeOptimizer,
LarsMomentumOptimizer, DistributedFusedLamb (1 rank), functional minimize_bfgs / minimize_lbfgs (reference tests:
test/legacy_test/test_lookahead.py, test_modelaverage.py, test_bfgs.py, test_lbfgs.py)."""
import copy

import numpy as np
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.incubate import optimizer as IO


def _net(seed=0):
    paddle.seed(seed)
    return paddle.nn.Sequential(paddle.nn.Linear(4, 8), paddle.nn.Tanh(), paddle.nn.Linear(8, 1))


def _batch(i):
    rs = np.random.RandomState(i)
    return paddle.to_tensor(rs.randn(6, 4).astype("float32")), paddle.to_tensor(rs.randn(6, 1).astype("float32"))


def _loss(net, i):
    x, y = _batch(i)
    return ((net(x) - y) ** 2).mean()


def test_lookahead_matches_manual_slow_weights():
    net = _net()
    ref = copy.deepcopy(net)
    la = IO.LookAhead(paddle.optimizer.SGD(0.1, parameters=net.parameters()), alpha=0.5, k=3)
    sgd = paddle.optimizer.SGD(0.1, parameters=ref.parameters())
    slow = [p.numpy().copy() for p in ref.parameters()]
    for i in range(7):
        _loss(net, i).backward()
        la.step()
        la.clear_grad()
        _loss(ref, i).backward()
        sgd.step()
        sgd.clear_grad()
        if (i + 1) % 3 == 0:
            for j, p in enumerate(ref.parameters()):
                slow[j] = slow[j] + 0.5 * (p.numpy() - slow[j])
                p.set_value(slow[j])
    for a, b in zip(net.parameters(), ref.parameters()):
        np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-5, atol=1e-6)
    sd = la.state_dict()
    assert sd["lookahead_step"] == 7 and any(k.endswith("_slow_0") for k in sd)


def test_model_average_apply_restore():
    net = _net()
    sgd = paddle.optimizer.SGD(0.1, parameters=net.parameters())
    ma = IO.ModelAverage(0.15, parameters=net.parameters(), min_average_window=2, max_average_window=10)
    hist = []
    for i in range(5):
        _loss(net, i).backward()
        sgd.step()
        sgd.clear_grad()
        ma.step()
        hist.append([p.numpy().copy() for p in net.parameters()])
    trained = [p.numpy().copy() for p in net.parameters()]
    with ma.apply():
        avg = [p.numpy().copy() for p in net.parameters()]
    # min window 2: the sums roll after iterates 2 and 4 (sum_3 keeps the last full window), so the average is
    # over the last full window plus the current partial one: iterates 3, 4, 5
    for j, a in enumerate(avg):
        np.testing.assert_allclose(a, np.mean([h[j] for h in hist[2:]], 0), rtol=1e-5, atol=1e-6)
    for a, b in zip(net.parameters(), trained):
        np.testing.assert_allclose(a.numpy(), b)     # restored


def test_gradient_merge_equals_accumulated_step():
    net = _net()
    ref = copy.deepcopy(net)
    gm = IO.GradientMergeOptimizer(paddle.optimizer.SGD(0.1, parameters=net.parameters()), k_steps=2, avg=True)
    sgd = paddle.optimizer.SGD(0.1, parameters=ref.parameters())
    for i in range(4):
        _loss(net, i).backward()
        gm.minimize(None)
        (_loss(ref, i) / 2).backward()
        if i % 2 == 1:
            sgd.step()
            sgd.clear_grad()
    for a, b in zip(net.parameters(), ref.parameters()):
        np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-5, atol=1e-6)


def test_lars_momentum_matches_formula():
    paddle.seed(0)
    lin = paddle.nn.Linear(3, 2)
    w0 = lin.weight.numpy().copy()
    opt = IO.LarsMomentumOptimizer(0.1, 0.9, lars_coeff=0.01, lars_weight_decay=0.001,
                                   parameters=[lin.weight])
    x = paddle.to_tensor(np.ones((2, 3), "float32"))
    lin(x).sum().backward()
    g = lin.weight.grad.numpy().copy()
    opt.step()
    local = 0.01 * np.linalg.norm(w0) / (np.linalg.norm(g) + 0.001 * np.linalg.norm(w0))
    v = 0.1 * local * (g + 0.001 * w0)
    np.testing.assert_allclose(lin.weight.numpy(), w0 - v, rtol=1e-5, atol=1e-6)


def test_distributed_fused_lamb_single_rank_is_lamb():
    net = _net()
    ref = copy.deepcopy(net)
    a = IO.DistributedFusedLamb(0.01, parameters=net.parameters())
    b = paddle.optimizer.Lamb(0.01, parameters=ref.parameters())
    for i in range(3):
        _loss(net, i).backward()
        a.step()
        a.clear_grad()
        _loss(ref, i).backward()
        b.step()
        b.clear_grad()
    for p, q in zip(net.parameters(), ref.parameters()):
        np.testing.assert_allclose(p.numpy(), q.numpy(), rtol=1e-5, atol=1e-6)


def test_recompute_optimizer_static_minimize():
    paddle.seed(2)
    net = _net(2)
    main = paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main, paddle.static.Program()):
            x = paddle.static.data("x", [6, 4], "float32")
            y = paddle.static.data("y", [6, 1], "float32")
            h = net[0](x)
            loss = ((net[2](net[1](h)) - y) ** 2).mean()
            ro = IO.RecomputeOptimizer(paddle.optimizer.SGD(0.1, parameters=net.parameters()))
            ro._set_checkpoints([h])
            ro.minimize(loss)
    finally:
        paddle.disable_static()
    assert any(o.kind == "optimize" for o in main.ops)
    ref = copy.deepcopy(net)
    exe = paddle.static.Executor()
    xb, yb = _batch(0)
    exe.run(main, feed={"x": xb.numpy(), "y": yb.numpy()}, fetch_list=[loss])
    rl = ((ref(xb) - yb) ** 2).mean()
    rl.backward()
    paddle.optimizer.SGD(0.1, parameters=ref.parameters()).step()
    for p, q in zip(net.parameters(), ref.parameters()):
        np.testing.assert_allclose(p.numpy(), q.numpy(), rtol=1e-5, atol=1e-6)


def test_pipeline_optimizer_single_stage():
    paddle.seed(4)
    net = _net(4)
    ref = copy.deepcopy(net)
    main = paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main, paddle.static.Program()):
            x = paddle.static.data("x", [6, 4], "float32")
            y = paddle.static.data("y", [6, 1], "float32")
            loss = ((net(x) - y) ** 2).mean()
            IO.PipelineOptimizer(paddle.optimizer.SGD(0.1, parameters=net.parameters()),
                                 num_microbatches=3).minimize(loss)
    finally:
        paddle.disable_static()
    exe = paddle.static.Executor()
    ropt = paddle.optimizer.SGD(0.1, parameters=ref.parameters())
    for i in range(2):
        xb, yb = _batch(i)
        (lv,) = exe.run(main, feed={"x": xb.numpy(), "y": yb.numpy()}, fetch_list=[loss])
        rl = ((ref(xb) - yb) ** 2).mean()
        rl.backward()
        ropt.step()
        ropt.clear_grad()
        np.testing.assert_allclose(float(lv), float(rl), rtol=1e-5)
    for p, q in zip(net.parameters(), ref.parameters()):
        np.testing.assert_allclose(p.numpy(), q.numpy(), rtol=1e-5, atol=1e-6)


def _quad():
    A = torch.tensor([[3.0, 0.5, 0.0], [0.5, 2.0, 0.3], [0.0, 0.3, 1.0]], dtype=torch.float64)
    b = torch.tensor([1.0, -2.0, 0.5], dtype=torch.float64)

    def f(x):
        t = x._t
        return paddle.Tensor._wrap(0.5 * t @ (A @ t) - b @ t)

    return f, torch.linalg.solve(A, b)


def test_minimize_bfgs_quadratic_and_rosenbrock():
    f, xs = _quad()
    conv, calls, x, fx, g, H = IO.functional.minimize_bfgs(f, paddle.to_tensor(np.zeros(3)), dtype="float64")
    assert bool(conv.numpy()) and int(calls.numpy()) > 1
    np.testing.assert_allclose(x.numpy(), xs.numpy(), rtol=1e-6, atol=1e-7)
    assert list(H.shape) == [3, 3]

    def rosen(x):
        t = x._t
        return paddle.Tensor._wrap(((1 - t[0]) ** 2 + 100 * (t[1] - t[0] ** 2) ** 2))

    conv, _, x, fx, _, _ = IO.functional.minimize_bfgs(rosen, paddle.to_tensor(np.array([-1.2, 1.0])),
                                                       max_iters=200, dtype="float64")
    np.testing.assert_allclose(x.numpy(), [1.0, 1.0], atol=1e-4)


def test_minimize_lbfgs_quadratic():
    f, xs = _quad()
    conv, calls, x, fx, g = IO.functional.minimize_lbfgs(f, paddle.to_tensor(np.zeros(3)), history_size=5,
                                                         dtype="float64")
    assert bool(conv.numpy())
    np.testing.assert_allclose(x.numpy(), xs.numpy(), rtol=1e-6, atol=1e-7)
    with pytest.raises(NotImplementedError):
        IO.functional.minimize_lbfgs(f, paddle.to_tensor(np.zeros(3)), line_search_fn="hager_zhang")
