"""dy2static control flow: static.nn.cond / while_loop and the AST conversion of tensor-dependent ``if`` /
``while`` under jit.to_static (reference tests: test/dygraph_to_static/test_ifelse.py, test_loop.py,
test/legacy_test/test_cond.py, test_while_loop_op.py)."""
import numpy as np
import pytest

import paddle2_amd as paddle


def _np(t):
    return t.numpy() if hasattr(t, "numpy") else np.asarray(t)


def test_cond_eager_picks_branch():
    x = paddle.to_tensor([1.0, 2.0])
    out = paddle.static.nn.cond(x.sum() > 0, lambda: x * 2, lambda: x - 1)
    np.testing.assert_allclose(_np(out), [2.0, 4.0])
    out = paddle.static.nn.cond(x.sum() < 0, lambda: x * 2, lambda: x - 1)
    np.testing.assert_allclose(_np(out), [0.0, 1.0])


def test_while_loop_eager():
    i = paddle.to_tensor([0.0])
    s = paddle.to_tensor([1.0])
    i, s = paddle.static.nn.while_loop(lambda i, s: i < 5, lambda i, s: (i + 1, s * 2), [i, s])
    assert float(_np(i)[0]) == 5.0 and float(_np(s)[0]) == 32.0


def _static_run(build, feeds):
    main, startup = paddle.static.Program(), paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main, startup):
            fetch = build()
    finally:
        paddle.disable_static()
    exe = paddle.static.Executor()
    return exe.run(main, feed=feeds, fetch_list=fetch)


def test_cond_and_while_in_static_program():
    def build():
        x = paddle.static.data("x", [3], "float32")
        y = paddle.static.nn.cond(x.sum() > 0, lambda: x * 2.0, lambda: x - 1.0)
        n = paddle.static.data("n", [1], "float32")
        i = paddle.zeros([1], "float32")
        acc = paddle.zeros([3], "float32")
        i, acc = paddle.static.nn.while_loop(lambda i, a: i < n, lambda i, a: (i + 1.0, a + y), [i, acc])
        return [y, i, acc]

    for xv, nv in ((np.array([1, 2, 3], "float32"), 4.0), (np.array([-1, -2, 0], "float32"), 2.0)):
        y, i, acc = _static_run(build, {"x": xv, "n": np.array([nv], "float32")})
        ref_y = xv * 2 if xv.sum() > 0 else xv - 1
        np.testing.assert_allclose(y, ref_y)
        assert float(i[0]) == nv
        np.testing.assert_allclose(acc, ref_y * nv, rtol=1e-6)


def _branchy(x):
    if x.mean() > 0:
        y = x * 3.0
        z = y + 1.0
    else:
        y = x - 2.0
        z = y * y
    return y + z


def _loopy(x, n):
    i = paddle.zeros([1], "float32")
    s = x
    while i < n:
        t = s * 0.5
        s = t + x
        i = i + 1.0
    return s


def test_to_static_tensor_dependent_if_matches_eager():
    sf = paddle.jit.to_static(_branchy)
    for v in ([1.0, 2.0, 3.0], [-4.0, 0.5, 1.0]):
        x = paddle.to_tensor(np.array(v, "float32"))
        np.testing.assert_allclose(_np(sf(x)), _np(_branchy(x)), rtol=1e-6)
    # one signature -> one recorded program serves both branches
    assert len(sf._cache) == 1


def test_to_static_tensor_dependent_while_matches_eager():
    sf = paddle.jit.to_static(_loopy)
    x = paddle.to_tensor(np.array([1.0, -2.0], "float32"))
    for n in (0.0, 1.0, 5.0):
        nt = paddle.to_tensor(np.array([n], "float32"))
        np.testing.assert_allclose(_np(sf(x, nt)), _np(_loopy(x, nt)), rtol=1e-6)
    assert len(sf._cache) == 1


class _Gate(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.fc = paddle.nn.Linear(4, 4)

    @paddle.jit.to_static
    def forward(self, x):
        h = self.fc(x)
        if h.sum() > 0:
            out = paddle.nn.functional.relu(h)
        else:
            out = -h
        return out


def test_to_static_method_with_tensor_if_trains():
    paddle.seed(1)
    net = _Gate()
    x = paddle.to_tensor(np.random.RandomState(0).randn(2, 4).astype("float32"))
    x.stop_gradient = False
    out = net(x)
    h = net.fc(x)
    ref = paddle.nn.functional.relu(h) if float(_np(h.sum())) > 0 else -h
    np.testing.assert_allclose(_np(out), _np(ref), rtol=1e-5, atol=1e-6)
    out.sum().backward()
    assert net.fc.weight.grad is not None
    # the bound StaticFunction keeps its program cache across calls
    net(x)
    bound = net.forward
    assert len(bound._cache) == 1


def test_python_control_flow_untouched():
    def f(x, flag):
        if flag:
            x = x + 1.0
        k = 0
        while k < 3:
            x = x * 2.0
            k += 1
        return x

    sf = paddle.jit.to_static(f)
    x = paddle.to_tensor(np.array([1.0], "float32"))
    np.testing.assert_allclose(_np(sf(x, True)), [16.0])
    np.testing.assert_allclose(_np(sf(x, False)), [8.0])


def test_convert_function_keeps_super_and_closures():
    from paddle2_amd.jit.dy2static import convert_function

    scale = 3.0

    class Base:
        def f(self, x):
            return x + 1

    class Child(Base):
        def f(self, x):
            if x > 0:
                y = super().f(x) * scale
            else:
                y = -x
            return y

    g = convert_function(Child.f)
    assert g is not Child.f
    assert g(Child(), 2) == 9.0 and g(Child(), -2) == 2


def test_while_gradient_through_loop():
    sf = paddle.jit.to_static(_loopy)
    x = paddle.to_tensor(np.array([1.0, 2.0], "float32"))
    x.stop_gradient = False
    n = paddle.to_tensor(np.array([2.0], "float32"))
    sf(x, n).sum().backward()
    # s2 = 0.5*(0.5x + x) + x = 1.75x
    np.testing.assert_allclose(_np(x.grad), [1.75, 1.75], rtol=1e-6)


def test_cond_mismatched_structure_raises():
    def build():
        x = paddle.static.data("x", [2], "float32")
        return [paddle.static.nn.cond(x.sum() > 0, lambda: (x, x), lambda: x)]

    with pytest.raises(ValueError):
        _static_run(build, {"x": np.ones(2, "float32")})


# ---------------------------------------------------------------- return / break / continue / for-range passes
def _early_return(x):
    if x.mean() > 0:
        return x * 2.0
    y = x - 1.0
    return y * y


def _break_loop(x, n):
    i = paddle.zeros([1], "float32")
    s = x
    while i < n:
        s = s + 1.0
        if s.sum() > 10.0:
            break
        i = i + 1.0
    return s


def _continue_range(x, n):
    s = x * 0.0
    for k in range(n):
        if k % 2 == 1:
            continue
        s = s + x * float(k)
    return s


def _range_tensor_bound(x, n):
    acc = x
    for _ in range(n):
        acc = acc * 0.5 + x
    return acc


def _return_in_loop(x, n):
    i = paddle.zeros([1], "float32")
    while i < n:
        x = x + 1.0
        if x.sum() > 6.0:
            return x * 10.0
        i = i + 1.0
    return x


def test_prepasses_keep_eager_semantics():
    from paddle2_amd.jit.dy2static import convert_function

    for fn, cases in ((_early_return, [([1.0, 2.0],), ([-3.0, 1.0],)]),
                      (_break_loop, [([1.0, 2.0], 10.0), ([0.0, 0.0], 2.0), ([5.0, 6.0], 3.0)]),
                      (_return_in_loop, [([1.0, 1.0], 5.0), ([0.0, 0.0], 1.0)])):
        g = convert_function(fn)
        assert g is not fn
        for c in cases:
            args = [paddle.to_tensor(np.array(c[0], "float32"))]
            if len(c) > 1:
                args.append(paddle.to_tensor(np.array([c[1]], "float32")))
            np.testing.assert_allclose(_np(g(*args)), _np(fn(*args)), rtol=1e-6)
    g = convert_function(_continue_range)
    x = paddle.to_tensor(np.array([1.0, 2.0], "float32"))
    for n in (0, 1, 4, 7):
        np.testing.assert_allclose(_np(g(x, n)), _np(_continue_range(x, n)))


def test_to_static_early_return_symbolic():
    sf = paddle.jit.to_static(_early_return)
    for v in ([1.0, 2.0], [-3.0, 1.0]):
        x = paddle.to_tensor(np.array(v, "float32"))
        np.testing.assert_allclose(_np(sf(x)), _np(_early_return(x)), rtol=1e-6)
    assert len(sf._cache) == 1  # one program serves both return paths


def test_to_static_break_in_tensor_while():
    sf = paddle.jit.to_static(_break_loop)
    for xv, n in (([1.0, 2.0], 10.0), ([0.0, 0.0], 2.0), ([5.0, 6.0], 3.0)):
        x = paddle.to_tensor(np.array(xv, "float32"))
        nt = paddle.to_tensor(np.array([n], "float32"))
        np.testing.assert_allclose(_np(sf(x, nt)), _np(_break_loop(x, nt)), rtol=1e-6)
    assert len(sf._cache) == 1


def test_to_static_return_inside_tensor_while():
    sf = paddle.jit.to_static(_return_in_loop)
    for xv, n in (([1.0, 1.0], 5.0), ([0.0, 0.0], 1.0), ([3.0, 3.0], 4.0)):
        x = paddle.to_tensor(np.array(xv, "float32"))
        nt = paddle.to_tensor(np.array([n], "float32"))
        np.testing.assert_allclose(_np(sf(x, nt)), _np(_return_in_loop(x, nt)), rtol=1e-6)


def test_to_static_for_range_over_tensor_bound():
    sf = paddle.jit.to_static(_range_tensor_bound)
    x = paddle.to_tensor(np.array([1.0, -2.0], "float32"))
    for n in (0, 1, 3):
        nt = paddle.to_tensor(np.array([n], "int64"))
        np.testing.assert_allclose(_np(sf(x, nt)), _np(_range_tensor_bound(x, n)), rtol=1e-6)
    assert len(sf._cache) == 1
