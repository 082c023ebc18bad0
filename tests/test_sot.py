"""SOT mode (to_static(full_graph=False), jit/sot.py): guarded Program cache, graph-break fallback with
sub-layer translation (reference tests: test/sot/test_guard*.py, test_break_graph.py, test_simulate_initialize)."""
import numpy as np

import paddle2_amd as paddle
from paddle2_amd.jit import sot

SCALE = 2.0


def _np(t):
    return t.numpy()


def _scaled(x, k):
    return x * SCALE + k


def test_guards_on_shape_scalar_value_and_global():
    global SCALE
    f = paddle.jit.to_static(_scaled, full_graph=False)
    assert isinstance(f, sot.SymbolicTranslator)
    x = paddle.to_tensor(np.ones([2, 3], "float32"))
    np.testing.assert_allclose(_np(f(x, 1.0)), np.full([2, 3], 3.0))
    np.testing.assert_allclose(_np(f(x, 1.0)), np.full([2, 3], 3.0))
    assert f.stats["compiled"] == 1 and f.stats["guard_hits"] == 1
    np.testing.assert_allclose(_np(f(x, 5.0)), np.full([2, 3], 7.0))      # scalar value guard
    assert f.stats["compiled"] == 2
    y = paddle.to_tensor(np.ones([4], "float32"))
    np.testing.assert_allclose(_np(f(y, 1.0)), np.full([4], 3.0))          # shape guard
    assert f.stats["compiled"] == 3
    SCALE = 10.0
    try:
        np.testing.assert_allclose(_np(f(x, 1.0)), np.full([2, 3], 11.0))  # global guard
        assert f.stats["compiled"] == 4
    finally:
        SCALE = 2.0
    assert f.stats["graph_breaks"] == 0


def _needs_value(x):
    n = int(x.sum().item())  # concrete value: a graph break
    return x * float(n)


def test_graph_break_falls_back_to_eager():
    f = paddle.jit.to_static(_needs_value, full_graph=False)
    x = paddle.to_tensor(np.array([1.0, 2.0], "float32"))
    np.testing.assert_allclose(_np(f(x)), [3.0, 6.0])
    x2 = paddle.to_tensor(np.array([2.0, 2.0], "float32"))
    np.testing.assert_allclose(_np(f(x2)), [8.0, 8.0])  # eager again, correct for the new value
    assert f.stats["graph_breaks"] == 1 and f.stats["eager_calls"] == 2 and f.stats["compiled"] == 0


class _Inner(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.fc = paddle.nn.Linear(4, 4)

    def forward(self, x):
        return paddle.nn.functional.relu(self.fc(x))


class _Outer(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.a = _Inner()
        self.b = _Inner()

    def forward(self, x):
        h = self.a(x)
        if float(h.mean().item()) > 1e9:  # data-dependent Python: breaks the outer graph
            h = h * 0.0
        return self.b(h)


def test_layer_break_pushes_translation_to_sublayers_and_trains():
    paddle.seed(0)
    net = _Outer()
    x = paddle.to_tensor(np.random.RandomState(0).randn(3, 4).astype("float32"))
    ref = net.b(net.a(x))
    paddle.jit.to_static(net, full_graph=False)
    out = net(x)
    np.testing.assert_allclose(_np(out), _np(ref), rtol=1e-5, atol=1e-6)
    out = net(x)  # second call: sub-layers replay their Programs
    np.testing.assert_allclose(_np(out), _np(ref), rtol=1e-5, atol=1e-6)
    ta = net.a.forward.translator
    assert ta.stats["compiled"] == 1 and ta.stats["guard_hits"] >= 1
    assert net.forward.translator.stats["graph_breaks"] == 1
    out.sum().backward()
    assert net.a.fc.weight.grad is not None and net.b.fc.weight.grad is not None
    s = sot.summary()
    assert s["compiled"] >= 2 and s["graph_breaks"] >= 1


def test_tensor_control_flow_compiles_without_break():
    def f(x):
        if x.mean() > 0:
            return x + 1.0
        return x - 1.0

    g = paddle.jit.to_static(f, full_graph=False)
    for v in ([1.0, 2.0], [-1.0, -2.0]):
        x = paddle.to_tensor(np.array(v, "float32"))
        np.testing.assert_allclose(_np(g(x)), _np(f(x)))
    assert g.stats["compiled"] == 1 and g.stats["graph_breaks"] == 0


def test_training_flag_is_guarded():
    net = paddle.nn.Sequential(paddle.nn.Linear(4, 4), paddle.nn.Dropout(0.5))
    paddle.jit.to_static(net, full_graph=False)
    x = paddle.to_tensor(np.ones([2, 4], "float32"))
    net.eval()
    a = net(x)
    net.train()
    net(x)
    net.eval()
    b = net(x)
    np.testing.assert_allclose(_np(a), _np(b))
    assert net.forward.translator.stats["compiled"] == 2


def test_env_selects_sot(monkeypatch):
    monkeypatch.setenv("ENABLE_FALL_BACK", "1")
    f = paddle.jit.to_static(_scaled)
    assert isinstance(f, sot.SymbolicTranslator)
    monkeypatch.setenv("ENABLE_FALL_BACK", "0")
    assert not isinstance(paddle.jit.to_static(_scaled), sot.SymbolicTranslator)
