"""SOT mode (to_static(full_graph=False)): the bytecode translator (jit/opcode_executor.py — CPython 3.10 opcodes
simulated into sub-graphs, graph breaks mid-function, trace replay under guards) and the Program-level mode
(jit/sot.py with PADDLE2_AMD_SOT_BYTECODE=0: guarded Program cache, Layer-granularity fallback).  Reference tests:
test/sot/test_guard*.py, test_break_graph.py, test_simulate_initialize.py, test_04_list.py, test_11_jumps.py."""
import numpy as np
import pytest

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


@pytest.fixture
def program_mode(monkeypatch):
    monkeypatch.setenv("PADDLE2_AMD_SOT_BYTECODE", "0")


def test_graph_break_falls_back_to_eager(program_mode):
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


def test_layer_break_pushes_translation_to_sublayers_and_trains(program_mode):
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


def test_tensor_control_flow_compiles_without_break(program_mode):
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


# ------------------------------------------------------------------------------------ bytecode translator
def _branchy(x, y):
    z = x + y
    if z.sum() > 0:          # tensor-dependent jump: graph break in the middle of the function
        z = z * 2
    else:
        z = z - 1
    return z * 3


def test_bytecode_break_mid_function_and_trace_replay():
    f = paddle.jit.to_static(_branchy, full_graph=False)
    x = paddle.to_tensor(np.ones([2, 3], "float32"))
    y = paddle.to_tensor(np.ones([2, 3], "float32"))
    np.testing.assert_allclose(_np(f(x, y)), _np(_branchy(x, y)))
    assert f.stats["compiled"] == 2 and f.stats["graph_breaks"] == 1 and f.stats["simulations"] == 1
    (tr,) = f.traces
    assert [s[0] for s in tr.steps] == ["graph", "branch", "graph", "return"]
    np.testing.assert_allclose(_np(f(x * 2, y)), _np(_branchy(x * 2, y)))   # same branch: replayed, no simulation
    assert f.stats["guard_hits"] == 1 and f.stats["simulations"] == 1
    xn = paddle.to_tensor(np.full([2, 3], -5.0, "float32"))
    np.testing.assert_allclose(_np(f(xn, y)), _np(_branchy(xn, y)))         # other branch: miss, new trace
    assert f.stats["trace_misses"] == 1 and f.stats["simulations"] == 2 and len(f.traces) == 2
    np.testing.assert_allclose(_np(f(xn, y)), _np(_branchy(xn, y)))         # both outcomes now replay
    np.testing.assert_allclose(_np(f(x, y)), _np(_branchy(x, y)))
    assert f.stats["simulations"] == 2


def _valued(x):
    n = int(x.max())         # a concrete Python value: break at the call, value guarded on replay
    h = x * n
    return h + 1, n


def test_bytecode_value_break_is_guarded():
    f = paddle.jit.to_static(_valued, full_graph=False)
    x = paddle.to_tensor(np.array([1.0, 2.0], "float32"))
    out, n = f(x)
    assert n == 2
    np.testing.assert_allclose(_np(out), [3.0, 5.0])
    (tr,) = f.traces
    assert [s[0] for s in tr.steps] == ["graph", "call", "graph", "return"]
    out, n = f(paddle.to_tensor(np.array([0.5, 2.0], "float32")))      # same max: replay
    np.testing.assert_allclose(_np(out), [2.0, 5.0])
    assert f.stats["guard_hits"] == 1
    out, n = f(paddle.to_tensor(np.array([1.0, 3.0], "float32")))      # max changed: guard miss, re-simulated
    assert n == 3
    np.testing.assert_allclose(_np(out), [4.0, 10.0])
    assert f.stats["trace_misses"] == 1 and f.stats["simulations"] == 2


def _helper(z, k):
    if z.mean() > k:          # the break is inside the inlined callee
        return z * 0.5
    return z


def _uses_closures(xs, k):
    ys = [x * 2 for x in xs]          # list comprehension: MAKE_FUNCTION, simulated inline
    s = ys[0] + ys[1]
    acc = 0
    for i in range(3):
        acc = acc + i
    s = _helper(s, k)
    scale = lambda v: v + acc          # noqa: E731 - a closure over a simulated cell
    return scale(s)


def test_bytecode_inlines_user_functions_comprehensions_and_closures():
    f = paddle.jit.to_static(_uses_closures, full_graph=False)
    xs = [paddle.to_tensor(np.ones([2], "float32")), paddle.to_tensor(np.full([2], 3.0, "float32"))]
    np.testing.assert_allclose(_np(f(xs, 1.0)), _np(_uses_closures(xs, 1.0)))
    assert f.stats["graph_breaks"] == 1 and f.stats["compiled"] == 2
    np.testing.assert_allclose(_np(f(xs, 100.0)), _np(_uses_closures(xs, 100.0)))   # new scalar: new guard


def test_bytecode_layer_break_trains_like_eager():
    paddle.seed(0)
    net = _Outer()
    x = paddle.to_tensor(np.random.RandomState(0).randn(3, 4).astype("float32"))
    ref = net.b(net.a(x))
    ref.sum().backward()
    g_ref = net.a.fc.weight.grad.numpy().copy()
    net.clear_gradients()
    paddle.jit.to_static(net, full_graph=False)
    for _ in range(2):   # simulate, then replay
        net.clear_gradients()
        out = net(x)
        np.testing.assert_allclose(_np(out), _np(ref), rtol=1e-6)
        out.sum().backward()
        np.testing.assert_allclose(net.a.fc.weight.grad.numpy(), g_ref, rtol=1e-6)
    st = net.forward.translator.stats
    assert st["graph_breaks"] == 1 and st["guard_hits"] == 1 and st["simulations"] == 1


def _with_try(x):
    try:
        return x + 1
    finally:
        pass


def test_bytecode_unsupported_construct_runs_eagerly():
    f = paddle.jit.to_static(_with_try, full_graph=False)
    x = paddle.to_tensor(np.ones([2], "float32"))
    np.testing.assert_allclose(_np(f(x)), [2.0, 2.0])
    np.testing.assert_allclose(_np(f(x)), [2.0, 2.0])
    assert f.stats["eager_calls"] == 2 and "Unsupported" in f.stats["breaks"][0]


def _with_no_grad(x, w):
    h = x * w
    with paddle.no_grad():
        d = (h * 2).detach() + w   # recorded inside the context: no graph to w from this term
    return h.sum() + d.sum()


def test_bytecode_with_block_breaks_and_replays_inside_context():
    f = paddle.jit.to_static(_with_no_grad, full_graph=False)
    x = paddle.to_tensor(np.arange(6, dtype="float32").reshape(2, 3))
    for step in range(2):
        w = paddle.to_tensor(np.full([2, 3], 0.5, "float32"), stop_gradient=False)
        out = f(x, w)
        np.testing.assert_allclose(float(out), float((x * 0.5).sum() + (x * 1.0 + 0.5).sum()), rtol=1e-6)
        out.backward()
        np.testing.assert_allclose(_np(w.grad), _np(x))        # only h.sum() carries gradient
        assert paddle.is_grad_enabled()
    assert f.stats["simulations"] == 1 and f.stats["guard_hits"] == 1
    (tr,) = f.traces
    assert [s[0] for s in tr.steps] == ["graph", "call", "graph", "call", "graph", "return"]


def _with_generator_ctx(x):
    with paddle.amp.auto_cast(enable=False):
        y = x + 1
    return y * 2


def test_bytecode_with_single_use_manager_simulates_each_call():
    f = paddle.jit.to_static(_with_generator_ctx, full_graph=False)
    x = paddle.to_tensor(np.ones([3], "float32"))
    for _ in range(2):
        np.testing.assert_allclose(_np(f(x)), [4.0, 4.0, 4.0])
    assert f.stats["simulations"] == 2 and f.stats["guard_hits"] == 0 and not f.traces


def _with_raise(x):
    with paddle.no_grad():
        if x.shape[0] > 1:
            raise ValueError("boom")
    return x


def test_bytecode_with_block_left_when_translation_is_abandoned():
    f = paddle.jit.to_static(_with_raise, full_graph=False)
    with pytest.raises(ValueError):
        f(paddle.to_tensor(np.ones([3], "float32")))
    assert paddle.is_grad_enabled()
