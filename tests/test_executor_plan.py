"""Executor execution plan: garbage collection of dead values and the stream analyzer (reference tests:
test/standalone_executor/test_standalone_executor.py, test_stream_analyzer / GC tests)."""
import numpy as np
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.static.executor import _plan


def _chain():
    main = paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main, paddle.static.Program()):
            x = paddle.static.data("x", [4, 8], "float32")
            h = x
            for _ in range(6):
                h = paddle.nn.functional.relu(h * 1.5 - 0.25)
            out = h.sum()
    finally:
        paddle.disable_static()
    return main, x, out


def test_gc_keeps_only_fetch_targets():
    main, x, out = _chain()
    exe = paddle.static.Executor()
    env = {x._t._vid: torch.randn(4, 8)}
    res = exe._replay(main, dict(env), keep={out._t._vid})
    assert set(res) == {out._t._vid}
    # without a keep set (legacy callers) nothing is dropped
    res_all = exe._replay(main, dict(env))
    assert len(res_all) > 10
    np.testing.assert_allclose(res[out._t._vid].numpy(), res_all[out._t._vid].numpy())
    plan = _plan(main, {out._t._vid})
    freed = {v for f in plan.free_after for v in f}
    assert out._t._vid not in freed and x._t._vid in freed
    assert not plan.multi_stream


def test_gc_disabled_by_flag():
    main, x, out = _chain()
    paddle.set_flags({"FLAGS_eager_delete_tensor_gb": -1.0})
    try:
        res = paddle.static.Executor()._replay(main, {x._t._vid: torch.randn(4, 8)}, keep={out._t._vid})
        assert len(res) > 10
    finally:
        paddle.set_flags({"FLAGS_eager_delete_tensor_gb": 0.0})


def _comm_marked_program(seen):
    def side_op(t):
        if t.device.type != "meta":
            seen.append(torch.cuda.current_stream() if t.is_cuda else None)
            torch.cuda._sleep(2_000_000) if t.is_cuda else None  # long enough to race if unfenced
        return t * 3.0

    side_op._pd_stream = "comm"
    main = paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main, paddle.static.Program()):
            x = paddle.static.data("x", [1024, 1024], "float32")
            a = x + 1.0
            b = paddle.Tensor._wrap(main._record(side_op, (a._t,), {}, kind="native"))
            c = b * 2.0 + a
    finally:
        paddle.disable_static()
    return main, x, c


def test_stream_analyzer_plan():
    main, x, c = _comm_marked_program([])
    plan = _plan(main, {c._t._vid})
    assert plan.multi_stream and plan.stream_of.count("comm") == 1
    i = plan.stream_of.index("comm")
    assert len(plan.waits_on[i]) == 1          # waits for `a` produced on compute
    assert any(plan.waits_on[j] for j in range(i + 1, len(main.ops)))   # consumer of `b` waits on comm
    res = paddle.static.Executor().run(main, feed={"x": np.ones((1024, 1024), "float32")}, fetch_list=[c])
    np.testing.assert_allclose(res[0], 14.0)


@pytest.mark.gpu
def test_comm_stream_op_runs_on_context_stream_and_is_fenced():
    seen = []
    main, x, c = _comm_marked_program(seen)
    paddle.set_device("gpu:0")
    exe = paddle.static.Executor("gpu:0")
    xv = np.random.RandomState(0).randn(1024, 1024).astype("float32")
    out = exe.run(main, feed={"x": xv}, fetch_list=[c])[0]
    np.testing.assert_allclose(out, (xv + 1) * 3 * 2 + (xv + 1), rtol=1e-5)
    assert seen and seen[0] == paddle.device.get_context().comm_stream()
