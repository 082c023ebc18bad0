"""The static Executor runs PIR after its pass pipeline (pir/lowering.py; reference
paddle/fluid/framework/new_executor/pir_interpreter.cc:804,1458 and the PIR passes under paddle/pir/transforms,
paddle/fluid/pir/transforms/gpu/fused_gemm_epilogue_pass.cc): DCE against the fetch targets and the side effects,
CSE of pure ops, fused_gemm_epilogue — checked against the recorded program run without PIR, inference and
training."""
import numpy as np
import pytest

import paddle2_amd as paddle
from paddle2_amd import static
from paddle2_amd.framework import flags


def _build():
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data("x", [4, 8], "float32")
        fc = paddle.nn.Linear(8, 16)
        h = paddle.nn.functional.relu(fc(x))
        w = paddle.create_parameter([16, 4], "float32")
        b = paddle.create_parameter([4], "float32", is_bias=True)
        y = paddle.matmul(h, w) + b                       # matmul + bias + gelu -> fused_gemm_epilogue
        z = paddle.nn.functional.gelu(y)
        o = z * 2 + z * 2                                 # two identical pure ops -> CSE
        dead = paddle.exp(h)                              # never fetched -> DCE
    return main, x, o, dead


@pytest.fixture
def static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def test_executor_runs_optimised_pir(static_mode):
    paddle.seed(1)
    main, x, o, _ = _build()
    xv = np.random.RandomState(0).randn(4, 8).astype("float32")
    exe = static.Executor()
    (r,) = exe.run(main, feed={"x": xv}, fetch_list=[o])
    st = exe.last_pass_stats
    assert st["dead_code_elimination_pass"] >= 1
    assert st["common_subexpression_elimination_pass"] == 1
    assert st["fused_gemm_epilogue_pass"] == 1
    names = exe.last_pir.op_names()
    assert "pd_op.fused_gemm_epilogue" in names and "pd_op.gelu" not in names and "pd_op.exp" not in names
    old = flags.flag("FLAGS_enable_pir_in_executor")
    flags.set_flags({"FLAGS_enable_pir_in_executor": False})
    try:
        (ref,) = static.Executor().run(main, feed={"x": xv}, fetch_list=[o])
    finally:
        flags.set_flags({"FLAGS_enable_pir_in_executor": old})
    np.testing.assert_allclose(r, ref, rtol=1e-5, atol=1e-6)


def test_pir_executor_trains_like_recorded_program(static_mode):
    """A training program (backward + optimizer instructions are side effects the passes keep) gives the same
    losses with and without the PIR pipeline."""
    losses = {}
    for mode in (True, False):
        paddle.seed(7)
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            x = static.data("x", [8, 6], "float32")
            h = paddle.nn.functional.gelu(paddle.nn.Linear(6, 12)(x))
            h2 = paddle.nn.Linear(12, 1)(h)
            loss = (h2 * h2).mean() + (h2 * h2).mean() * 0.0
            paddle.optimizer.SGD(0.1, parameters=main.all_parameters()).minimize(loss)
        old = flags.flag("FLAGS_enable_pir_in_executor")
        flags.set_flags({"FLAGS_enable_pir_in_executor": mode})
        try:
            exe = static.Executor()
            exe.run(startup)
            xv = np.random.RandomState(3).randn(8, 6).astype("float32")
            losses[mode] = [float(exe.run(main, feed={"x": xv}, fetch_list=[loss])[0]) for _ in range(4)]
        finally:
            flags.set_flags({"FLAGS_enable_pir_in_executor": old})
    np.testing.assert_allclose(losses[True], losses[False], rtol=1e-5)
    assert losses[True][-1] < losses[True][0]
