"""Pipeline scheduler passes (job lists per schedule / stage) and the DistModel static engine that runs them
(reference tests: test/auto_parallel/pipeline_scheduler_unittest.py, test_pipeline_scheduler_*.py,
semi_auto_parallel_dist_to_static*.py)."""
import copy

import numpy as np
import pytest

import paddle2_amd as paddle
import paddle2_amd.distributed as dist
from paddle2_amd.distributed.passes import apply_pass, create_job_list, new_pass


def _names(jobs):
    return [f"{j.type()}{j.micro_batch_id()}" for j in jobs]


def test_fthenb_and_1f1b_orders():
    assert _names(create_job_list("FThenB", 3)) == ["forward0", "forward1", "forward2", "backward0", "backward1",
                                                     "backward2", "optimizer0"]
    # stage 0 of 2: 2 warm-up forwards, then backward-first steady state, then the cool-down
    assert _names(create_job_list("1F1B", 4, 0, 2)) == ["forward0", "forward1", "backward0", "forward2", "backward1",
                                                         "forward3", "backward2", "backward3", "optimizer0"]
    assert _names(create_job_list("1F1B", 4, 1, 2)) == ["forward0", "backward0", "forward1", "backward1", "forward2",
                                                         "backward2", "forward3", "backward3", "optimizer0"]
    eager = _names(create_job_list("Eager1F1B", 4, 0, 2))
    assert eager[:3] == ["forward0", "forward1", "forward2"] and eager[-1] == "optimizer0"
    with pytest.raises(ValueError):
        create_job_list("Eager1F1B", 2, 0, 2)


def test_vpp_and_zbh1_orders():
    vpp = _names(create_job_list("VPP", 4, 0, 2, vpp_degree=2))
    # every (chunk, micro-batch) forward and backward appears exactly once; forwards of a chunk precede its
    # backwards; 2 chunks x 4 micro-batches
    fw = [n for n in vpp if n.startswith("forward")]
    bw = [n for n in vpp if n.startswith("backward")]
    assert sorted(fw) == sorted(f"forward{c}{i}" for c in range(2) for i in range(4))
    assert sorted(bw) == sorted(f"backward{c}{i}" for c in range(2) for i in range(4))
    for c in range(2):
        for i in range(4):
            assert vpp.index(f"forward{c}{i}") < vpp.index(f"backward{c}{i}")
    zb = _names(create_job_list("ZBH1", 4, 1, 2))
    assert zb == ["forward0", "backward_b0", "forward1", "backward2" if False else "backward1", "forward2",
                  "backward2", "forward3", "backward_b3", "backward_w3", "backward_w0", "optimizer0"]
    assert _names(create_job_list("ZBH1", 4, 0, 2))[-2:] == ["backward3", "optimizer0"]


class _MLP(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.l1 = paddle.nn.Linear(8, 16)
        self.l2 = paddle.nn.Linear(16, 1)

    def forward(self, x):
        return self.l2(paddle.nn.functional.tanh(self.l1(x)))


def _mse(out, y):
    return ((out - y) ** 2).mean()


@pytest.mark.parametrize("mode", ["FThenB", "1F1B", "ZBH1", "Eager1F1B"])
def test_dist_model_gradient_accumulation_matches_dygraph(mode):
    paddle.seed(0)
    net = _MLP()
    ref = copy.deepcopy(net)
    opt = paddle.optimizer.SGD(0.1, parameters=net.parameters())
    ropt = paddle.optimizer.SGD(0.1, parameters=ref.parameters())
    st = dist.Strategy({"pipeline": {"enable": True, "accumulate_steps": 4, "schedule_mode": mode}})
    dm = dist.to_static(net, None, _mse, opt, strategy=st)
    rs = np.random.RandomState(0)
    for _ in range(3):
        x = paddle.to_tensor(rs.randn(8, 8).astype("float32"))
        y = paddle.to_tensor(rs.randn(8, 1).astype("float32"))
        loss = dm(x, y)
        rl = _mse(ref(x), y)
        rl.backward()
        ropt.step()
        ropt.clear_grad()
        np.testing.assert_allclose(float(loss), float(rl), rtol=1e-5)
    for a, b in zip(net.parameters(), ref.parameters()):
        np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-5, atol=1e-6)
    assert len(dm._cache) == 1   # one recorded program for the micro-batch shape


def test_dist_model_eval_predict_and_gradient_merge():
    paddle.seed(1)
    net = _MLP()
    opt = paddle.optimizer.SGD(0.05, parameters=net.parameters())
    st = dist.Strategy({"gradient_merge": {"enable": True, "k_steps": 2}})
    dm = dist.to_static(net, None, _mse, opt, strategy=st)
    x = paddle.to_tensor(np.ones((4, 8), "float32"))
    y = paddle.to_tensor(np.zeros((4, 1), "float32"))
    dm(x, y)
    dm.eval()
    ev = dm(x, y)
    np.testing.assert_allclose(float(ev), float(_mse(net(x), y)), rtol=1e-5)
    dm.predict()
    out = dm(x)
    np.testing.assert_allclose(out.numpy(), net(x).numpy(), rtol=1e-5)


def test_apply_pass_and_new_pass_api():
    main, startup = paddle.static.Program(), paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main, startup):
            x = paddle.static.data("x", [2, 4], "float32")
            h = paddle.static.nn.fc(x, 3)
            loss = h.mean()
            paddle.optimizer.SGD(0.1, parameters=main.all_parameters()).minimize(loss)
    finally:
        paddle.disable_static()
    plan = apply_pass(main, "1F1B", num_micro_batches=2)
    assert plan.job_types() == ["backward", "forward", "optimizer"]
    assert len(plan.program("forward").ops) > 0 and len(plan.program("optimizer").ops) == 1
    plan2 = new_pass("pipeline_scheduler_FThenB", {"num_micro_batches": 3}).apply(main)
    assert plan2.micro_batch_num() == 3
