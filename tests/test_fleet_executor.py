"""FleetExecutor: native carrier + interceptors (csrc/runtime/fleet_executor.cpp) driven from Python
(reference tests: test/cpp/fluid/fleet_executor/compute_interceptor_test.cc, interceptor_pipeline_*_test.cc,
test/legacy_test/test_fleet_executor*.py)."""
import threading

import numpy as np
import pytest

from _dist import run_workers
from paddle2_amd.distributed.fleet.fleet_executor_utils import FleetExecutor, FleetExecutorUtils, TaskNode


def _chain(m, buf_ab, log, lock):
    def mk(name):
        def f(step):
            with lock:
                log.append((name, step))
        return f

    src = TaskNode(0, m, node_type="Source", task_id=1)
    a = TaskNode(0, m, node_type="Compute", task_id=2, fn=mk("a"))
    b = TaskNode(0, m, node_type="Compute", task_id=3, fn=mk("b"))
    sink = TaskNode(0, m, node_type="Sink", task_id=4)
    src.add_downstream_task(2, 2)
    a.add_upstream_task(1, 2)
    a.add_downstream_task(3, buf_ab)
    b.add_upstream_task(2, buf_ab)
    b.add_downstream_task(4, 2)
    sink.add_upstream_task(3, 2)
    return [src, a, b, sink]


@pytest.mark.parametrize("buf", [1, 3])
def test_chain_respects_buffer_bound(buf):
    log, lock = [], threading.Lock()
    fe = FleetExecutor(_chain(8, buf, log, lock), num_threads=3)
    fe.run(timeout_s=30)
    fe.release()
    a_steps = [s for n, s in log if n == "a"]
    b_steps = [s for n, s in log if n == "b"]
    assert a_steps == list(range(8)) and b_steps == list(range(8))
    # `a` may run at most `buf` steps ahead of `b`'s completions
    done_b = 0
    for n, s in log:
        if n == "b":
            done_b += 1
        else:
            assert s - done_b < buf


def test_1f1b_task_graph_order():
    """2 stages x (lr, fwd, bwd, opt) on one carrier: each micro-batch's backward follows its forward, stage 1
    finishes a backward before stage 0 starts it, lr runs once first, opt once last, and stage 0 never has more
    than pp_degree forwards outstanding."""
    log, lock = [], threading.Lock()

    def mk(stage, kind):
        def f(step):
            with lock:
                log.append((stage, kind, step))
        return f

    m = 6
    fns = [{k: mk(s, k) for k in ("lr", "fwd", "bwd", "opt")} for s in range(2)]
    nodes = FleetExecutorUtils({"pp_degree": 2}, nrank=2).construct_task_nodes_1f1b(fns, m,
                                                                                    stage_rank=lambda s: 0)
    fe = FleetExecutor(nodes, num_threads=4)
    fe.run(timeout_s=30)
    fe.release()
    pos = {e: i for i, e in enumerate(log)}
    for s in range(2):
        assert [e for e in log if e[0] == s and e[1] == "lr"] == [(s, "lr", 0)]
        assert [e for e in log if e[0] == s and e[1] == "opt"] == [(s, "opt", m - 1)]
        assert pos[(s, "lr", 0)] < pos[(s, "fwd", 0)]
        assert pos[(s, "opt", m - 1)] > pos[(s, "bwd", m - 1)]
        for k in range(m):
            assert pos[(s, "fwd", k)] < pos[(s, "bwd", k)]
    for k in range(m):
        assert pos[(0, "fwd", k)] < pos[(1, "fwd", k)] < pos[(1, "bwd", k)] < pos[(0, "bwd", k)]
    outstanding = 0
    for st, kind, _ in log:
        if st == 0 and kind == "fwd":
            outstanding += 1
        elif st == 0 and kind == "bwd":
            outstanding -= 1
        assert outstanding <= 2


def test_error_in_task_is_raised():
    def boom(step):
        if step == 2:
            raise ValueError("bad micro-batch")

    src = TaskNode(0, 4, node_type="Source", task_id=1)
    a = TaskNode(0, 4, node_type="Compute", task_id=2, fn=boom)
    sink = TaskNode(0, 4, node_type="Sink", task_id=3)
    src.add_downstream_task(2)
    a.add_upstream_task(1)
    a.add_downstream_task(3)
    sink.add_upstream_task(2)
    fe = FleetExecutor([src, a, sink])
    with pytest.raises(RuntimeError, match="bad micro-batch"):
        fe.run(timeout_s=30)
    fe.release()


def test_static_program_task():
    import paddle2_amd as paddle

    main = paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main, paddle.static.Program()):
            x = paddle.static.data("x", [2], "float32")
            y = x * 3.0
    finally:
        paddle.disable_static()
    src = TaskNode(0, 3, node_type="Source", task_id=1)
    t = TaskNode(0, 3, node_type="Compute", task_id=2, program=main,
                 feed_fn=lambda s: {"x": np.full(2, s, "float32")}, fetch_list=[y])
    sink = TaskNode(0, 3, node_type="Sink", task_id=3)
    src.add_downstream_task(2)
    t.add_upstream_task(1)
    t.add_downstream_task(3)
    sink.add_upstream_task(2)
    fe = FleetExecutor([src, t, sink])
    fe.run(timeout_s=30)
    fe.release()
    assert [float(o[0][0]) for o in t.fetches] == [0.0, 3.0, 6.0]


def test_two_rank_pipeline_over_message_bus():
    res = run_workers("fleet_executor_worker.py", 2)
    assert res[1]["results"] == [4 * (2.0 * (k + 1) + 1.0) for k in range(6)] * 5  # 1 + 4 repeated runs
    assert [t[1] for t in res[0]["trace"]] == list(range(6))
