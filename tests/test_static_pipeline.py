"""Static pipeline training across ranks (incubate.optimizer.PipelineOptimizer + distributed/passes
StagePlanExecutor; reference python/paddle/incubate/optimizer/pipeline.py and
distributed/passes/pipeline_scheduler_pass/) and DistributedFusedLamb's sharded update, on 2 gloo ranks."""
import numpy as np
import pytest

from _dist import run_workers


@pytest.mark.parametrize("mode", ["FThenB", "1F1B", "Eager1F1B"])
def test_static_pipeline_two_stages_matches_serial(mode):
    res = sorted(run_workers("static_pipeline_worker.py", 2, args=(mode,)), key=lambda o: o["stage"])
    s0, s1 = res
    # the loss lives on the last stage; the first stage fetches nothing for it
    assert all(v is None for v in s0["losses"])
    np.testing.assert_allclose(s1["losses"], s1["ref"], rtol=1e-5, atol=1e-6)
    for o in res:
        assert o["param_err"] < 1e-5, o
        assert o["other_moved"] > 1e-4      # the other stage's copy here is not trained by this rank
    assert s0["n_send"] == 1 and s0["n_recv"] == 0 and s1["n_send"] == 0 and s1["n_recv"] == 1


def test_distributed_fused_lamb_sharded_matches_lamb():
    for o in run_workers("static_pipeline_worker.py", 2, args=("dfl",)):
        assert o["param_err"] < 1e-5, o
