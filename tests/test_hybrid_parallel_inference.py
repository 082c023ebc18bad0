"""Pipeline(+mp)-parallel static inference: device_guard-annotated program (stage chain + a generation
while-loop spanning the stages) split per rank by HybridParallelInferenceHelper, run over gloo; results
must match the unsplit program (reference test: test/collective/fleet/hybrid_parallel_inference_helper.py)."""
import pytest

import paddle2_amd as paddle
from _dist import run_workers
from paddle2_amd.distributed.fleet.utils.hybrid_parallel_inference import HybridParallelInferenceHelper


@pytest.mark.parametrize("num_pp,num_mp", [(2, 1), (3, 1), (2, 2)])
def test_pipeline_inference_matches_unsplit(num_pp, num_mp):
    res = run_workers("pp_infer_worker.py", num_pp * num_mp, args=(str(num_pp), str(num_mp)))
    for r in res:
        assert r["i_ok"] and r["tok_err"] < 1e-6 and r["h_err"] < 1e-6, r
        assert r["stage"] == r["rank"] // num_mp
        assert r["n_ops"] < r["n_ops_full"] + r["sends"] + r["recvs"] + 2
    # every stage hands values on: the first stage sends, the last receives
    assert res[0]["sends"] > 0 and res[-1]["recvs"] > 0
    assert res[0]["pp_group"] == [i * num_mp for i in range(num_pp)]


def test_device_guard_annotates_ops():
    main, startup = paddle.static.Program(), paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main, startup):
            x = paddle.static.data("x", [2, 4], "float32")
            with paddle.static.device_guard("gpu:1"):
                y = x * 2.0
            z = y + 1.0
    finally:
        paddle.disable_static()
    devs = [o.attrs.get("op_device") for o in main.ops]
    assert devs == ["gpu:1", None]
    with pytest.raises(ValueError):
        paddle.static.device_guard("npu:0")
    with pytest.raises(ValueError):
        HybridParallelInferenceHelper(startup, main, num_mp=1, num_pp=2)   # 1 rank, 2 stages
    assert z is not None
