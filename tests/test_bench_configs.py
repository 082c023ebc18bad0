"""bench.py's BASELINE configs 4 and 5 in miniature, end to end through the bench entry point (self-launch, gloo):
Llama TP2 x PP2 (1F1B) and GPT fp8 TP2 + SP + sharding-3 on 4 CPU ranks; on the GPU box the same two paths with
2 ranks sharing cuda:0 (TP2 x PP1 1F1B-free, PP2, and fp8 TP2 + SP).  Each run must print one metric line with
the config's own parallelism and a finite loss."""
import json
import os
import subprocess
import sys

import pytest

from _dist import ROOT, pypath


def _bench(args, gpu=False, timeout=600):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_RANK"):
        env.pop(k, None)
    env.update({"PADDLE_DISTRI_BACKEND": "gloo", "PYTHONPATH": pypath(ROOT), "OMP_NUM_THREADS": "1"})
    env["PADDLE2_AMD_DEVICE"] = "gpu:0" if gpu else "cpu"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1]
    res = json.loads(line)
    assert res["value"] > 0 and res["final_loss"] == res["final_loss"] and res["final_loss"] > 0
    return res


def test_config4_llama_tp2_pp2_cpu():
    res = _bench(["--gpus", "4", "--model", "tiny", "--mp", "2", "--pp", "2", "--seq-len", "64", "--micro-batch", "2",
                  "--steps", "2", "--warmup", "1"])
    assert res["config"]["parallelism"] == "mp2xpp2(1F1B)" and res["config"]["accumulate_steps"] == 8
    assert res["config"]["global_batch"] == 16 and "mp2 x pp2(1F1B)" in res["metric"]


def test_config5_gpt_fp8_sp_sharding3_cpu():
    res = _bench(["--gpus", "4", "--model", "gpt3-tiny", "--fp8", "--mp", "2", "--sp", "--seq-len", "64",
                  "--micro-batch", "2", "--steps", "2", "--warmup", "1"])
    assert res["config"]["parallelism"] == "mp2+spxsharding3(2)" and res["dtype"].startswith("fp8")
    assert res["config"]["global_batch"] == 4


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["--model", "tiny", "--mp", "2"], ["--model", "tiny", "--pp", "2"],
                                  ["--model", "gpt3-tiny", "--fp8", "--mp", "2", "--sp"]])
def test_hybrid_bench_two_ranks_share_one_gpu(args):
    res = _bench(["--gpus", "2", "--seq-len", "128", "--micro-batch", "2", "--steps", "2", "--warmup", "1"] + args,
                 gpu=True, timeout=400)
    assert res["n_gpus"] == 2


def _bench_raw(args, timeout=600):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_RANK"):
        env.pop(k, None)
    env.update({"PADDLE_DISTRI_BACKEND": "gloo", "PYTHONPATH": pypath(ROOT), "OMP_NUM_THREADS": "1",
                "PADDLE2_AMD_DEVICE": "cpu"})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_bench_reports_communicator_self_diagnosis():
    """VERDICT r5 Next 4: the metric line names the process group that ran, the canary verdicts, the communicator's
    world size, the IPC all-reduce state, every rank's peak memory and stage 3's keep_gathered."""
    res = _bench(["--gpus", "4", "--model", "tiny", "--seq-len", "64", "--micro-batch", "2", "--steps", "2",
                  "--warmup", "1"])
    assert res["pg_backend"] == "gloo" and res["comm_world_size"] == 4
    assert len(res["peak_mem_gb_per_rank"]) == 4
    assert "canary" in res and "ipc_allreduce" in res
    assert res["stage3_keep_gathered"] is False      # CPU: the keep-gathered policy stays off
    assert res["hang_guard_s"] >= 300
    cp = res["comm_probe"]                           # the communicator's own bus bandwidth beside the number
    assert cp["mb_per_rank"] == 1.0
    for op in ("allgather", "reduce_scatter", "allreduce"):
        assert cp[op + "_busbw_GBps"] > 0 and cp[op + "_ms"] > 0


def test_bench_refuses_fallen_back_process_group():
    """A communicator other than the expected one (here: gloo where the run demands the native RCCL group, as after a
    failed start-up canary) ends the bench with exit status 3 and no metric line."""
    r = _bench_raw(["--gpus", "2", "--model", "tiny", "--seq-len", "64", "--micro-batch", "2", "--steps", "1",
                    "--warmup", "1", "--expect-pg", "pdrccl"])
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert '{"metric"' not in r.stdout and "expected 'pdrccl'" in r.stdout + r.stderr


def test_bench_pg_check_with_injected_canary_failure():
    sys.path.insert(0, ROOT)
    import bench

    status = {"backend": "c10d", "canary": ["ok", "rank 1: all_reduce mismatch (injected)"], "ipc": None}
    want = bench.expected_pg(8, True, True)
    assert want == "pdrccl"
    err = bench.pg_problem(status, want)
    assert err and "injected" in err and "'c10d'" in err
    assert bench.pg_problem(status, bench.expected_pg(8, True, True, "any")) is None
    assert bench.pg_problem({"backend": "c10d"}, bench.expected_pg(8, True, False)) is None   # explicit opt-out
    assert bench.expected_pg(1, True, True) is None
    assert bench.expected_pg(2, True, True, requested="gloo") == "gloo"    # explicit gloo on GPUs (shared-GPU tests)


def test_bench_hang_guard_exits_with_report():
    """A timed region that outlives its guard: every rank prints its communicator state and last collective per
    group, and the run exits 124 instead of hanging."""
    r = _bench_raw(["--gpus", "2", "--model", "tiny", "--seq-len", "64", "--micro-batch", "2", "--steps", "50",
                    "--warmup", "1", "--hang-guard-s", "0.05"])
    assert r.returncode != 0, r.stdout[-2000:]
    out = r.stdout + r.stderr
    assert "exceeded its guard" in out and '"last_ops"' in out, out[-3000:]
