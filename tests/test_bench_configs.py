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
