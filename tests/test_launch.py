"""Launcher / spawn (reference tests: test/legacy_test/test_launch_coverage.py, test_spawn_and_init_parallel_env.py)."""
import os

from _dist import pypath as _pypath  # noqa: E402
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys
sys.path.insert(0, %r)
import paddle2_amd as paddle
import paddle2_amd.distributed as dist
dist.init_parallel_env()
t = paddle.to_tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
assert float(t) == sum(range(1, dist.get_world_size() + 1))
assert os.environ["PADDLE_TRAINERS_NUM"] == str(dist.get_world_size())
if os.environ.get("FAIL_ONCE") and not os.path.exists(os.environ["FAIL_ONCE"]) and dist.get_rank() == 1:
    open(os.environ["FAIL_ONCE"], "w").close()
    sys.exit(3)
print("OK rank", dist.get_rank(), flush=True)
''' % ROOT


def _env():
    env = dict(os.environ, PYTHONPATH=_pypath(ROOT), PADDLE2_AMD_DEVICE="cpu", PADDLE_DISTRI_BACKEND="gloo")
    return env


def test_launch_single_node(tmp_path):
    w = tmp_path / "w.py"
    w.write_text(WORKER)
    r = subprocess.run([sys.executable, "-m", "paddle2_amd.distributed.launch", "--nproc_per_node", "2", "--log_dir",
                        str(tmp_path / "log"), str(w)], env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    assert "OK rank 0" in r.stdout
    assert "OK rank 1" in (tmp_path / "log" / "workerlog.1").read_text()


def test_launch_restarts_failed_pod(tmp_path):
    w = tmp_path / "w.py"
    w.write_text(WORKER)
    env = _env()
    env["FAIL_ONCE"] = str(tmp_path / "failed_once")
    r = subprocess.run([sys.executable, "-m", "paddle2_amd.distributed.launch", "--nproc_per_node", "2",
                        "--max_restart", "1", "--log_dir", str(tmp_path / "log"), str(w)], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    assert "restarting pod" in r.stderr


def test_launch_propagates_failure(tmp_path):
    w = tmp_path / "w.py"
    w.write_text("import sys; sys.exit(5)\n")
    r = subprocess.run([sys.executable, "-m", "paddle2_amd.distributed.launch", "--nproc_per_node", "2", "--log_dir",
                        str(tmp_path / "log"), str(w)], env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 5


def _spawn_fn(x):
    import paddle2_amd as paddle
    import paddle2_amd.distributed as dist

    dist.init_parallel_env()
    t = paddle.to_tensor([x])
    dist.all_reduce(t)
    assert float(t) == x * dist.get_world_size()


def test_spawn():
    os.environ["PADDLE2_AMD_DEVICE"] = "cpu"
    import paddle2_amd.distributed as dist

    dist.spawn(_spawn_fn, args=(2.0,), nprocs=2, backend="gloo")


def _bench_json(stdout):
    import json

    lines = [l for l in stdout.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_self_launches_ranks():
    """bench.py --gpus 2 (no WORLD_SIZE) starts 2 ranks through the in-tree launcher and reports n_gpus=2,
    on the same stage-3 sharding path as every other N."""
    env = _env()
    env.pop("WORLD_SIZE", None)
    args = ["--model", "tiny", "--steps", "2", "--warmup", "1", "--seq-len", "32", "--micro-batch", "2"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + args, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = _bench_json(r.stdout)
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 4
    assert out["config"]["parallelism"] == "sharding3x2"
    assert out["steps"] == 2 and out["warmup"] == 1


def test_bench_single_runs_sharding3_and_rejects_world_mismatch():
    env = _env()
    env.pop("WORLD_SIZE", None)
    args = ["--model", "tiny", "--steps", "1", "--warmup", "1", "--seq-len", "32", "--micro-batch", "2"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = _bench_json(r.stdout)
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "sharding3x1"
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"] + args, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_gpt_tied_embedding_under_stage3():
    """GPT ties the logits to the word embedding: under stage-3 sharding that layer stays in the root unit
    (gathered all step) instead of being released after the embedding forward."""
    env = _env()
    env.pop("WORLD_SIZE", None)
    args = ["--model", "gpt3-1.3b", "--layers", "2", "--seq-len", "32", "--micro-batch", "1", "--steps", "1",
            "--warmup", "1"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _bench_json(r.stdout)
    assert out["config"]["parallelism"] == "sharding3x1" and out["final_loss"] > 0
