"""The bench's N>1 GPU code path on one MI355X: two ranks share cuda:0 and exchange over gloo (RCCL cannot
place two ranks on one device), so stage-3 all-gather / reduce-scatter / barrier / max-over-ranks timing run on
device tensors end to end (tiny Llama, bench.py self-launch)."""
import json
import os

from _dist import pypath as _pypath  # noqa: E402
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_share_one_gpu():
    env = dict(os.environ)
    env.update({"PADDLE_DISTRI_BACKEND": "gloo", "PADDLE2_AMD_DEVICE": "gpu:0", "PYTHONPATH": _pypath(ROOT)})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "tiny",
                        "--seq-len", "512", "--micro-batch", "2", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["value"] > 0 and res["config"]["global_batch"] == 4
    assert res["final_loss"] == res["final_loss"] and res["final_loss"] > 0
