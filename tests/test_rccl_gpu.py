"""RCCL (torch "nccl" backend on ROCm) path on one MI355X: the ProcessGroup surface with GPU tensors in a
one-rank RCCL world (the collectives run through RCCL kernels, not the gloo fallbacks)."""
import json
import os

from _dist import pypath as _pypath  # noqa: E402
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_process_group_on_rccl(tmp_path):
    from _dist import free_port

    out = tmp_path / "r.json"
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()), PYTHONPATH=_pypath(ROOT), PD_TEST_OUT=str(out))
    env.pop("PADDLE_DISTRI_BACKEND", None)
    env.pop("PADDLE2_AMD_DEVICE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "workers", "rccl_pg_worker.py")], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["backend"] == "ProcessGroupNCCL" and res["device"].startswith("cuda")
    assert res["x"] == [1.0, 2.0, 3.0, 4.0] and res["y"] == [2.0, 4.0]
    assert res["rs"] == [1.0, 2.0, 3.0, 4.0] and res["ag"] == [5.0, 6.0, 7.0] and res["a2a"] == [9.0]
