"""Elastic scale-in (reference: test/collective/fleet/test_fleet_elastic_manager.py and the
launch elastic controller): two launcher 'nodes' with --nnodes 1:2 rendezvous over the native
TCPStore; when one node dies the survivor detects the missing heartbeat, re-rendezvouses and
restarts its worker with world size 1."""
import os

from _dist import pypath as _pypath  # noqa: E402
import signal
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wait(pred, timeout):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.2)
    return False


@pytest.mark.timeout(240)
def test_elastic_scale_in(tmp_path):
    port = _port()
    env = dict(os.environ, PYTHONPATH=_pypath(ROOT), PADDLE_DISTRI_BACKEND="gloo")
    env.pop("CUDA_VISIBLE_DEVICES", None)
    base = [sys.executable, "-m", "paddle2_amd.distributed.launch", "--master", f"127.0.0.1:{port}", "--nnodes",
            "1:2", "--nproc_per_node", "1", "--elastic_ttl", "2", "--host", "127.0.0.1", "--job_id", "el"]
    script = [os.path.join(ROOT, "tests", "workers", "elastic_worker.py"), str(tmp_path)]
    a = subprocess.Popen(base + ["--rank", "0", "--log_dir", str(tmp_path / "la")] + script, env=env, cwd=ROOT,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
    time.sleep(1.0)
    b = subprocess.Popen(base + ["--log_dir", str(tmp_path / "lb")] + script, env=env, cwd=ROOT,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)
    try:
        assert _wait(lambda: (tmp_path / "round_w2_r0").exists() and (tmp_path / "round_w2_r1").exists(), 90), \
            os.listdir(tmp_path)
        os.killpg(b.pid, signal.SIGKILL)  # node B dies (its launcher and worker)
        b.wait(timeout=30)
        assert _wait(lambda: (tmp_path / "round_w1_r0").exists(), 90), os.listdir(tmp_path)
        (tmp_path / "stop").write_text("1")
        out, _ = a.communicate(timeout=90)
        assert a.returncode == 0, out.decode()[-3000:]
        assert b"elastic round" in out
    finally:
        for p in (a, b):
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
