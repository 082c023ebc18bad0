"""Multi-process test harness: spawn N ranks on localhost (gloo on CPU), like the reference's
TestMultipleAccelerators / CommunicationTestDistBase (test/legacy_test/test_parallel_dygraph_dataparallel.py:100-209)."""
import json
import os
import socket
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pypath(root):
    """PYTHONPATH for a child process: ``root`` first, then the caller's entries (an interposer some harnesses put
    there, e.g. a loaded-library recorder, must survive into the children)."""
    old = os.environ.get("PYTHONPATH", "")
    return root if not old else root + os.pathsep + old


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_workers(script, nprocs, args=(), timeout=300, extra_env=None):
    """Run ``script`` as ``nprocs`` ranks; returns the list of per-rank JSON results."""
    port = free_port()
    out_dir = tempfile.mkdtemp(prefix="pd_dist_")
    procs = []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(nprocs), "LOCAL_RANK": str(r), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "PADDLE_TRAINER_ID": str(r), "PADDLE_TRAINERS_NUM": str(nprocs),
                    "PD_TEST_OUT": os.path.join(out_dir, f"rank{r}.json"), "PYTHONPATH": pypath(ROOT),
                    "PADDLE2_AMD_DEVICE": "cpu", "OMP_NUM_THREADS": "1", "PADDLE_DISTRI_BACKEND": "gloo"})
        if extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "workers", script)] + list(args),
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    failed = False
    for r, p in enumerate(procs):
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
            failed = True
        outs.append(o)
        # an abort during interpreter teardown AFTER the rank wrote its complete result (gloo / store threads
        # torn down at exit: "terminate called without an active exception") does not invalidate the result
        done = p.returncode in (-6, 134) and "terminate called" in o and _complete(
            os.path.join(out_dir, f"rank{r}.json"))
        failed |= p.returncode != 0 and not done
    if failed:
        raise AssertionError("worker failed:\n" + "\n----\n".join(o[-3000:] for o in outs))
    res = []
    for r in range(nprocs):
        with open(os.path.join(out_dir, f"rank{r}.json")) as f:
            res.append(json.load(f))
    return res


def _complete(path):
    try:
        with open(path) as f:
            json.load(f)
        return True
    except (OSError, ValueError):
        return False


def write_result(obj):
    with open(os.environ["PD_TEST_OUT"], "w") as f:
        json.dump(obj, f)
