"""Stage 3's N > 1 collective path forced on one rank (PADDLE2_AMD_STAGE3_FORCE_COMM=1: real all-gather /
reduce-scatter on the group's process group, the fp32 flat-gradient pool, prefetch, retire_rs) trains bit for bit
like the N = 1 short-circuit (reference group_sharded_stage3.py:851-1074).  CPU: gloo; GPU: the framework's RCCL
group on the comm stream."""
import json
import os
import subprocess
import sys
import tempfile

import pytest

from _dist import ROOT, pypath


def _run(dev, force, acc=1, keep="auto"):
    out = os.path.join(tempfile.mkdtemp(prefix="pd_fc_"), "r.json")
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_RANK"):
        env.pop(k, None)
    env.update({"PYTHONPATH": pypath(ROOT), "PD_TEST_OUT": out, "PD_TEST_DEVICE": dev, "PD_TEST_ACC": str(acc),
                "PADDLE2_AMD_STAGE3_FORCE_COMM": "1" if force else "0", "OMP_NUM_THREADS": "2",
                "PADDLE2_AMD_STAGE3_KEEP_GATHERED": keep})
    if dev == "cpu":
        env.update({"PADDLE2_AMD_DEVICE": "cpu", "PADDLE_DISTRI_BACKEND": "gloo"})
    else:
        # deterministic flash backward (per-key-block dQ slabs summed in a fixed order): the default fp32-atomic dQ
        # makes two identical runs differ in the last bits, which would hide what this test compares
        env["PADDLE2_AMD_FA_DQ_ATOMIC"] = "0"
        env["FLAGS_embedding_deterministic"] = "1"   # the embedding gradient's fp32 atomics, likewise
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "workers", "force_comm_worker.py")], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-4000:]
    with open(out) as f:
        return json.load(f)


def _check(dev, acc):
    a, b = _run(dev, False, acc), _run(dev, True, acc)
    assert not any(a["comm"]) and not a["initialized"]
    assert all(b["comm"]) and b["initialized"] and b["peak_live_flat"] >= 1
    assert a["losses"] == b["losses"]
    assert a["digest"] == b["digest"]
    return b


@pytest.mark.parametrize("acc", [1, 2])
def test_force_comm_matches_short_circuit_cpu(acc):
    _check("cpu", acc)


@pytest.mark.gpu
@pytest.mark.parametrize("acc", [1, 2])
def test_force_comm_matches_short_circuit_gpu(acc):
    """The runs use the deterministic flash dQ and embedding gradient, so the short-circuit path normally repeats
    bit for bit and the forced-comm run must then match it bitwise.  Should some other kernel still add with
    atomics (two short-circuit runs differ), the losses diverge chaotically from the first differing bit over the
    4 steps, so the bound is a multiple of that run-to-run noise with a floor of 5e-3 (a missing or doubled
    gradient moves the losses by far more)."""
    a, a2, b = _run("cuda", False, acc), _run("cuda", False, acc), _run("cuda", True, acc)
    assert not any(a["comm"]) and all(b["comm"]) and b["initialized"] and b["pg"] == "pdrccl"
    assert a["losses"][0] == b["losses"][0]   # the first forward reads the same parameters
    noise = max(abs(x - y) for x, y in zip(a["losses"], a2["losses"]))
    diff = max(abs(x - y) for x, y in zip(a["losses"], b["losses"]))
    if noise == 0.0:
        assert a["losses"] == b["losses"] and a["digest"] == b["digest"], (a, b)
    else:
        assert diff <= max(8 * noise, 5e-3), (a["losses"], a2["losses"], b["losses"])


@pytest.mark.gpu
def test_force_comm_keep_gathered_gpu():
    """Forced comm with every unit kept gathered from forward to backward (the N > 1 MI355X default): the same
    training as the N = 1 short-circuit on the GPU comm path."""
    a, a2, b = _run("cuda", False), _run("cuda", False), _run("cuda", True, keep="1")
    assert all(b["comm"]) and b["pg"] == "pdrccl"
    assert a["losses"][0] == b["losses"][0]
    noise = max(abs(x - y) for x, y in zip(a["losses"], a2["losses"]))
    if noise == 0.0:
        assert a["losses"] == b["losses"] and a["digest"] == b["digest"], (a, b)
    else:
        assert max(abs(x - y) for x, y in zip(a["losses"], b["losses"])) <= max(8 * noise, 5e-3)


def test_force_comm_keep_gathered_cpu():
    a, b = _run("cpu", False), _run("cpu", True, keep="1")
    assert all(b["comm"]) and a["losses"] == b["losses"] and a["digest"] == b["digest"]
