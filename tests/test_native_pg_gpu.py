"""The framework's own RCCL process group ("pdrccl": csrc/comm/rccl_group.cpp + distributed/rccl_pg.py) on one
MI355X: every collective of the torch ProcessGroup surface, AVG / PreMulSum natively, coalescing, p2p in a
group, stream ordering of an async collective behind a long GEMM, non-contiguous outputs."""
import json
import os

from _dist import pypath as _pypath  # noqa: E402
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_native_rccl_process_group(tmp_path):
    from _dist import free_port

    out = tmp_path / "r.json"
    env = dict(os.environ, MASTER_PORT=str(free_port()), PYTHONPATH=_pypath(ROOT), PD_TEST_OUT=str(out))
    env.pop("PADDLE2_AMD_DEVICE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "workers", "native_pg_worker.py")], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["backend"] == "ProcessGroupRCCL", res
    base = [float(i) for i in range(1, 9)]
    assert res["sum"] == base and res["avg"] == base and res["max"] == base
    assert res["premul"] == [v * 0.5 for v in base] and res["premul_bf16"] == [v * 2 for v in base]
    assert res["noncontig"] == [[float(4 * i + j) for j in range(4)] for i in range(3)]
    assert res["async_exact"]
    assert res["bcast"] == [3.0, 4.0] and res["reduce"] == [5.0, 6.0]
    assert res["ag"] == [1.0, 2.0, 3.0] and res["ag_list"] == [1.0, 2.0, 3.0] and res["rs"] == [1.0, 2.0, 3.0, 4.0]
    assert res["a2a"] == [9.0, 8.0, 7.0, 6.0] and res["a2av"] == [1.0, 2.0, 3.0] and res["a2a_list"] == [4.0, 5.0]
    assert res["coalesced"] == [10.0, 21.0]
    assert res["p2p_self"] == [float(i) for i in range(6)]
    assert res["num_comms"] == 0 or res["num_comms"] >= 1
    assert res["canary"] == [True, ["ok"]], res["canary"]


def test_native_rccl_module_builds_and_loads():
    """CPU: the extension is built in-tree against librccl and exposes the group / task API."""
    from paddle2_amd import _rccl

    assert _rccl.version() >= 21800
    for name in ("all_reduce", "reduce_scatter", "all_gather", "all_to_all_v", "send", "recv", "group_start",
                 "group_end", "barrier", "abort"):
        assert hasattr(_rccl.RcclGroup, name)
