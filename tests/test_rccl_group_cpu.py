"""Multi-rank CPU test of the own ProcessGroupRCCL core (csrc/comm/rccl_core.h) — the code behind the ``pdrccl``
torch backend — against a threaded fake RCCL / HIP (csrc/comm/test/fake/): 4 ranks run every collective (all
reduce ops incl. avg / premul, reduce-scatter, all-gather, broadcast, reduce, all-to-all(-v)), pair-communicator
send / recv with the lo->hi rank mapping, coalesced p2p over several pair communicators, calc<->comm stream fences
against still-queued work, use_calc_stream, barrier, and timeout -> abort, under ThreadSanitizer and under
AddressSanitizer + UBSan.  Reference: paddle/fluid/distributed/collective/process_group_nccl.cc:840-847 (fences),
:999-1037 (p2p pair comms, coalescing)."""
import subprocess

import pytest

from paddle2_amd import _build


@pytest.mark.parametrize("kind", ["thread", "address"])
def test_rccl_group_core_four_ranks_under_sanitizer(kind):
    exe = _build.build_rccl_stress(kind)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr


def test_default_process_group_policy(monkeypatch):
    """The own group is the GPU default; PADDLE2_AMD_PG=c10d opts out; only an explicit request disables the
    fallback; the IPC all-reduce mode parses auto / on / off."""
    from paddle2_amd.distributed import ipc_allreduce, rccl_pg

    monkeypatch.delenv("PADDLE2_AMD_PG", raising=False)
    assert rccl_pg.enabled() and not rccl_pg.requested()
    monkeypatch.setenv("PADDLE2_AMD_PG", "c10d")
    assert not rccl_pg.enabled()
    monkeypatch.setenv("PADDLE2_AMD_PG", "rccl")
    assert rccl_pg.enabled() and rccl_pg.requested()
    monkeypatch.delenv("PADDLE2_AMD_IPC_ALLREDUCE", raising=False)
    assert ipc_allreduce._mode() == "auto"
    monkeypatch.setenv("PADDLE2_AMD_IPC_ALLREDUCE", "0")
    assert ipc_allreduce._mode() == "off"
    monkeypatch.setenv("PADDLE2_AMD_IPC_ALLREDUCE", "1")
    assert ipc_allreduce._mode() == "on"


def test_canary_agreement_through_store():
    """Ranks agree on the start-up verdict through the store: one failing rank makes every rank fall back."""
    import threading

    from paddle2_amd.distributed.rccl_pg import _agree

    class S:
        def __init__(self):
            self.d, self.lk = {}, threading.Lock()

        def set(self, k, v):
            with self.lk:
                self.d[k] = v.encode() if isinstance(v, str) else v

        def get(self, k):
            with self.lk:
                if k not in self.d:
                    raise KeyError(k)
                return self.d[k]

    st, out = S(), {}

    def rank(r):
        out[r] = _agree(st, "c", r, 3, "ok" if r != 1 else "error:x")

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(3)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert all(out[r] == ["ok", "error:x", "ok"] for r in range(3))
