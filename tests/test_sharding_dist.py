"""Sharding stages 1/2/3 on 2 gloo ranks must match a single-process run on the global batch
(reference test strategy: test/collective/fleet/dygraph_group_sharded_stage3.py compares against DP)."""
import pytest

from _dist import run_workers


@pytest.mark.parametrize("level", ["os", "os_g", "p_g_os"])
def test_group_sharded_matches_single(level):
    res = run_workers("sharding_worker.py", 2, [level])
    for r in res:
        for a, b in zip(r["losses"], r["ref"]):
            assert abs(a - b) < 1e-3 * max(1.0, abs(b)), (r["losses"], r["ref"])
        assert abs(r["csum"] - r["csum_ref"]) < 1e-2 * max(1.0, abs(r["csum_ref"])), (r["csum"], r["csum_ref"])
