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


def _close(a, b, tol=2e-3):
    for x, y in zip(a, b):
        assert abs(x - y) < tol * max(1.0, abs(y)), (a, b)


@pytest.mark.parametrize("opt", ["offload", "exclude"])
def test_stage3_offload_exclude_4ranks(opt, tmp_path):
    """4 gloo ranks: stage 3 with host-offloaded optimizer state / exclude_layer matches one process."""
    res = run_workers("sharding_ckpt_worker.py", 4, ["train", opt, str(tmp_path / "ck")])
    for r in res:
        _close(r["losses"], r["ref"])
        if opt == "exclude":
            assert r["norm_full"]


def test_stage3_checkpoint_resumes_at_other_degree(tmp_path):
    """Checkpoint written by 4 sharded ranks (reference per-parameter layout) resumes on 2 ranks and
    continues exactly like an uninterrupted single-process run."""
    ck = str(tmp_path / "ck")
    run_workers("sharding_ckpt_worker.py", 4, ["train", "plain", ck])
    res = run_workers("sharding_ckpt_worker.py", 2, ["resume", "plain", ck])
    for r in res:
        _close(r["losses"], r["ref"])


def test_stage3_grad_buffers_bounded_4ranks():
    """4 gloo ranks, 6 decoder layers, stage 3: at most 2 fp32 flat unit-gradient buffers are ever alive (the one
    being written + one reduce-scatter in flight), buffers are recycled, and losses / parameters still match the
    single-process run (reference keeps a full fp32 grad per parameter alive: group_sharded_stage3.py:743-805)."""
    res = run_workers("sharding_worker.py", 4, ["p_g_os"], extra_env={"PD_TEST_LAYERS": "6"})
    for r in res:
        for a, b in zip(r["losses"], r["ref"]):
            assert abs(a - b) < 1e-3 * max(1.0, abs(b)), (r["losses"], r["ref"])
        assert abs(r["csum"] - r["csum_ref"]) < 1e-2 * max(1.0, abs(r["csum_ref"]))
        assert r["peak_live_flat"] is not None and r["peak_live_flat"] <= 2, r["peak_live_flat"]
        # recycled per unit size (6 equal decoder layers share their buffers), not re-allocated per unit
        assert r["pool_bufs"] <= 2 * r["unit_sizes"] < 12, (r["pool_bufs"], r["unit_sizes"])


def test_stage3_keep_gathered_skips_backward_gathers():
    """PADDLE2_AMD_STAGE3_KEEP_GATHERED=1 (the MI355X default when the bf16 model is <= 8 % of HBM): units stay
    gathered from forward to backward, so the backward issues no all-gather — fewer gathers per step than the
    re-gathering path, the same losses / parameters as the single-process run."""
    keep = run_workers("sharding_worker.py", 2, ["p_g_os"],
                       extra_env={"PD_TEST_LAYERS": "4", "PADDLE2_AMD_STAGE3_KEEP_GATHERED": "1"})
    regather = run_workers("sharding_worker.py", 2, ["p_g_os"],
                           extra_env={"PD_TEST_LAYERS": "4", "PADDLE2_AMD_STAGE3_KEEP_GATHERED": "0"})
    for r in keep + regather:
        for a, b in zip(r["losses"], r["ref"]):
            assert abs(a - b) < 1e-3 * max(1.0, abs(b)), (r["losses"], r["ref"])
        assert abs(r["csum"] - r["csum_ref"]) < 1e-2 * max(1.0, abs(r["csum_ref"]))
    assert all(r["keep"] for r in keep) and not any(r["keep"] for r in regather)
    assert keep[0]["losses"] == regather[0]["losses"]
    # 3 steps x 4 decoder units: the re-gathering path gathers most units twice per step, keep_gathered once
    assert keep[0]["gathers"] < regather[0]["gathers"], (keep[0]["gathers"], regather[0]["gathers"])
    assert keep[0]["gathers"] <= 3 * keep[0]["n_units"] + 1


def test_stage3_kept_units_released_without_backward():
    """with keep_gathered, a grad-enabled forward that never gets a backward (eval without no_grad)
    leaves its units gathered; the next forward releases them instead of holding them for good."""
    res = run_workers("sharding_worker.py", 2, ["p_g_os"],
                      extra_env={"PD_TEST_LAYERS": "4", "PADDLE2_AMD_STAGE3_KEEP_GATHERED": "1",
                                 "PD_TEST_EVAL_NO_BWD": "1"})
    for r in res:
        assert r["held_after_eval"] >= 3, r          # kept for a backward that never comes
        assert r["held_next"] == 0, r                # released by the next (no-grad) forward


def test_stage3_comm_model_llama7b():
    """Bytes per rank per step of stage 3 at N = 8 for Llama-2-7B: all-gathers of the bf16 flat units (forward and
    backward, the last unit kept across the turn) and one fp32 reduce-scatter per unit."""
    from paddle2_amd.distributed.sharding import comm_model as CM

    units, root = CM.llama_units()
    assert units[0] == 202_383_360 and len(units) == 32          # 7B decoder layer parameters
    b = CM.stage3_bytes_per_step(units, 8, root_numel=root)
    layer_ag = 202_383_360 * 2 * 7 / 8
    assert abs(b["max_unit_ag"] - layer_ag) < 16
    assert abs(b["ag_bwd"] - 31 * layer_ag) < 1e3
    assert abs(b["rs"] / b["ag_bwd"] - 2 * (32 * 202_383_360 + root) / (31 * 202_383_360)) < 1e-6
    assert 40e9 < b["total"] < 50e9                               # ~45 GB per rank per step
    b16 = CM.stage3_bytes_per_step(units, 8, grad_bytes=2, root_numel=root)
    assert abs((b["total"] - b16["total"]) - b["rs"] / 2) < 1e3   # bf16 reduce-scatter saves half the RS bytes
    assert CM.stage3_bytes_per_step(units, 1)["total"] == 0
    kept = CM.stage3_bytes_per_step(units, 8, root_numel=root, keep_gathered=True)
    assert kept["ag_bwd"] == 0 and abs((b["total"] - kept["total"]) - b["ag_bwd"]) < 1e3   # ~11 GB less per step
