"""Context parallelism (Ulysses all-to-all and zigzag ring flash attention over the sep axis) on gloo
ranks vs. full-sequence single-process attention / Llama (reference sep tests compare against single-card
runs, test/collective/fleet/hybrid_parallel_sep_model.py:213-235)."""
import pytest

from _dist import run_workers


@pytest.mark.parametrize("kind", ["ulysses", "ring"])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("n", [2, 4])
def test_context_parallel_attention_matches_full(kind, causal, n):
    if kind == "ulysses" and n == 4 and not causal:
        pytest.skip("covered by the causal case")
    for r in run_workers("cp_worker.py", n, ["attn", kind, "1" if causal else "0"]):
        assert max(r.values()) < 1e-4, r


@pytest.mark.parametrize("kind", ["ulysses", "ring"])
def test_context_parallel_llama_matches_single(kind):
    for r in run_workers("cp_worker.py", 2, ["llama", kind]):
        assert abs(r["loss"] - r["loss_ref"]) < 1e-4 * max(1.0, abs(r["loss_ref"])), r
        assert r["grad_rel"] < 1e-3, r
