"""Pruning rules (reference: auto_tuner/prune.py — prune_by_mp, prune_by_pp, prune_by_mbs,
prune_by_sharding, prune_by_recompute, prune_by_memory_estimation, ...).  Each rule returns True
when the candidate must be skipped."""
from __future__ import annotations

from .cost_model import HBM_GB, estimate_memory_gb

_PRUNE_FUNC = []


def register_prune(fn):
    _PRUNE_FUNC.append(fn)
    return fn


@register_prune
def prune_by_world(tuner_cfg, cur, history):
    n = tuner_cfg["num_gpus"]
    return cur["dp_degree"] * cur["mp_degree"] * cur["pp_degree"] * cur["sharding_degree"] != n


@register_prune
def prune_by_mp(tuner_cfg, cur, history):
    m = tuner_cfg["model_cfg"]
    mp = cur["mp_degree"]
    if mp > tuner_cfg.get("gpus_per_node", 8):
        return True  # keep TP inside one xGMI-connected node
    for key in ("num_attention_heads", "hidden_size", "vocab_size"):
        if m.get(key) and m[key] % mp:
            return True
    kv = m.get("num_key_value_heads")
    return bool(kv and kv % mp and mp % kv)


@register_prune
def prune_by_pp(tuner_cfg, cur, history):
    L = tuner_cfg["model_cfg"]["num_layers"]
    pp = cur["pp_degree"]
    if L % pp:
        return True
    gbs = tuner_cfg["model_cfg"]["global_batch_size"]
    acc = gbs // (cur["dp_degree"] * cur["sharding_degree"] * cur["micro_batch_size"])
    return pp > 1 and acc < pp  # 1F1B needs at least pp micro batches


@register_prune
def prune_by_mbs(tuner_cfg, cur, history):
    gbs = tuner_cfg["model_cfg"]["global_batch_size"]
    return gbs % (cur["dp_degree"] * cur["sharding_degree"] * cur["micro_batch_size"]) != 0


@register_prune
def prune_by_sharding(tuner_cfg, cur, history):
    return cur["sharding_degree"] == 1 and cur.get("sharding_stage", 1) > 1


@register_prune
def prune_by_memory_estimation(tuner_cfg, cur, history):
    budget = tuner_cfg.get("max_mem_usage_gb", HBM_GB * 0.92)
    est = estimate_memory_gb(tuner_cfg["model_cfg"], cur)
    cur["estimated_memory_gb"] = round(est, 1)
    return est > budget


@register_prune
def prune_by_history_oom(tuner_cfg, cur, history):
    """A config that needs at least as much memory as one that already OOM'd is skipped."""
    for h in history:
        if h.get("has_error") == "OOM" and h.get("estimated_memory_gb", 1e9) <= cur.get("estimated_memory_gb", 0):
            return True
    return False
