"""Pruning rules of the auto tuner (reference: python/paddle/distributed/auto_tuner/prune.py —
prune_by_mp :129, prune_by_pp :173, prune_by_vpp :234, prune_by_mbs :307, prune_by_sharding :395,
prune_by_recompute :486, prune_by_num_gpus :588, prune_by_memory_estimation :605,
prune_by_invalid_strategy :812, prune_by_refined_recompute :823 and their ``*_history`` twins).

Two registries: ``register_prune`` rules look at the candidate alone (``(tuner_cfg, cur_cfg,
history_cfgs)``), ``register_prune_history`` rules compare it with configurations already run or
pruned (``(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs)``): a dimension that only trades memory for
speed is skipped when its faster neighbour already ran (``time`` > 0) or its leaner neighbour already
OOM'd (``max_mem_usage == "OOM"``).  Each rule returns True to skip; the reason is kept in
``tuner_cfg['pruned_reasons']``.  MI355X additions: TP stays inside one node's xGMI mesh, GQA head
counts must split evenly, and the default memory check is the analytical model against 288 GB HBM3E.
"""
from __future__ import annotations

import os
import subprocess
import sys

from .cost_model import HBM_GB, estimate_memory_gb
from .utils import _matched

_PRUNE_FUNC = []
_PRUNE_HISTORY_FUNC = []


def register_prune(fn):
    _PRUNE_FUNC.append(fn)
    return fn


def register_prune_history(fn):
    _PRUNE_HISTORY_FUNC.append(fn)
    return fn


def log_pruned_info(cur_cfg, reason, tuner_cfg):
    tuner_cfg.setdefault("pruned_reasons", []).append((dict(cur_cfg), reason))


def same_cfgs_beside(attrs, cur_cfg, history_cfgs=()):
    """History configs equal to ``cur_cfg`` on every dimension except ``attrs``."""
    attrs = [attrs] if isinstance(attrs, str) else list(attrs)
    skip = set(attrs) | {"time", "max_mem_usage", "has_error", "error_info", "job_id", "task_id", "wall_s",
                         "estimated_memory_gb", "estimated_step_time_s", "recompute_level"}
    out = []
    for h in history_cfgs:
        if all(h.get(k) == v for k, v in cur_cfg.items() if k not in skip and not isinstance(v, dict)):
            out.append(h)
    return out


def _cands(tuner_cfg, key):
    v = tuner_cfg.get(key)
    if v == "auto":
        return tuner_cfg.get("candidates", {}).get(key)
    if isinstance(v, int) and not isinstance(v, bool):
        return [v]
    return v if isinstance(v, list) else None


def _gbs(tuner_cfg, cur_cfg):
    g = cur_cfg.get("global_batch_size") or tuner_cfg["model_cfg"].get("global_batch_size")
    return None if g == "auto" else g


def _recompute_level(cfg):
    rc = cfg.get("use_recompute")
    if rc is None:
        return None
    if not rc:
        return 0
    return {"full": 3, "full_attn": 2, "core_attn": 1}.get(cfg.get("recompute_granularity"), 3)


@register_prune
def prune_by_num_gpus(tuner_cfg, cur_cfg, history_cfgs=()):
    n = cur_cfg.get("num_gpus", tuner_cfg.get("num_gpus"))
    prod = 1
    for k in ("dp_degree", "mp_degree", "pp_degree", "sharding_degree"):
        prod *= cur_cfg.get(k, 1) or 1
    return prod != n


@register_prune
def prune_by_mp(tuner_cfg, cur_cfg, history_cfgs=()):
    mp = cur_cfg.get("mp_degree")
    if mp is None:
        return False
    m = tuner_cfg["model_cfg"]
    for key in ("hidden_size", "vocab_size", "num_attention_heads"):
        if m.get(key) and m[key] % mp:
            return True
    kv = m.get("num_key_value_heads")
    if kv and kv % mp and mp % kv:
        return True   # GQA: kv heads split evenly or replicate evenly
    if m.get("seq_length") and m["seq_length"] % mp and tuner_cfg.get("use_sequence_parallel", False):
        return True
    if tuner_cfg.get("enable_mp_prune", True) and mp > tuner_cfg.get("gpus_per_node", 8):
        log_pruned_info(cur_cfg, f"mp_degree {mp} leaves the node's xGMI mesh", tuner_cfg)
        return True
    c = _cands(tuner_cfg, "mp_degree")
    return bool(c) and mp not in c


@register_prune
def prune_by_pp(tuner_cfg, cur_cfg, history_cfgs=()):
    pp = cur_cfg.get("pp_degree")
    if pp is None:
        return False
    L = tuner_cfg["model_cfg"].get("num_layers")
    if L and L % pp:
        return True
    c = _cands(tuner_cfg, "pp_degree")
    if c:
        return pp not in c
    nodes = cur_cfg.get("nodes", tuner_cfg.get("nodes", 1))
    return nodes != 1 and pp > nodes


@register_prune
def prune_by_vpp(tuner_cfg, cur_cfg, history_cfgs=()):
    pp, vpp = cur_cfg.get("pp_degree"), cur_cfg.get("vpp_degree")
    if pp is None or vpp is None:
        return False
    L = tuner_cfg["model_cfg"].get("num_layers")
    if L:
        g = _gbs(tuner_cfg, cur_cfg)
        if g:
            acc = g // cur_cfg.get("dp_degree", 1) // cur_cfg.get("sharding_degree", 1) // cur_cfg["micro_batch_size"]
            if vpp > 1 and acc % pp:
                return True
        if L % (pp * vpp):
            return True
        if vpp != 1 and pp <= 2:
            return True   # interleaving only pays with >2 stages
    c = _cands(tuner_cfg, "vpp_degree")
    return bool(c) and vpp not in c


@register_prune
def prune_by_mbs(tuner_cfg, cur_cfg, history_cfgs=()):
    mbs = cur_cfg.get("micro_batch_size")
    if mbs is None:
        return False
    g = _gbs(tuner_cfg, cur_cfg)
    if g:
        local = g // cur_cfg.get("dp_degree", 1) // cur_cfg.get("sharding_degree", 1)
        if local == 0 or local % mbs:
            return True
        acc = local // mbs
        pp = cur_cfg.get("pp_degree")
        if pp is not None and acc < pp:
            return True   # 1F1B needs at least pp micro-batches in flight
        vpp = cur_cfg.get("vpp_degree")
        if vpp and vpp > 1 and pp and acc % pp:
            return True
    c = _cands(tuner_cfg, "micro_batch_size")
    return bool(c) and mbs not in c


@register_prune
def prune_by_sharding(tuner_cfg, cur_cfg, history_cfgs=()):
    stage, deg, pp = cur_cfg.get("sharding_stage"), cur_cfg.get("sharding_degree"), cur_cfg.get("pp_degree")
    if not stage or not deg:
        return False
    c = _cands(tuner_cfg, "sharding_stage")
    if c and stage not in c:
        return True
    c = _cands(tuner_cfg, "sharding_degree")
    if c and deg not in c:
        return True
    if pp and pp != 1 and stage != 1 and deg != 1:
        return True   # stage 2/3 re-gathers parameters per micro-batch: not combined with pipelining
    if deg == 1 and same_cfgs_beside("sharding_stage", cur_cfg, history_cfgs):
        return True   # stages are identical without sharding: keep one
    return False


@register_prune
def prune_by_recompute(tuner_cfg, cur_cfg, history_cfgs=()):
    rc, gran = cur_cfg.get("use_recompute"), cur_cfg.get("recompute_granularity")
    if rc is None:
        return False
    cands = tuner_cfg.get("candidates", {})
    if cands.get("use_recompute") and rc not in cands["use_recompute"]:
        return True
    if cands.get("recompute_granularity") and gran and gran not in cands["recompute_granularity"]:
        return True
    if not rc:
        if gran not in (None, "full"):
            return True   # granularity is meaningless without recompute: keep one copy
        level = _recompute_level(cur_cfg)
        for h in same_cfgs_beside(["use_recompute", "recompute_granularity"], cur_cfg, history_cfgs):
            if _recompute_level(h) == level:
                return True
    return False


@register_prune
def prune_by_memory_estimation(tuner_cfg, cur_cfg, history_cfgs=()):
    """External ``memory_estimation_tool`` (prints MiB) when configured, else the analytical model against
    ``max_mem_usage`` GiB (default 92% of 288 GB HBM3E)."""
    tool = tuner_cfg.get("memory_estimation_tool")
    if tool:
        if not os.path.exists(tool):
            raise ValueError(f"memory_estimation_tool should be a valid path, got {tool}")
        if tuner_cfg.get("max_mem_usage") is None:
            raise ValueError("max_mem_usage must be set when using a memory estimation tool")
        cmd = [sys.executable, tool]
        for k in ("dp_degree", "mp_degree", "pp_degree", "vpp_degree", "sharding_degree", "sharding_stage",
                  "use_recompute", "micro_batch_size", "recompute_granularity"):
            cmd += [f"--{k}", str(cur_cfg.get(k))]
        for k in ("hidden_size", "num_attention_heads", "num_layers", "max_sequence_length", "vocab_size",
                  "intermediate_size", "seq_length", "num_key_value_heads"):
            if tuner_cfg["model_cfg"].get(k) is not None:
                cmd += [f"--{k}", str(tuner_cfg["model_cfg"][k])]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise ValueError(f"memory_estimation_tool failed: {r.stderr}")
        mib = int(round(float(r.stdout.strip().split()[-1]), 2))
        cur_cfg["estimated_memory_usage"] = mib
        return mib > tuner_cfg["max_mem_usage"] * 1024
    budget = tuner_cfg.get("max_mem_usage", tuner_cfg.get("max_mem_usage_gb", HBM_GB * 0.92))
    est = estimate_memory_gb(tuner_cfg["model_cfg"], cur_cfg)
    cur_cfg["estimated_memory_gb"] = round(est, 1)
    if est > budget:
        log_pruned_info(cur_cfg, f"estimated {est:.1f} GB > {budget:.1f} GB", tuner_cfg)
        return True
    return False


@register_prune
def prune_by_invalid_strategy(tuner_cfg, cur_cfg, history_cfgs=()):
    """``invalid_strategy``: list of patterns like "mp4_pp*" or "sharding*_stage3"."""
    inv = tuner_cfg.get("invalid_strategy")
    if not inv:
        return False
    if not isinstance(inv, list):
        raise ValueError("invalid_strategy must be a list")
    return any(_matched(cur_cfg, s) for s in inv)


@register_prune
def prune_by_refined_recompute(tuner_cfg, cur_cfg, history_cfgs=()):
    """Refined recompute (per-op layer counts) only with pp > 1 and full recompute; counts <= layers/pp."""
    rr = tuner_cfg.get("refined_recompute")
    if not rr:
        return False
    vals = [cur_cfg.get(k, 0) for k in rr]
    pp = cur_cfg.get("pp_degree", 1)
    if not cur_cfg.get("use_recompute") or pp == 1 or cur_cfg.get("recompute_granularity") != "full":
        return any(v for v in vals)
    limit = tuner_cfg["model_cfg"]["num_layers"] // pp
    return any(v > limit for v in vals)


# ------------------------------------------------------------------------------------------ history rules
def _history(history_cfgs, pruned_cfgs):
    return list(history_cfgs or []) + list(pruned_cfgs or [])


def _speed_or_memory(tuner_cfg, cur_cfg, attrs, key_fn, history_cfgs, pruned_cfgs, name):
    """Common shape of the history rules: a neighbour with a smaller key that ran makes this one
    redundant (slower); one with a larger key that OOM'd makes this one hopeless."""
    mine = key_fn(cur_cfg)
    if mine is None:
        return False
    for h in same_cfgs_beside(attrs, cur_cfg, _history(history_cfgs, pruned_cfgs)):
        theirs = key_fn(h)
        if theirs is None:
            continue
        if theirs < mine and (h.get("time") or -1) > 0:
            log_pruned_info(cur_cfg, f"{name} {mine} may be slower: {theirs} already ran", tuner_cfg)
            cur_cfg["time"] = h["time"]
            return True
        if theirs > mine and h.get("max_mem_usage") == "OOM":
            log_pruned_info(cur_cfg, f"{name} {mine} may OOM: {theirs} already did", tuner_cfg)
            cur_cfg["max_mem_usage"] = "OOM"
            return True
    return False


@register_prune_history
def prune_by_mp_pp_history(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=()):
    mp, pp, rc = cur_cfg.get("mp_degree"), cur_cfg.get("pp_degree"), cur_cfg.get("use_recompute")
    if mp is None or pp is None or rc is None or rc:
        return False
    for h in same_cfgs_beside(["mp_degree", "pp_degree"], cur_cfg, _history(history_cfgs, pruned_cfgs)):
        if h["mp_degree"] * h["pp_degree"] == mp * pp and h["mp_degree"] > mp and h.get("max_mem_usage") == "OOM":
            log_pruned_info(cur_cfg, f"mp {mp} pp {pp} may OOM: mp {h['mp_degree']} already did", tuner_cfg)
            cur_cfg["max_mem_usage"] = "OOM"
            return True
    return False


@register_prune_history
def prune_by_vpp_history(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=()):
    if cur_cfg.get("vpp_degree") is None:
        return False
    for h in same_cfgs_beside("vpp_degree", cur_cfg, _history(history_cfgs, pruned_cfgs)):
        if h["vpp_degree"] > cur_cfg["vpp_degree"] and h.get("max_mem_usage") == "OOM":
            log_pruned_info(cur_cfg, f"vpp {cur_cfg['vpp_degree']} may OOM", tuner_cfg)
            cur_cfg["max_mem_usage"] = "OOM"
            return True
    return False


@register_prune_history
def prune_by_mbs_history(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=()):
    # a larger micro-batch that ran is faster; a smaller one that OOM'd dooms this one (key = -mbs)
    return _speed_or_memory(tuner_cfg, cur_cfg, ["micro_batch_size", "acc_steps"],
                            lambda c: -c["micro_batch_size"] if c.get("micro_batch_size") else None,
                            history_cfgs, pruned_cfgs, "micro_batch_size")


@register_prune_history
def prune_by_sharding_history(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=()):
    if cur_cfg.get("sharding_degree") is None:
        return False
    return _speed_or_memory(tuner_cfg, cur_cfg, "sharding_stage", lambda c: c.get("sharding_stage"),
                            history_cfgs, pruned_cfgs, "sharding_stage")


@register_prune_history
def prune_by_recompute_history(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=()):
    return _speed_or_memory(tuner_cfg, cur_cfg, ["use_recompute", "recompute_granularity"], _recompute_level,
                            history_cfgs, pruned_cfgs, "recompute level")


@register_prune_history
def prune_by_refined_recompute_history(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=()):
    rr = tuner_cfg.get("refined_recompute")
    if not rr:
        return False
    return _speed_or_memory(tuner_cfg, cur_cfg, list(rr), lambda c: tuple(c.get(k, 0) for k in rr),
                            history_cfgs, pruned_cfgs, "refined recompute")


@register_prune_history
def prune_by_custom_search_dim_history(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=()):
    """Custom dims flagged ``"prune": True`` are treated as memory-for-speed knobs ordered by value."""
    dims = tuner_cfg.get("custom_search_dim") or {}
    for key, spec in dims.items():
        if not spec.get("prune") or key not in cur_cfg:
            continue
        if _speed_or_memory(tuner_cfg, cur_cfg, key, lambda c, k=key: c.get(k), history_cfgs, pruned_cfgs, key):
            return True
    return False


@register_prune_history
def prune_by_sharding_overlap(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=()):
    """dp-estimation: the overlap pair only runs for layouts whose single-dp run produced a metric."""
    if "sharding_overlap" not in cur_cfg:
        return False
    metric = tuner_cfg["metric_cfg"]["name"]
    keys = ("mp_degree", "pp_degree", "vpp_degree", "micro_batch_size", "use_recompute", "recompute_granularity")
    base = [h for h in history_cfgs if "sharding_overlap" not in h and all(h.get(k) == cur_cfg.get(k) for k in keys)]
    return not base or not base[0].get(metric)


@register_prune_history
def prune_by_history_oom(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=()):
    """A config whose analytical estimate is at least that of one which already OOM'd is skipped."""
    est = cur_cfg.get("estimated_memory_gb")
    if est is None:
        return False
    for h in history_cfgs or []:
        if h.get("max_mem_usage") == "OOM" and h.get("estimated_memory_gb", 1e9) <= est:
            return True
    return False
