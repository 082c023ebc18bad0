"""Candidate generation, search-space enumeration and trial-log parsing for the auto tuner
(reference: python/paddle/distributed/auto_tuner/utils.py — divisor :32, dist_degree :56,
default_candidates :162, search_all :308, sort_by_special :511, _param2range :632,
search_by_dp_estimation :665, gen_new_args :982, read_metric_log :1406, read_log :1597,
find_error_from_log :1654, gbs_default_candidates :1704, gbs_search_all :1733,
load_configs_from_csv :1784).

Semantics kept from the reference: a dimension the user leaves unset is pinned to 1, ``"auto"`` opens
it to every divisor, a list / ``{"min", "max"}`` / int restricts it; ``schedule_mode`` "memory"
(default) orders candidates from the most memory-frugal (large mp/pp/sharding, stage 3, small
micro-batch, recompute on) to the least, "performance" the reverse.  MI355X-specific: tensor
parallelism is kept inside one node's xGMI mesh (mp <= gpus_per_node) unless ``enable_mp_prune`` is off.
"""
from __future__ import annotations

import copy
import csv
import itertools
import json
import os
import re

RECOMPUTE_GRANULARITIES = ["full", "full_attn", "core_attn"]
_DIMS = ["mp_degree", "sharding_degree", "pp_degree", "dp_degree", "sharding_stage", "micro_batch_size",
         "vpp_degree", "use_recompute", "recompute_granularity"]
_SHORT = {"dp_degree": "dp", "mp_degree": "mp", "pp_degree": "pp", "vpp_degree": "vpp", "micro_batch_size": "mbs",
          "sharding_degree": "sharding", "sharding_stage": "stage", "use_recompute": "recompute",
          "recompute_granularity": "granularity"}
_GRAN_CODE = {0: "full", 1: "full_attn", 2: "core_attn"}


def divisor(num, reverse=False):
    """Sorted divisors of ``num``."""
    out = sorted({d for i in range(1, int(num ** 0.5) + 1) if num % i == 0 for d in (i, num // i)})
    return out[::-1] if reverse else out


def _memory_first(tuner_cfg):
    return tuner_cfg.get("schedule_mode", "memory") != "performance"


def dist_degree(mode, num_gpus, num_nodes, tuner_cfg=None):
    """Candidate degrees of one dimension before the user's range is applied."""
    tuner_cfg = tuner_cfg or {}
    m = tuner_cfg.get("model_cfg", {})
    mem = _memory_first(tuner_cfg)
    if mode == "dp_degree":
        return divisor(num_gpus, reverse=not mem)
    if mode == "sharding_degree":
        return divisor(num_gpus, reverse=True)
    if mode == "pp_degree":
        if num_nodes > 1 and tuner_cfg.get("enable_pp_prune", True):
            cands = list(range(num_nodes + 1, 0, -1))
        else:
            cands = divisor(num_gpus, reverse=True)
        L = m.get("num_layers")
        return [p for p in cands if not L or L % p == 0]
    if mode == "mp_degree":
        pool = num_gpus // num_nodes if tuner_cfg.get("enable_mp_prune", True) else num_gpus
        cands = divisor(pool, reverse=mem)
        return [d for d in cands if _mp_divides(tuner_cfg, d)]
    if mode == "micro_batch_size":
        return divisor(m["global_batch_size"], reverse=not mem)
    if mode == "vpp_degree":
        return divisor(m["num_layers"], reverse=not mem)
    raise ValueError(f"unknown dimension {mode!r}")


def _mp_divides(tuner_cfg, mp):
    m = tuner_cfg.get("model_cfg", {})
    for key in ("hidden_size", "vocab_size", "num_attention_heads"):
        if m.get(key) and m[key] % mp:
            return False
    kv = m.get("num_key_value_heads")
    if kv and kv % mp and mp % kv:
        return False
    s = m.get("seq_length")
    return not (s and s % mp and tuner_cfg.get("use_sequence_parallel", False))


def param2range(value, max_value, key):
    """User spec of one dimension -> allowed values (None -> [1], "auto" -> 1..max)."""
    if value is None:
        return [1]
    if isinstance(value, str):
        if "auto" in value.lower():
            return list(range(1, max_value + 1))
        raise ValueError(f"{key}: only 'auto' is accepted as a string")
    if isinstance(value, dict):
        lo, hi = value.get("min"), value.get("max")
        if not (lo and hi):
            raise ValueError(f"{key}: a dict range needs both min and max")
        return list(range(lo, hi + 1))
    if isinstance(value, bool):
        raise ValueError(f"{key}: expected int / list / dict / 'auto'")
    if isinstance(value, int):
        return [value]
    if isinstance(value, (list, tuple)):
        return list(value)
    raise ValueError(f"{key}: expected int / list / dict / 'auto', got {type(value).__name__}")


def _nodes(tuner_cfg):
    est = (tuner_cfg.get("search_algo") or {}).get("estimated_num_gpus") \
        if isinstance(tuner_cfg.get("search_algo"), dict) else None
    if est is not None:
        return est, max(1, est // tuner_cfg.get("gpus_per_node", 8))
    return tuner_cfg["num_gpus"], tuner_cfg.get("nodes", 1)


def _bool_dim(value, mem, key):
    if value is None:
        return [None]
    if isinstance(value, str):
        if value.lower() != "auto":
            raise ValueError(f"{key} supports auto/True/False")
        return [True, False] if mem else [False, True]
    if isinstance(value, bool):
        return [value]
    if isinstance(value, list):
        if any(v not in (True, False) for v in value):
            raise ValueError(f"{key} only supports auto/True/False")
        return list(value) or [None]
    raise ValueError(f"{key} supports auto/True/False")


def _granularity_dim(value, mem):
    if value is None:
        return [None]
    vals = value if isinstance(value, list) else [value]
    if len(vals) == 1 and isinstance(vals[0], str) and vals[0].lower() == "auto":
        return list(RECOMPUTE_GRANULARITIES) if mem else RECOMPUTE_GRANULARITIES[::-1]
    out = []
    for v in vals:
        if str(v).lower() not in RECOMPUTE_GRANULARITIES:
            raise ValueError(f"recompute_granularity only supports auto/{'/'.join(RECOMPUTE_GRANULARITIES)}")
        out.append(str(v).lower())
    return out or [None]


def default_candidates(tuner_cfg):
    """Per-dimension candidate lists from the user's tuner config."""
    num_gpus, num_nodes = _nodes(tuner_cfg)
    if num_gpus <= 0:
        raise ValueError("num_gpus must be positive")
    m = tuner_cfg["model_cfg"]
    mem = _memory_first(tuner_cfg)
    cands = {}
    for dim in ("dp_degree", "mp_degree", "pp_degree", "sharding_degree"):
        allowed = param2range(tuner_cfg.get(dim), num_gpus, dim)
        cands[dim] = [d for d in dist_degree(dim, num_gpus, num_nodes, tuner_cfg) if d in allowed]
    allowed = param2range(tuner_cfg.get("vpp_degree"), m["num_layers"], "vpp_degree")
    cands["vpp_degree"] = [d for d in dist_degree("vpp_degree", num_gpus, num_nodes, tuner_cfg) if d in allowed]
    allowed = param2range(tuner_cfg.get("micro_batch_size"), m["global_batch_size"], "micro_batch_size")
    cands["micro_batch_size"] = [d for d in dist_degree("micro_batch_size", num_gpus, num_nodes, tuner_cfg)
                                 if d in allowed]
    allowed = param2range(tuner_cfg.get("sharding_stage"), 3, "sharding_stage")
    stages = [s for s in (3, 2, 1) if s in allowed]
    cands["sharding_stage"] = stages if mem else stages[::-1]
    cands["use_recompute"] = _bool_dim(tuner_cfg.get("use_recompute"), mem, "use_recompute")
    cands["recompute_granularity"] = _granularity_dim(tuner_cfg.get("recompute_granularity"), mem)
    if tuner_cfg.get("custom_search_dim"):
        cands["custom_search_dim"] = [v["value"] for v in tuner_cfg["custom_search_dim"].values()]
    return cands


def _refined_recompute_grid(n_ops, max_value, mem):
    """Per-op refined-recompute layer counts: op i may be > 0 only once ops < i are at max_value."""
    grid = []
    for i in range(n_ops):
        for v in range(0, max_value + 1):
            cfg = [max_value] * i + [v] + [0] * (n_ops - i - 1)
            if cfg not in grid:
                grid.append(cfg)
    return grid if mem else sorted(grid, reverse=True)


def _valid_degrees(cands, num_gpus):
    out = []
    for mp in cands["mp_degree"]:
        if num_gpus % mp:
            continue
        for sh in cands["sharding_degree"]:
            if (num_gpus // mp) % sh:
                continue
            for pp in cands["pp_degree"]:
                if (num_gpus // mp // sh) % pp:
                    continue
                dp = num_gpus // mp // sh // pp
                if dp in cands["dp_degree"]:
                    out.append([mp, sh, pp, dp])
    return out


def search_all(tuner_cfg):
    """Every valid configuration (degrees multiply to the GPU count, batch / layer divisibility),
    after the registered prune rules, in the candidate order (optionally re-ranked by schedule_prior)."""
    from .prune import _PRUNE_FUNC

    cands = tuner_cfg["candidates"]
    num_gpus, _ = _nodes(tuner_cfg)
    m = tuner_cfg["model_cfg"]
    mem = _memory_first(tuner_cfg)
    others = list(itertools.product(cands["sharding_stage"], cands["micro_batch_size"], cands["vpp_degree"],
                                    cands["use_recompute"], cands["recompute_granularity"]))
    custom = tuner_cfg.get("custom_search_dim")
    if custom:
        others = [list(o) + list(c) for o in others for c in itertools.product(*cands["custom_search_dim"])]
    rr = tuner_cfg.get("refined_recompute")
    keys = list(_DIMS) + (list(custom) if custom else []) + (list(rr) if rr else [])
    rows = []
    for deg in _valid_degrees(cands, num_gpus):
        mp, sh, pp, dp = deg
        for o in others:
            stage, mbs, vpp, rc, gran = list(o)[:5]
            if m["global_batch_size"] % (mbs * sh * dp) or m["num_layers"] % (pp * vpp):
                continue
            if not rr:
                rows.append(deg + list(o))
                continue
            if pp == 1 or not rc or gran != "full":
                row = deg + list(o) + [0] * len(rr)
                if row not in rows:
                    rows.append(row)
                continue
            for r in _refined_recompute_grid(len(rr), m["num_layers"] // pp, mem):
                row = deg + list(o) + r
                if row not in rows:
                    rows.append(row)
    cfgs = [dict(zip(keys, r)) for r in rows]
    tuner_cfg["num_gpus"] = num_gpus
    kept = []
    for c in cfgs:
        if not any(f(tuner_cfg, c, kept) for f in _PRUNE_FUNC):
            kept.append(c)
    tuner_cfg["search_space_size"] = (len(cfgs), len(kept))
    if tuner_cfg.get("schedule_prior"):
        kept = sort_by_special(kept, tuner_cfg)
    return kept


def _matched(cfg, strategy):
    """``strategy`` like "mp4_pp2" / "sharding*_stage3": every named dim matches (``*`` = enabled)."""
    rev = {v: k for k, v in _SHORT.items()}
    for part in strategy.split("_"):
        key = next((s for s in sorted(rev, key=len, reverse=True) if part.startswith(s)), None)
        if key is None:
            return False
        val, dim = part[len(key):], rev[key]
        if key in ("dp", "mp", "pp", "vpp", "sharding"):
            ok = cfg.get(dim, 1) != 1 if val == "*" else cfg.get(dim) == int(val)
        elif key == "recompute":
            ok = bool(cfg.get(dim)) if val == "*" else bool(cfg.get(dim)) == bool(int(val))
        elif key == "stage":
            ok = cfg.get("sharding_degree", 1) != 1 if val == "*" else cfg.get(dim) == int(val)
        elif key == "mbs":
            ok = val == "*" or cfg.get(dim) == int(val)
        else:  # granularity
            ok = bool(cfg.get("use_recompute")) if val == "*" else cfg.get(dim) == _GRAN_CODE[int(val)]
        if not ok:
            return False
    return True


def sort_by_special(cfgs, tuner_cfg):
    """Move configs matching ``tuner_cfg['schedule_prior']`` strategies to the front (first listed first)."""
    front, rest = [], list(cfgs)
    for strategy in tuner_cfg["schedule_prior"]:
        hit = [c for c in rest if _matched(c, strategy)]
        front += hit
        rest = [c for c in rest if not _matched(c, strategy)]
    return front + rest


def memory_sort(cfg):
    return (-cfg["mp_degree"], -cfg["pp_degree"], -cfg["vpp_degree"], -cfg["sharding_degree"],
            -cfg["sharding_stage"], cfg["micro_batch_size"], -int(bool(cfg["use_recompute"])))


def performance_sort(cfg):
    return -cfg["micro_batch_size"]


def _nodes_for(cards, tuner_cfg):
    per = tuner_cfg.get("gpus_per_node", 8)
    if cards <= per:
        return 1
    if cards % per == 0:
        return cards // per
    for i in range(2, tuner_cfg.get("nodes", 1) + 1):
        if cards % i == 0 and cards // i <= per:
            return i
    raise ValueError(f"{cards} GPUs cannot be spread evenly over the nodes")


def search_by_dp_estimation(tuner_cfg):
    """Single-dp estimation: run each mp x pp layout with dp = sharding = 1 on mp*pp GPUs and a
    proportionally smaller global batch; the multi-dp throughput is then extrapolated.  With
    ``sharding_overlap`` the sharded layout is also queued with and without comm overlap."""
    tasks = []
    for c in search_all(tuner_cfg):
        t = dict(c)
        t["estimated_dp_degree"] = int(c["dp_degree"] * c["sharding_degree"])
        t.update(dp_degree=1, sharding_degree=1, sharding_stage=1, num_gpus=c["mp_degree"] * c["pp_degree"])
        t["nodes"] = _nodes_for(t["num_gpus"], tuner_cfg)
        t["global_batch_size"] = tuner_cfg["model_cfg"]["global_batch_size"] // t["estimated_dp_degree"]
        if t not in tasks and t["nodes"] <= tuner_cfg.get("nodes", 1):
            tasks.append(t)
    extra = []
    if tuner_cfg["search_algo"].get("sharding_overlap"):
        total = tuner_cfg.get("nodes", 1) * tuner_cfg.get("gpus_per_node", 8)
        for t in tasks:
            sh = total // t["num_gpus"]
            if sh <= 1:
                continue
            n = dict(t, sharding_degree=sh, sharding_stage=1, estimated_dp_degree=None)
            n["num_gpus"] = n["mp_degree"] * n["pp_degree"] * sh
            n["nodes"] = _nodes_for(n["num_gpus"], tuner_cfg)
            n["global_batch_size"] = t["global_batch_size"] * sh
            extra += [dict(n, sharding_overlap=False), dict(n, sharding_overlap=True)]
    return tasks + extra


def add_overlap_performance(cur_cfg, tuner_cfg, history_cfgs):
    """dp-estimation: scale the single-dp metric by the measured overlap speed-up of the sharded pair."""
    metric = tuner_cfg["metric_cfg"]["name"]
    if not cur_cfg.get(metric):
        return
    keys = ("mp_degree", "pp_degree", "vpp_degree", "micro_batch_size", "use_recompute", "recompute_granularity")
    same = [h for h in history_cfgs if all(h.get(k) == cur_cfg.get(k) for k in keys)]
    plain = next((h for h in same if h.get("sharding_overlap") is False and h.get(metric)), None)
    over = next((h for h in same if h.get("sharding_overlap") is True and h.get(metric)), None)
    if plain and over:
        ratio = over[metric] / plain[metric]
        if tuner_cfg["metric_cfg"].get("OptimizationDirection", "Maximize") == "Minimize":
            ratio = 1.0 / ratio
        cur_cfg[f"{metric}_with_overlap"] = round(cur_cfg[metric] * ratio, 5)


def three_mul_combinations(target):
    """(i, j, k) with i <= j and i * j * k == target."""
    return [(i, j, target // i // j) for i in range(1, target // 3 + 1) if target % i == 0
            for j in range(i, target // 2 + 1) if (target // i) % j == 0]


def gbs_dp_mp_pp_candidates(tuner_cfg, num_gpus, num_nodes):
    """A balanced (dp, mp, pp) split of the GPUs (cube-root first factor)."""
    for i in range(round(num_gpus ** (1 / 3)), 0, -1):
        if num_gpus % i == 0:
            rest = num_gpus // i
            j = round(rest ** 0.5)
            while rest % j:
                j -= 1
            return i, j, rest // j
    raise ValueError("cannot split the GPUs evenly")


def gbs_default_candidates(tuner_cfg):
    """Global-batch search: a fixed balanced layout, micro-batch 1..512, gbs = pp * sharding * mbs (one
    micro-batch per stage in flight per data-parallel rank: the smallest batch 1F1B keeps busy)."""
    num_gpus, num_nodes = tuner_cfg["num_gpus"], tuner_cfg.get("nodes", 1)
    dp, mp, pp = gbs_dp_mp_pp_candidates(tuner_cfg, num_gpus, num_nodes)
    mbs = [2 ** i for i in range(10)]
    return {"dp_degree": [1], "mp_degree": [mp], "pp_degree": [pp], "sharding_degree": [dp],
            "sharding_stage": [1], "use_recompute": [False], "recompute_granularity": [None],
            "micro_batch_size": mbs, "global_batch_size": [pp * dp * m for m in mbs]}   # sharding = dp here


def gbs_search_all(tuner_cfg):
    c = tuner_cfg["candidates"]
    keys = ["dp_degree", "mp_degree", "pp_degree", "micro_batch_size", "sharding_degree", "sharding_stage",
            "use_recompute", "recompute_granularity"]
    out = []
    for vals in itertools.product(*(c[k] for k in keys)):
        cfg = dict(zip(keys, vals))
        cfg["global_batch_size"] = cfg["pp_degree"] * cfg["dp_degree"] * cfg["sharding_degree"] * \
            cfg["micro_batch_size"]
        out.append(cfg)
    return out


def load_configs_from_csv(path):
    """Customize search: configs from a CSV with the dimension columns."""
    out = []
    with open(path) as f:
        for row in csv.DictReader(f):
            cfg = {}
            for k in ("dp_degree", "mp_degree", "pp_degree", "vpp_degree", "micro_batch_size", "sharding_degree",
                      "sharding_stage"):
                try:
                    cfg[k] = int(row.get(k, ""))
                except ValueError:
                    raise ValueError(f"{k} must be an integer, got {row.get(k)!r}") from None
            rc = row.get("use_recompute", "").lower()
            if rc not in ("true", "false"):
                raise ValueError(f"use_recompute must be true or false, got {rc!r}")
            cfg["use_recompute"] = rc == "true"
            g = row.get("recompute_granularity", "")
            if g and g.lower() not in RECOMPUTE_GRANULARITIES:
                raise ValueError(f"recompute_granularity must be one of {RECOMPUTE_GRANULARITIES}")
            cfg["recompute_granularity"] = g.lower() or None
            out.append(cfg)
    return out


# ------------------------------------------------------------------------------------------ trial I/O
def gen_new_args(raw_args, cfg, tuner_cfg, run_best=False):
    """Script argv for one trial: ``run_cmd`` maps a config key to ``[flag, default]`` (the reference's
    json layout; ``"./config.json"``-style flags are not supported) and ``args_template`` maps a key to a
    flag; a flag already in ``raw_args`` has its value replaced, otherwise the pair is appended."""
    out = list(raw_args)
    mapping = {}
    for key, spec in (tuner_cfg.get("run_cmd") or {}).items():
        if isinstance(spec, (list, tuple)) and spec:
            mapping[key] = spec[0]
    mapping.update(tuner_cfg.get("args_template", {}))
    if run_best and tuner_cfg.get("run_best_args"):
        mapping.update(tuner_cfg["run_best_args"])
    for key, flag in mapping.items():
        if key not in cfg or cfg[key] is None:
            continue
        val = cfg[key]
        sval = str(int(val)) if isinstance(val, bool) else str(val)
        if flag in out:
            i = out.index(flag)
            if i + 1 < len(out):
                out[i + 1] = sval
            else:
                out.append(sval)
        else:
            out += [flag, sval]
    return out


_NUM = r"([-+]?\d+(?:\.\d*)?(?:[eE][-+]?\d+)?)"
_OOM = re.compile(r"out of memory|OutOfMemoryError|hipErrorOutOfMemory", re.IGNORECASE)


def read_metric_log(path, file="workerlog.0", target_metric="step/s"):
    """-> (metric, err_code): the mean of the last 10 readings (of readings 10+ when fewer than 20, the last
    one when fewer than 10); err bit 0 = no metric, bit 1 = out of memory.  A reading is
    ``<metric>: v`` / ``<metric> = v`` / ``"<metric>": v`` / ``v <metric>``."""
    target = os.path.join(path, file) if file else path
    if not os.path.exists(target):
        return 0.0, 1
    name = re.escape(target_metric)
    pats = [re.compile(rf'"?{name}"?\s*[:=]?\s*{_NUM}'), re.compile(rf"{_NUM}\s*{name}")]
    vals, oom = [], False
    with open(target, errors="ignore") as f:
        for line in f:
            if _OOM.search(line):
                oom = True
            for p in pats:
                hit = p.findall(line)
                if hit:
                    vals.append(float(hit[-1]))
                    break
    err = (2 if oom else 0) | (0 if vals else 1)
    if oom or not vals:
        return 0.0, err
    if len(vals) < 10:
        v = vals[-1]
    elif len(vals) < 20:
        v = sum(vals[9:]) / len(vals[9:])
    else:
        v = sum(vals[-10:]) / 10
    return round(v, 5), err


def read_memory_log(path, file="0.gpu.log"):
    """-> (peak MiB, err).  Reads a per-GPU CSV (``index, utilization, memory_total, memory_used, ...``
    rows; the launcher's monitor writes one) or, failing that, the largest ``peak_mem_gb`` /
    ``max_memory_allocated`` reading in the worker logs."""
    p = os.path.join(path, file)
    if os.path.exists(p):
        used = []
        with open(p) as f:
            rows = list(csv.reader(f))
        header = next((i for i, r in enumerate(rows) if "memory_used" in [c.strip() for c in r]), None)
        if header is not None:
            col = [c.strip() for c in rows[header]].index("memory_used")
            for r in rows[header + 1:]:
                try:
                    used.append(float(r[col]))
                except (ValueError, IndexError):
                    pass
        if used:
            return max(used), False
    best = None
    if os.path.isdir(path):
        for fn in sorted(os.listdir(path)):
            if not fn.startswith("workerlog"):
                continue
            with open(os.path.join(path, fn), errors="ignore") as f:
                txt = f.read()
            for m in re.finditer(rf'"?peak_mem_gb"?\s*[:=]\s*{_NUM}', txt):
                best = max(best or 0.0, float(m.group(1)) * 1024)
            for m in re.finditer(rf"max_memory_allocated\s*[:=]\s*{_NUM}", txt):
                best = max(best or 0.0, float(m.group(1)) / 2**20)
    return (best, False) if best is not None else (0.0, True)


def read_completed(path):
    """True when a worker log says the training finished."""
    if not os.path.isdir(path):
        return False
    for fn in os.listdir(path):
        if fn.startswith("workerlog"):
            with open(os.path.join(path, fn), errors="ignore") as f:
                if re.search(r"training completed", f.read(), re.IGNORECASE):
                    return True
    return False


def read_log(path, metric_file="workerlog.0", target_metric="step/s", memory_file="0.gpu.log"):
    """-> (metric, peak memory MiB, err_code): bit 0 no metric, bit 1 OOM on any rank, bit 2 no memory log."""
    err = 0
    if os.path.isdir(path):
        for fn in os.listdir(path):
            if fn.startswith("workerlog"):
                err |= read_metric_log(path, fn, target_metric)[1] & 2
    metric, e = read_metric_log(path, metric_file, target_metric)
    err |= e
    mem, merr = read_memory_log(path, memory_file)
    err |= int(bool(merr)) << 2
    return metric, mem, err


def get_error_info(filename):
    infos = set()
    with open(filename, errors="ignore") as f:
        for line in f.readlines()[-100:]:
            if re.search(r"error", line, re.IGNORECASE):
                infos.add("Out of memory" if _OOM.search(line) else line.strip())
    return sorted(infos)


def find_error_from_log(path):
    """Comma-joined distinct error lines from the last 100 lines of every worker log."""
    infos = set()
    if os.path.isdir(path):
        for fn in sorted(os.listdir(path)):
            if fn.startswith("workerlog"):
                infos.update(get_error_info(os.path.join(path, fn)))
    return ",".join(sorted(infos))


def cfg_key(cfg, extra=()):
    """Stable identity of a configuration (used for resume and history de-duplication)."""
    keys = list(_DIMS) + ["num_gpus", "nodes", "global_batch_size", "sharding_overlap", "acc_steps"] + list(extra)
    return json.dumps({k: cfg.get(k) for k in keys if cfg.get(k) not in (None, False, "")}, sort_keys=True,
                      default=str)


def copy_cfg(cfg):
    return copy.deepcopy(cfg)
