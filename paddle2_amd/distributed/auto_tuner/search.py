"""Search algorithms (reference: auto_tuner/search.py)."""
from __future__ import annotations

import itertools
from abc import ABC, abstractmethod

from .cost_model import estimate_step_time
from .prune import _PRUNE_FUNC


def _cands(tuner_cfg, key, n):
    v = tuner_cfg.get(key, "auto")
    if v == "auto" or v is None:
        return [d for d in range(1, n + 1) if n % d == 0]
    return list(v) if isinstance(v, (list, tuple)) else [v]


def search_all(tuner_cfg):
    n = tuner_cfg["num_gpus"]
    gbs = tuner_cfg["model_cfg"]["global_batch_size"]
    dims = {
        "dp_degree": _cands(tuner_cfg, "dp_degree", n),
        "mp_degree": _cands(tuner_cfg, "mp_degree", n),
        "pp_degree": _cands(tuner_cfg, "pp_degree", n),
        "sharding_degree": _cands(tuner_cfg, "sharding_degree", n),
        "sharding_stage": tuner_cfg.get("sharding_stage", [1, 2, 3]) if tuner_cfg.get("sharding_stage") != "auto"
        else [1, 2, 3],
        "micro_batch_size": tuner_cfg.get("micro_batch_size", "auto") if tuner_cfg.get("micro_batch_size", "auto")
        != "auto" else [d for d in (1, 2, 4, 8, 16) if gbs % d == 0],
        "use_recompute": tuner_cfg.get("use_recompute", [False, True]) if tuner_cfg.get("use_recompute", "auto")
        != "auto" else [False, True],
    }
    dims = {k: (v if isinstance(v, (list, tuple)) else [v]) for k, v in dims.items()}
    keys = list(dims)
    return [dict(zip(keys, vals)) for vals in itertools.product(*(dims[k] for k in keys))]


class SearchAlgo(ABC):
    def __init__(self, tuner_cfg):
        self.tuner_cfg = tuner_cfg
        self.pruned = []

    @abstractmethod
    def search_once(self, history_cfgs):
        ...

    def prune(self, tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=None):
        return any(f(tuner_cfg, cur_cfg, history_cfgs) for f in _PRUNE_FUNC)


class GridSearch(SearchAlgo):
    """All feasible configs, best analytical estimate first."""

    def __init__(self, tuner_cfg):
        super().__init__(tuner_cfg)
        gbs = tuner_cfg["model_cfg"]["global_batch_size"]
        cands = []
        for c in search_all(tuner_cfg):
            if self.prune(tuner_cfg, c, []):
                self.pruned.append(c)
                continue
            c["estimated_step_time_s"] = round(estimate_step_time(tuner_cfg["model_cfg"], c, gbs), 4)
            cands.append(c)
        cands.sort(key=lambda c: c["estimated_step_time_s"])
        self.all_tasks = cands[: tuner_cfg.get("max_search_time_trials", len(cands))]
        self.idx = 0

    def search_once(self, history_cfgs):
        while self.idx < len(self.all_tasks):
            c = self.all_tasks[self.idx]
            self.idx += 1
            if not self.prune(self.tuner_cfg, c, history_cfgs):
                return c
        return None


class CustomizeSearch(SearchAlgo):
    """Only the configurations listed in ``tuner_cfg['configs']``."""

    def __init__(self, tuner_cfg):
        super().__init__(tuner_cfg)
        self.all_tasks = list(tuner_cfg.get("configs", []))
        self.idx = 0

    def search_once(self, history_cfgs):
        if self.idx < len(self.all_tasks):
            self.idx += 1
            return self.all_tasks[self.idx - 1]
        return None
