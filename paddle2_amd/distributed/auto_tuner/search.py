"""Search algorithms of the auto tuner (reference: python/paddle/distributed/auto_tuner/search.py —
SearchAlgo :31, GridSearch :48, DpEstimationSearch :96, GBSSearch :123, CustomizeSearch :144).

GridSearch enumerates the pruned space (utils.search_all) and, unlike the reference's plain candidate
order, ranks it by the analytical MI355X step-time estimate (``cost_model.estimate_step_time``) when
``tuner_cfg['sort_by_estimate']`` is on (default), so the most promising trials run first under a task
limit.  Every algorithm re-checks each candidate against all rules — including the history rules — just
before handing it out, so trials already made redundant by measured runs are skipped.
"""
from __future__ import annotations

import os
from abc import ABC, abstractmethod

from .cost_model import estimate_step_time
from .prune import _PRUNE_FUNC, _PRUNE_HISTORY_FUNC
from .utils import gbs_search_all, load_configs_from_csv, search_all, search_by_dp_estimation


class SearchAlgo(ABC):
    def __init__(self, tuner_cfg):
        self.tuner_cfg = tuner_cfg
        self.pruned = []
        self.idx = 0
        self.all_tasks = []

    @abstractmethod
    def search_once(self, history_cfgs):
        ...

    def prune(self, tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs=None):
        if pruned_cfgs is None:
            pruned_cfgs = self.pruned
        for f in _PRUNE_FUNC:
            if f(tuner_cfg, cur_cfg, history_cfgs):
                return True
        for f in _PRUNE_HISTORY_FUNC:
            if f(tuner_cfg, cur_cfg, history_cfgs, pruned_cfgs):
                return True
        return False

    def _next_unpruned(self, history_cfgs, before=None):
        while self.idx < len(self.all_tasks):
            c = self.all_tasks[self.idx]
            self.idx += 1
            if before is not None:
                before(c)
            if self.prune(self.tuner_cfg, c, history_cfgs):
                self.pruned.append(c)
                continue
            return c
        return None


class GridSearch(SearchAlgo):
    """The pruned search space, best analytical estimate first."""

    def __init__(self, tuner_cfg):
        super().__init__(tuner_cfg)
        tasks = search_all(tuner_cfg)
        gbs = tuner_cfg["model_cfg"]["global_batch_size"]
        for c in tasks:
            c["estimated_step_time_s"] = round(estimate_step_time(tuner_cfg["model_cfg"], c, gbs), 4)
        if tuner_cfg.get("sort_by_estimate", True) and not tuner_cfg.get("schedule_prior"):
            tasks.sort(key=lambda c: c["estimated_step_time_s"])
        self.all_tasks = tasks[: tuner_cfg.get("max_search_time_trials", len(tasks))]

    def search_once(self, history_cfgs):
        return self._next_unpruned(history_cfgs)


class DpEstimationSearch(SearchAlgo):
    """Run each layout at dp = 1 on mp*pp GPUs and extrapolate (utils.search_by_dp_estimation)."""

    def __init__(self, tuner_cfg):
        super().__init__(tuner_cfg)
        if tuner_cfg["candidates"]["dp_degree"] != [1]:
            tuner_cfg["candidates"]["dp_degree"] = [1]
        self.all_tasks = search_by_dp_estimation(tuner_cfg)
        if not self.all_tasks:
            raise ValueError("no layout is feasible for single-dp estimation")

    def search_once(self, history_cfgs):
        return self._next_unpruned(history_cfgs)


class GBSSearch(SearchAlgo):
    """Global-batch search on a fixed balanced layout (utils.gbs_search_all)."""

    def __init__(self, tuner_cfg):
        super().__init__(tuner_cfg)
        self.all_tasks = gbs_search_all(tuner_cfg)

    def search_once(self, history_cfgs):
        def set_gbs(c):
            self.tuner_cfg["model_cfg"]["global_batch_size"] = c["global_batch_size"]

        return self._next_unpruned(history_cfgs, before=set_gbs)


class CustomizeSearch(SearchAlgo):
    """Exactly the configs of ``configs_csv`` (or the inline ``configs`` list), in order, unpruned."""

    def __init__(self, tuner_cfg):
        super().__init__(tuner_cfg)
        path = tuner_cfg.get("configs_csv")
        if path:
            if not os.path.exists(path):
                raise ValueError(f"configs_csv {path} does not exist")
            self.all_tasks = load_configs_from_csv(path)
        else:
            self.all_tasks = [dict(c) for c in tuner_cfg.get("configs", [])]
        if not self.all_tasks:
            raise ValueError("customize search needs configs_csv or configs")

    def search_once(self, history_cfgs):
        if self.idx < len(self.all_tasks):
            self.idx += 1
            return self.all_tasks[self.idx - 1]
        return None
