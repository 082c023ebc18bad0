"""AutoTuner (reference: python/paddle/distributed/auto_tuner/tuner.py:21 — search-algorithm
selection :30, search_once :62, add_cfg :71, resume_form_history :75, get_cfg_from_resume :118)."""
from __future__ import annotations

import os
import shutil

from .recorder import HistoryRecorder
from .search import CustomizeSearch, DpEstimationSearch, GBSSearch, GridSearch
from .utils import cfg_key, default_candidates, gbs_default_candidates


class AutoTuner:
    """Hands out one trial configuration at a time (``search_once``) until the space or ``task_limit`` is
    exhausted; measured trials come back through ``add_cfg`` and feed the history prune rules."""

    def __init__(self, tuner_cfg):
        self.cur_task_id = 1
        self.task_limit = tuner_cfg.get("task_limit", 100)
        algo = tuner_cfg.get("search_algo", {"name": "grid"})
        name = algo.get("name", "grid") if isinstance(algo, dict) else str(algo)
        tuner_cfg["search_algo"] = algo if isinstance(algo, dict) else {"name": name}
        tuner_cfg.setdefault("metric_cfg", {"name": "step_time", "OptimizationDirection": "Minimize"})
        if name == "grid":
            tuner_cfg["candidates"] = default_candidates(tuner_cfg)
            self.algo = GridSearch(tuner_cfg)
        elif name == "dp_estimation":
            tuner_cfg["candidates"] = default_candidates(tuner_cfg)
            self.algo = DpEstimationSearch(tuner_cfg)
        elif name == "gbs":
            tuner_cfg["candidates"] = gbs_default_candidates(tuner_cfg)
            self.algo = GBSSearch(tuner_cfg)
        elif name == "customize":
            self.algo = CustomizeSearch(tuner_cfg)
        else:
            raise NotImplementedError(f"search_algo {name!r}")
        self.history_cfgs = []
        self.resume_cfgs = []
        self.tuner_cfg = tuner_cfg
        self.recorder = HistoryRecorder(tuner_cfg)

    def search_once(self):
        if self.cur_task_id > self.task_limit:
            return None
        cfg = self.algo.search_once(self.history_cfgs)
        if cfg is not None:
            self.cur_task_id += 1
        return cfg

    def add_cfg(self, cfg):
        self.history_cfgs.append(cfg)
        self.recorder.add_cfg(**cfg)

    def get_best(self, buffer=None, max_mem_usage=None):
        metric = self.tuner_cfg["metric_cfg"].get("name", "step_time")
        direction = self.tuner_cfg["metric_cfg"].get("OptimizationDirection", "Minimize")
        best, err = self.recorder.get_best(metric, direction, buffer, max_mem_usage)
        return None if err else best

    def resume_form_history(self, history_csv_path="./history.csv"):
        """Load an earlier run's history (a ``*_copy.csv`` backup is kept); ``get_cfg_from_resume`` then
        returns the stored result of a config instead of re-running it."""
        if not os.path.exists(history_csv_path):
            return []
        root, _ = os.path.splitext(history_csv_path)
        shutil.copyfile(history_csv_path, root + "_copy.csv")
        rows, err = HistoryRecorder(self.tuner_cfg).load_history(history_csv_path)
        metric = self.tuner_cfg["metric_cfg"]["name"]
        for r in rows:
            r["time"] = r.get(metric) if r.get(metric) else -1
        self.resume_cfgs = [] if err else rows
        return self.resume_cfgs

    def get_cfg_from_resume(self, cur_cfg):
        extra = list(self.tuner_cfg.get("refined_recompute") or []) + list(self.tuner_cfg.get("custom_search_dim")
                                                                          or {})
        want = cfg_key(cur_cfg, extra)
        for r in self.resume_cfgs:
            if cfg_key(r, extra) == want:
                return r
        return None
