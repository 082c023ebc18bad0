"""AutoTuner (reference: auto_tuner/tuner.py:21)."""
from __future__ import annotations

from .recorder import HistoryRecorder
from .search import CustomizeSearch, GridSearch


class AutoTuner:
    def __init__(self, tuner_cfg):
        self.cur_task_id = 1
        self.task_limit = tuner_cfg.get("task_limit", 100)
        algo = tuner_cfg.get("search_algo", {"name": "grid"})
        name = algo.get("name", "grid") if isinstance(algo, dict) else str(algo)
        self.algo = CustomizeSearch(tuner_cfg) if name == "customize" else GridSearch(tuner_cfg)
        self.history_cfgs = []
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

    def get_best(self):
        metric = self.tuner_cfg.get("metric_cfg", {}).get("name", "step_time")
        direction = self.tuner_cfg.get("metric_cfg", {}).get("OptimizationDirection", "Minimize")
        return self.recorder.get_best(metric, direction)[0]

    def resume_form_history(self, history_csv_path="./history.csv"):
        hist, err = self.recorder.load_history(history_csv_path)
        if not err:
            self.history_cfgs = list(hist)
        return self.history_cfgs
