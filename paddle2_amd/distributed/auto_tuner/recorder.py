"""Trial history (reference: auto_tuner/recorder.py HistoryRecorder)."""
from __future__ import annotations

import csv
import os


class HistoryRecorder:
    def __init__(self, tuner_cfg=None):
        self.tuner_cfg = tuner_cfg or {}
        self.history = []

    def add_cfg(self, **kwargs):
        self.history.append(dict(kwargs))

    def sort_metric(self, direction, metric_name):
        ok = [h for h in self.history if h.get(metric_name) is not None and not h.get("has_error")]
        bad = [h for h in self.history if h not in ok]
        ok.sort(key=lambda h: h[metric_name], reverse=(direction == "Maximize"))
        self.history = ok + bad

    def get_best(self, metric, direction, buffer=None, max_mem_usage=None):
        self.sort_metric(direction, metric)
        for h in self.history:
            if h.get(metric) is not None and not h.get("has_error"):
                return h, False
        return None, True

    def store_history(self, path="./history.csv"):
        if not self.history:
            return
        keys = sorted({k for h in self.history for k in h})
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys)
            w.writeheader()
            for h in self.history:
                w.writerow(h)

    def load_history(self, path="./history.csv"):
        if not os.path.exists(path):
            return [], True
        with open(path) as f:
            rows = list(csv.DictReader(f))

        def conv(v):
            for t in (int, float):
                try:
                    return t(v)
                except (TypeError, ValueError):
                    pass
            return {"True": True, "False": False, "": None}.get(v, v)

        self.history = [{k: conv(v) for k, v in r.items()} for r in rows]
        return self.history, False

    def clean_history(self):
        self.history = []
