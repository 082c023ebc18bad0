"""Trial history of the auto tuner (reference: python/paddle/distributed/auto_tuner/recorder.py
HistoryRecorder — sort_metric :38, get_best :58 with the memory ``buffer`` rule, store_history :123 with
the dp-estimation "enhanced" report, load_history :151).

Every record is a config plus ``job_id``, the metric, ``time`` (the metric, or -1 when the trial produced
none), ``max_mem_usage`` (peak MiB, or "OOM") and ``error_info``.  The CSV keeps ``job_id`` first and
drops the internal ``time`` / ``has_error`` columns, like the reference.
"""
from __future__ import annotations

import csv
import os


def _conv(v):
    if v is None or v == "":
        return None
    if v in ("True", "False"):
        return v == "True"
    for t in (int, float):
        try:
            return t(v)
        except (TypeError, ValueError):
            pass
    return v


class HistoryRecorder:
    def __init__(self, tuner_cfg=None):
        self.tuner_cfg = tuner_cfg or {}
        self.search_algo = (self.tuner_cfg.get("search_algo") or {}).get("name", "grid") \
            if isinstance(self.tuner_cfg.get("search_algo"), dict) else "grid"
        self.history = []
        self.store_path = None
        metric = self.tuner_cfg.get("metric_cfg", {}).get("name")
        self.additional_metric_key = f"{metric}_with_overlap" if metric and self.search_algo == "dp_estimation" \
            else None

    def add_cfg(self, **kwargs):
        rec = dict(kwargs)
        rec.setdefault("job_id", len(self.history) + 1)
        self.history.append(rec)

    def sort_metric(self, direction, metric_name):
        maximize = direction == "Maximize"

        def key(h):
            v = h.get(metric_name)
            if v is None or h.get("has_error") or h.get("max_mem_usage") == "OOM":
                return float("-inf") if maximize else float("inf")
            return v

        self.history.sort(key=key, reverse=maximize)

    def get_best(self, metric, direction, buffer=None, max_mem_usage=None):
        """-> (best record, err).  With ``buffer`` (MiB), among the measured records prefer the first one (in
        metric order) whose peak memory leaves ``buffer`` of headroom under ``max_mem_usage``, else the
        leanest one measured."""
        self.sort_metric(direction, metric)
        if not self.history:
            return None, True
        best = self.history[0]
        if isinstance(best.get("max_mem_usage"), str) or best.get("time", best.get(metric)) in (None, -1) \
                or best.get(metric) is None:
            return best, True
        if buffer is None:
            return best, False
        if buffer < 0:
            raise ValueError("buffer must be >= 0")
        if not max_mem_usage or max_mem_usage <= 0:
            raise ValueError("max_mem_usage must be > 0 when a buffer is given")
        measured = [h for h in self.history if isinstance(h.get("max_mem_usage"), (int, float))
                    and h.get("max_mem_usage") and h.get(metric) is not None and h.get("time", 0) != -1]
        for h in measured:
            if h["max_mem_usage"] < max_mem_usage - buffer:
                return h, False
        return (min(measured, key=lambda h: h["max_mem_usage"]) if measured else best), False

    def _write(self, rows, path):
        if not rows:
            return
        keys = []
        for h in rows:
            for k in h:
                if k not in keys and k not in ("time", "has_error"):
                    keys.append(k)
        if "job_id" in keys:
            keys.remove("job_id")
            keys.insert(0, "job_id")
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys, extrasaction="ignore")
            w.writeheader()
            for h in rows:
                w.writerow({k: h.get(k) for k in keys})

    def store_history(self, path="./history.csv"):
        if self.search_algo == "dp_estimation" and self.additional_metric_key:
            rows = [h for h in self.history if h.get("sharding_overlap") is None and not h.get("error_info")]
            rows.sort(key=lambda h: h.get(self.additional_metric_key) or float("-inf"), reverse=True)
            self._write(rows, path.rsplit(".csv", 1)[0] + "_enhanced.csv")
        self.store_path = path
        self._write(self.history, path)

    def load_history(self, path="./history.csv"):
        if self.store_path is None:
            self.store_path = path
        if not os.path.exists(self.store_path):
            return [], True
        with open(self.store_path) as f:
            self.history = [{k: _conv(v) for k, v in r.items()} for r in csv.DictReader(f)]
        return self.history, False

    def clean_history(self):
        self.history = []
