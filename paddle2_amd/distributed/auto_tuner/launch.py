"""Trial runner behind ``launch --auto_tuner_json`` (reference: distributed/launch/main.py auto-tuner
branch + auto_tuner/utils.py gen_new_args / read_metric_log).

Each candidate config is exposed to the training script as environment variables
(PADDLE_AUTO_TUNER_DP/MP/PP/SHARDING/SHARDING_STAGE/MICRO_BATCH/RECOMPUTE) and as
``--key value`` arguments when ``tuner_cfg['args_template']`` maps config keys to flags; the
trial runs as a normal launch, and the metric is parsed from rank 0's log as the last
``<metric_name>: <number>`` (or ``"metric_name": number`` JSON) occurrence.
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
import time

from .tuner import AutoTuner

_ENV = {"dp_degree": "PADDLE_AUTO_TUNER_DP", "mp_degree": "PADDLE_AUTO_TUNER_MP", "pp_degree": "PADDLE_AUTO_TUNER_PP",
        "sharding_degree": "PADDLE_AUTO_TUNER_SHARDING", "sharding_stage": "PADDLE_AUTO_TUNER_SHARDING_STAGE",
        "micro_batch_size": "PADDLE_AUTO_TUNER_MICRO_BATCH", "use_recompute": "PADDLE_AUTO_TUNER_RECOMPUTE"}


def gen_new_args(raw_args, cfg, tuner_cfg):
    out = list(raw_args)
    for key, flag in tuner_cfg.get("args_template", {}).items():
        if key in cfg:
            out += [flag, str(cfg[key])]
    return out


def read_metric_log(path, metric):
    if not os.path.exists(path):
        return None, "no_log"
    txt = open(path, errors="ignore").read()
    if "out of memory" in txt.lower() or "OutOfMemoryError" in txt:
        return None, "OOM"
    pats = [rf'"{re.escape(metric)}"\s*:\s*([-+0-9.eE]+)', rf"{re.escape(metric)}\s*[:=]\s*([-+0-9.eE]+)"]
    last = None
    for pat in pats:
        for m in re.finditer(pat, txt):
            last = float(m.group(1))
    return last, None if last is not None else "no_metric"


def run(tuner_cfg, launch_args, script, script_args, log_root="./auto_tuner_logs", runner=None):
    """-> (best cfg, tuner).  ``runner(cfg, env, argv, log_dir) -> returncode`` defaults to a
    subprocess launch (tests pass a fake)."""
    tuner = AutoTuner(tuner_cfg)
    metric = tuner_cfg.get("metric_cfg", {}).get("name", "step_time")
    while True:
        cfg = tuner.search_once()
        if cfg is None:
            break
        tid = tuner.cur_task_id - 1
        log_dir = os.path.join(log_root, f"trial_{tid}")
        env = dict(os.environ)
        env.update({v: str(int(cfg[k]) if isinstance(cfg[k], bool) else cfg[k]) for k, v in _ENV.items() if k in cfg})
        argv = [sys.executable, "-m", "paddle2_amd.distributed.launch", *launch_args, "--log_dir", log_dir, script,
                *gen_new_args(script_args, cfg, tuner_cfg)]
        t0 = time.time()
        if runner is None:
            rc = subprocess.call(argv, env=env, timeout=tuner_cfg.get("max_time_per_task", 3600))
        else:
            rc = runner(cfg, env, argv, log_dir)
        val, err = read_metric_log(os.path.join(log_dir, "workerlog.0"), metric)
        rec = dict(cfg, **{metric: val, "has_error": err if rc == 0 else (err or f"exit_{rc}"), "task_id": tid,
                           "wall_s": round(time.time() - t0, 1)})
        tuner.add_cfg(rec)
        tuner.recorder.store_history(os.path.join(log_root, "history.csv"))
    best = tuner.get_best()
    if best is not None:
        with open(os.path.join(log_root, "best_cfg.json"), "w") as f:
            json.dump(best, f, indent=1)
    return best, tuner
