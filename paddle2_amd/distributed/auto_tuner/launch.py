"""Trial runner behind ``launch --auto_tuner_json`` (reference: python/paddle/distributed/launch/main.py
auto-tuner branch, with auto_tuner/utils.py gen_new_args / read_log / find_error_from_log).

Each candidate config is exposed to the training script as environment variables
(PADDLE_AUTO_TUNER_DP/MP/PP/VPP/SHARDING/SHARDING_STAGE/MICRO_BATCH/RECOMPUTE/RECOMPUTE_GRANULARITY plus
PADDLE_AUTO_TUNER_CFG = the whole config as JSON) and as script flags through ``run_cmd`` /
``args_template`` (utils.gen_new_args); the trial runs as a normal launch, the metric is the
reference's last-10-readings mean from rank 0's log, peak memory comes from the GPU log or the
``peak_mem_gb`` the script prints, and any error lines are kept.  With ``resume`` the stored result of an
already-run config is reused; with ``run_best`` the best config is launched once more at the end.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

from .tuner import AutoTuner
from .utils import add_overlap_performance, find_error_from_log, gen_new_args, read_log, read_metric_log  # noqa: F401

_ENV = {"dp_degree": "PADDLE_AUTO_TUNER_DP", "mp_degree": "PADDLE_AUTO_TUNER_MP", "pp_degree": "PADDLE_AUTO_TUNER_PP",
        "vpp_degree": "PADDLE_AUTO_TUNER_VPP", "sharding_degree": "PADDLE_AUTO_TUNER_SHARDING",
        "sharding_stage": "PADDLE_AUTO_TUNER_SHARDING_STAGE", "micro_batch_size": "PADDLE_AUTO_TUNER_MICRO_BATCH",
        "use_recompute": "PADDLE_AUTO_TUNER_RECOMPUTE",
        "recompute_granularity": "PADDLE_AUTO_TUNER_RECOMPUTE_GRANULARITY"}


def trial_env(cfg):
    env = {}
    for k, v in _ENV.items():
        if cfg.get(k) is not None:
            env[v] = str(int(cfg[k]) if isinstance(cfg[k], bool) else cfg[k])
    env["PADDLE_AUTO_TUNER_CFG"] = json.dumps({k: v for k, v in cfg.items() if not isinstance(v, dict)},
                                              default=str)
    return env


def _launch(cfg, tuner_cfg, launch_args, script, script_args, log_dir, runner, run_best=False):
    env = dict(os.environ)
    env.update(trial_env(cfg))
    argv = [sys.executable, "-m", "paddle2_amd.distributed.launch", *launch_args, "--log_dir", log_dir, script,
            *gen_new_args(script_args, cfg, tuner_cfg, run_best=run_best)]
    if runner is not None:
        return runner(cfg, env, argv, log_dir)
    try:
        return subprocess.call(argv, env=env, timeout=tuner_cfg.get("max_time_per_task", 3600))
    except subprocess.TimeoutExpired:
        return 124


def run(tuner_cfg, launch_args, script, script_args, log_root="./auto_tuner_logs", runner=None):
    """-> (best cfg, tuner).  ``runner(cfg, env, argv, log_dir) -> returncode`` defaults to a subprocess
    launch (tests pass a fake)."""
    tuner = AutoTuner(tuner_cfg)
    metric = tuner_cfg["metric_cfg"].get("name", "step_time")
    hist_path = os.path.join(log_root, "history.csv")
    if tuner_cfg.get("resume"):
        tuner.resume_form_history(hist_path)
    while True:
        cfg = tuner.search_once()
        if cfg is None:
            break
        tid = tuner.cur_task_id - 1
        prev = tuner.get_cfg_from_resume(cfg) if tuner.resume_cfgs else None
        if prev is not None:
            rec = dict(cfg, **{k: prev.get(k) for k in (metric, "max_mem_usage", "error_info")})
            rec.update(job_id=tid, time=prev.get("time", -1), resumed=True)
        else:
            log_dir = os.path.join(log_root, f"trial_{tid}")
            t0 = time.time()
            rc = _launch(cfg, tuner_cfg, launch_args, script, script_args, log_dir, runner)
            val, mem, err = read_log(log_dir, target_metric=metric)
            oom = bool(err & 2)
            has_metric = not (err & 1)
            errors = find_error_from_log(log_dir) if (rc != 0 or not has_metric) else ""
            rec = dict(cfg, **{metric: val if has_metric else None, "job_id": tid,
                               "time": val if has_metric else -1,
                               "max_mem_usage": "OOM" if oom else (round(mem, 1) if not err & 4 else None),
                               "error_info": errors or (f"exit {rc}" if rc else None),
                               "has_error": "OOM" if oom else (None if (rc == 0 and has_metric) else "error"),
                               "wall_s": round(time.time() - t0, 1)})
        if tuner_cfg["search_algo"].get("name") == "dp_estimation":
            add_overlap_performance(rec, tuner_cfg, tuner.history_cfgs)
        tuner.add_cfg(rec)
        tuner.recorder.store_history(hist_path)
    best = tuner.get_best(tuner_cfg.get("buffer"), tuner_cfg.get("max_mem_usage"))
    if best is not None:
        os.makedirs(log_root, exist_ok=True)
        with open(os.path.join(log_root, "best_cfg.json"), "w") as f:
            json.dump(best, f, indent=1, default=str)
        if tuner_cfg.get("run_best"):
            _launch(best, tuner_cfg, launch_args, script, script_args, os.path.join(log_root, "best"), runner,
                    run_best=True)
    return best, tuner
