"""Hybrid-parallel auto tuner (reference: python/paddle/distributed/auto_tuner/ — tuner.py:21
AutoTuner, search.py GridSearch / DpEstimationSearch / GBSSearch / CustomizeSearch, prune.py rules,
recorder.py HistoryRecorder, cost_model.py / memory_cost_model.py, utils.py search_all / gen_new_args /
log readers).

Given a ``tuner_cfg`` (GPU count, model shape, candidate degrees), it enumerates
dp x mp x pp x vpp x sharding(degree, stage) x micro-batch x recompute(granularity, refined per-op counts)
x custom dimensions, prunes the infeasible ones (divisibility, xGMI-local TP, MI355X HBM budget from an
analytical memory model or a user tool, invalid-strategy patterns), orders the rest (memory- or
performance-first, ``schedule_prior`` patterns, analytical step time) and hands them out one at a time
(``search_once``), re-pruning each against measured history.  The launcher
(``python -m paddle2_amd.distributed.launch --auto_tuner_json cfg.json train.py``) runs each as a short
trial, reads metric / peak memory / errors from the trial logs, records it (``add_cfg``), can resume
from an earlier history and reports (and optionally re-runs) the best.
"""
from .cost_model import estimate_memory_gb, estimate_step_time, get_mem, get_not_oom_cfgs  # noqa: F401
from .prune import _PRUNE_FUNC, _PRUNE_HISTORY_FUNC, register_prune, register_prune_history  # noqa: F401
from .recorder import HistoryRecorder  # noqa: F401
from .search import CustomizeSearch, DpEstimationSearch, GBSSearch, GridSearch  # noqa: F401
from .tuner import AutoTuner  # noqa: F401
from .utils import default_candidates, divisor, search_all  # noqa: F401
