"""Hybrid-parallel auto tuner (reference: python/paddle/distributed/auto_tuner/ — tuner.py:21
AutoTuner, search.py GridSearch / DpEstimationSearch / CustomizeSearch, prune.py rules,
recorder.py HistoryRecorder, memory_cost_model.py, utils.py search_all / gen_new_args).

Given a ``tuner_cfg`` (GPU count, model shape, candidate degrees), it enumerates
dp x mp x pp x sharding x micro-batch x recompute configurations, prunes the infeasible ones
(divisibility, MI355X HBM budget from an analytical memory model), orders the rest by an
analytical step-time estimate, and hands them out one at a time (``search_once``); the launcher
(``python -m paddle2_amd.distributed.launch --auto_tuner_json cfg.json train.py``) runs each as a
short trial, reads the metric from the trial log, records it (``add_cfg``) and reports the best.
"""
from .cost_model import estimate_memory_gb, estimate_step_time  # noqa: F401
from .recorder import HistoryRecorder  # noqa: F401
from .search import CustomizeSearch, GridSearch, search_all  # noqa: F401
from .tuner import AutoTuner  # noqa: F401
from .prune import register_prune, _PRUNE_FUNC  # noqa: F401
