"""Fleet logger (reference: fleet/utils/log_util.py)."""
from __future__ import annotations

import logging
import os

logger = logging.getLogger("paddle2_amd.fleet")
if not logger.handlers:
    _h = logging.StreamHandler()
    _h.setFormatter(logging.Formatter("[%(asctime)s] [%(levelname)8s] %(filename)s:%(lineno)d - %(message)s"))
    logger.addHandler(_h)
logger.setLevel(os.environ.get("PADDLE2_AMD_LOG_LEVEL", "INFO"))


def set_log_level(level):
    logger.setLevel(level if isinstance(level, int) else str(level).upper())


def get_log_level_code():
    return logger.getEffectiveLevel()


def get_log_level_name():
    return logging.getLevelName(logger.getEffectiveLevel())


def layer_to_str(base, *args, **kwargs):
    name = base + "("
    if args:
        name += ", ".join(str(a) for a in args)
        if kwargs:
            name += ", "
    if kwargs:
        name += ", ".join(f"{k}={v}" for k, v in kwargs.items())
    return name + ")"
