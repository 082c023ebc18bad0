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


class DistributedLogger(logging.Logger):
    """Rank-tagged logger (reference log_util.py:80): ``info`` emits only when FLAGS_distributed_debug_logger
    is set, after a device synchronize so the message orders with the kernels it describes."""

    def __init__(self, name, level=logging.NOTSET):
        super().__init__(name, level)

    def info(self, msg, *args, **kwargs):
        if os.environ.get("FLAGS_distributed_debug_logger", "0").lower() in ("1", "true", "yes", "on"):
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize()
            rank = os.environ.get("RANK", os.environ.get("PADDLE_TRAINER_ID", "0"))
            super().info(f"Distributed Debug [rank {rank}]: {msg}", *args, **kwargs)


def get_rotate_file_logger(log_level, name="root"):
    """Per-device rotating file logger under ./hybrid_parallel/worker_{gpu}.log (2 GB x 3 backups)."""
    from logging.handlers import RotatingFileHandler

    lg = DistributedLogger(name + "_rotate", level=log_level)
    lg.propagate = False
    dev = int(os.environ.get("FLAGS_selected_gpus", os.environ.get("LOCAL_RANK", "0")).split(",")[0])
    log_dir = os.path.join(os.getcwd(), "hybrid_parallel")
    os.makedirs(log_dir, exist_ok=True)
    h = RotatingFileHandler(os.path.join(log_dir, f"worker_{dev}.log"), maxBytes=2 << 30, backupCount=3)
    h.setFormatter(logging.Formatter("[%(asctime)-15s] [%(levelname)8s] %(filename)s:%(lineno)s - %(message)s"))
    lg.addHandler(h)
    return lg


_sync_rotate = None


def sync_rotate_logger():
    global _sync_rotate
    if _sync_rotate is None:
        _sync_rotate = get_rotate_file_logger("INFO", __name__)
    return _sync_rotate


def check_memory_usage(msg=""):
    """Log device (allocated / reserved, current and peak) and host RSS memory in GB; returns the dict."""
    import torch

    GB = float(1 << 30)
    out = {}
    if torch.cuda.is_available():
        from ....device import cuda as _dc   # native-allocator stats when it is the device allocator

        out["max_memory_allocated_size"] = _dc.max_memory_allocated() / GB
        out["max_memory_reserved_size"] = _dc.max_memory_reserved() / GB
        out["memory_allocated_size"] = _dc.memory_allocated() / GB
        out["memory_reserved_size"] = _dc.memory_reserved() / GB
    try:
        import psutil

        out["host_rss_size"] = psutil.Process().memory_info().rss / GB
    except ImportError:  # pragma: no cover
        pass
    text = f"checking memory usage {msg}:" + "".join(f"\n{k}: {v:.4f}GB" for k, v in out.items())
    logger.info(text)
    return out
