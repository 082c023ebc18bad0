"""Kernel autotuning (reference: python/paddle/incubate/autotune.py ``set_config`` — kernel
algorithm search for cuBLASLt/cuDNN; phi/kernels/autotune/ cache keyed by shape).

On MI355X the plain library GEMMs go through hipBLASLt.  Autotuning benchmarks every hipBLASLt /
rocBLAS solution for each (transpose, M, N, K, dtype) actually executed and caches the winner in
a CSV (torch's TunableOp engine drives the search; the cache is ours and lives in-tree under
``tuning/`` so the selection travels with the code and is reused without re-tuning).
"""
from __future__ import annotations

import json
import os

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_GEMM_CACHE = os.path.join(_ROOT, "tuning", "gemm_gfx950.csv")

_state = {"kernel": False, "tuning": False, "file": None}


def enable_gemm_autotune(tuning=False, filename=None, max_tuning_ms=10, max_iters=20):
    """Use (and with ``tuning=True`` extend) the GEMM selection cache."""
    import torch.cuda.tunable as tun

    filename = filename or DEFAULT_GEMM_CACHE
    os.makedirs(os.path.dirname(filename), exist_ok=True)
    tun.enable(True)
    tun.set_filename(filename, insert_device_ordinal=False)
    tun.tuning_enable(bool(tuning))
    if tuning:
        tun.set_max_tuning_duration(int(max_tuning_ms))
        tun.set_max_tuning_iterations(int(max_iters))
    if os.path.exists(filename):
        tun.read_file(filename)
    _state.update(kernel=True, tuning=bool(tuning), file=filename)
    return filename


def disable_gemm_autotune():
    import torch.cuda.tunable as tun

    tun.enable(False)
    _state.update(kernel=False, tuning=False)


def set_config(config=None):
    """paddle.incubate.autotune.set_config({"kernel": {"enable": True, "tuning_range": [a, b]}, ...})."""
    if config is None:
        config = {"kernel": {"enable": True}}
    if isinstance(config, str):
        with open(config) as f:
            config = json.load(f)
    k = config.get("kernel", {})
    if k.get("enable", False):
        enable_gemm_autotune(tuning=True, filename=k.get("cache_file"))
    elif "kernel" in config:
        disable_gemm_autotune()
    return dict(_state)


def status():
    """Newly tuned entries are written to the cache file when the process exits."""
    return dict(_state)
