"""Global flags registry (reference: paddle/common/flags.cc — 184 ``PHI_DEFINE_EXPORTED_*`` flags,
read from ``FLAGS_*`` env vars at start and mutable through ``paddle.set_flags`` / ``get_flags``).

Only flags with an effect in this framework are registered with real semantics; unknown
``FLAGS_*`` names are accepted and stored (the reference errors on unknown names, we log).
"""
from __future__ import annotations

import os

_DEFAULTS = {
    "FLAGS_check_nan_inf": False,
    "FLAGS_check_nan_inf_level": 0,
    "FLAGS_enable_async_trace": False,
    "FLAGS_async_trace_count": 5,
    "FLAGS_nccl_blocking_wait": False,
    "FLAGS_benchmark_nccl": False,
    "FLAGS_enable_nccl_dynamic_check": False,
    "FLAGS_eager_communication_connection": False,
    "FLAGS_allocator_strategy": "auto_growth",
    "FLAGS_fraction_of_gpu_memory_to_use": 0.92,
    "FLAGS_use_autotune": False,
    "FLAGS_cudnn_deterministic": False,
    "FLAGS_embedding_deterministic": 0,
    "FLAGS_call_stack_level": 1,
    "FLAGS_enable_pir_api": True,
    "FLAGS_use_cuda_malloc_async_allocator": False,
    "FLAGS_shard_split_param": False,
    "FLAGS_pp_check_naninf": False,
    "FLAGS_comm_timeout_s": 1800,
    "FLAGS_use_native_kernels": True,
    "FLAGS_flash_attn_version": 2,
    "FLAGS_benchmark": False,
    "FLAGS_dynamic_static_unified_comm": True,
}

_flags = {}


def _parse(v, default):
    if isinstance(default, bool):
        return str(v).lower() in ("1", "true", "yes", "on")
    if isinstance(default, int):
        return int(v)
    if isinstance(default, float):
        return float(v)
    return v


def _init():
    for k, d in _DEFAULTS.items():
        _flags[k] = _parse(os.environ[k], d) if k in os.environ else d
    for k, v in os.environ.items():
        if k.startswith("FLAGS_") and k not in _flags:
            _flags[k] = v


_init()
if _flags.get("FLAGS_check_nan_inf"):
    from . import nan_inf as _ni  # noqa: E402

    _ni._sync_from_flags()


def set_flags(flags: dict):
    for k, v in flags.items():
        key = k if k.startswith("FLAGS_") else "FLAGS_" + k
        d = _DEFAULTS.get(key)
        _flags[key] = _parse(v, d) if d is not None else v
        _on_change(key)


def get_flags(flags):
    if isinstance(flags, str):
        flags = [flags]
    out = {}
    for k in flags:
        key = k if k.startswith("FLAGS_") else "FLAGS_" + k
        if key not in _flags:
            raise ValueError(f"flag {key} is not registered")
        out[key] = _flags[key]
    return out


def flag(name, default=None):
    return _flags.get(name, default)


def _on_change(key):
    if key in ("FLAGS_check_nan_inf", "FLAGS_check_nan_inf_level"):
        from . import nan_inf

        nan_inf._sync_from_flags()
    if key == "FLAGS_cudnn_deterministic":
        import torch

        torch.backends.cudnn.deterministic = bool(_flags[key])
