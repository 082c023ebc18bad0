"""Global flags registry (reference: paddle/common/flags.cc — 182 ``PHI_DEFINE_EXPORTED_*`` flags,
read from ``FLAGS_*`` env vars at start and mutable through ``paddle.set_flags`` / ``get_flags``).

Every reference flag name is registered with its reference default (``_flag_table.py``) plus this
framework's own.  The ones with an effect here:

  FLAGS_check_nan_inf / _level          NaN/Inf checker at Layer boundaries (framework/nan_inf.py)
  FLAGS_cudnn_deterministic             deterministic MIOpen + torch deterministic algorithms (warn-only);
                                        flash-attention bwd sums dQ slabs in order (no fp32 atomics)
  FLAGS_cudnn_exhaustive_search         MIOpen Find: convolutions benchmark their solvers per shape once and
                                        keep the fastest (torch.backends.cudnn.benchmark); off under
                                        FLAGS_cudnn_deterministic
  FLAGS_embedding_deterministic         embedding backward through a sorted, atomics-free reduction
  FLAGS_fraction_of_gpu_memory_to_use   per-process cap of the caching allocator (set at device init)
  FLAGS_gpu_memory_limit_mb             absolute cap (MiB), wins over the fraction
  FLAGS_native_allocator_headroom_mb    device MiB every native-allocator growth leaves free for the HIP
                                        runtime (kernel scratch), RCCL and the driver (default 0 = off)
  FLAGS_allocator_strategy              auto_growth -> expandable segments; naive_best_fit -> plain caching
  FLAGS_auto_growth_chunk_size_in_mb    allocator rounding granularity
  FLAGS_use_cuda_malloc_async_allocator stream-ordered async allocator backend
  (the allocator flags are applied through PYTORCH_HIP_ALLOC_CONF before the first HIP allocation)
  FLAGS_nccl_blocking_wait              every collective blocks the host until done (debug)
  FLAGS_benchmark_nccl                  collectives synchronise and record their wall time
                                        (distributed.collective.comm_benchmark_stats())
  FLAGS_enable_nccl_dynamic_check       cross-rank shape/dtype check before each collective
  FLAGS_comm_timeout_s                  process-group / watchdog timeout
  FLAGS_use_autotune                    hipBLASLt solution search + cache (incubate.autotune)
  FLAGS_check_kernel_launch             synchronise + check after each native kernel launch
  FLAGS_paddle_num_threads              intra-op CPU threads
  FLAGS_benchmark                       synchronise after every Layer call (timing runs)
  FLAGS_use_native_kernels              0 disables the HIP kernels (PyTorch reference ops)
  FLAGS_enable_async_trace / _count     comm watchdog dumps in-flight collectives on timeout
  FLAGS_host_trace_level                profiler host-event detail
Other names are accepted, stored and returned (no effect on this backend: CINN, oneDNN, PIR passes,
parameter-server / GPU-graph tables, CUDA library paths).
"""
from __future__ import annotations

import os

from ._flag_table import REFERENCE_FLAGS

_DEFAULTS = dict(REFERENCE_FLAGS)
_DEFAULTS.update({
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
    "FLAGS_gpu_memory_limit_mb": 0,
    "FLAGS_native_allocator_headroom_mb": 0,
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
    "FLAGS_check_kernel_launch": False,
    "FLAGS_dynamic_static_unified_comm": True,
})

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


def _alloc_conf():
    """Translate the allocator flags into PYTORCH_HIP_ALLOC_CONF (read by the caching allocator at its
    first use; an explicit user setting wins)."""
    if "PYTORCH_HIP_ALLOC_CONF" in os.environ or "PYTORCH_CUDA_ALLOC_CONF" in os.environ:
        return
    opts = []
    if _flags.get("FLAGS_use_cuda_malloc_async_allocator"):
        opts.append("backend:cudaMallocAsync")
    elif _flags.get("FLAGS_allocator_strategy") == "auto_growth":
        opts.append("expandable_segments:True")
    chunk = int(_flags.get("FLAGS_auto_growth_chunk_size_in_mb") or 0)
    if chunk > 0 and not _flags.get("FLAGS_use_cuda_malloc_async_allocator"):
        opts.append(f"roundup_power2_divisions:{max(1, min(16, chunk))}")
    if opts and any(k in os.environ for k in ("FLAGS_allocator_strategy", "FLAGS_use_cuda_malloc_async_allocator",
                                                "FLAGS_auto_growth_chunk_size_in_mb")):
        os.environ["PYTORCH_HIP_ALLOC_CONF"] = ",".join(opts)


_alloc_conf()
if _flags.get("FLAGS_cudnn_deterministic"):
    os.environ.setdefault("PADDLE2_AMD_FA_DQ_ATOMIC", "0")


def _apply_conv_search():
    import torch

    torch.backends.cudnn.benchmark = bool(_flags.get("FLAGS_cudnn_exhaustive_search")) and \
        not _flags.get("FLAGS_cudnn_deterministic")


if _flags.get("FLAGS_cudnn_exhaustive_search"):
    _apply_conv_search()
if _flags.get("FLAGS_check_nan_inf"):
    from . import nan_inf as _ni  # noqa: E402

    _ni._sync_from_flags()


def set_flags(flags: dict):
    for k, v in flags.items():
        key = k if k.startswith("FLAGS_") else "FLAGS_" + k
        d = _DEFAULTS.get(key)
        _flags[key] = _parse(v, d) if d is not None else v
        if key == "FLAGS_fraction_of_gpu_memory_to_use":
            _flags["_memory_limit_explicit"] = True
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

        on = bool(_flags[key])
        os.environ["PADDLE2_AMD_FA_DQ_ATOMIC"] = "0" if on else "1"  # flash bwd: ordered dQ slab sum
        torch.backends.cudnn.deterministic = on
        torch.backends.cudnn.benchmark = False if on else bool(_flags.get("FLAGS_cudnn_exhaustive_search"))
        torch.use_deterministic_algorithms(on, warn_only=True)
    if key == "FLAGS_cudnn_exhaustive_search":
        _apply_conv_search()
    if key == "FLAGS_paddle_num_threads":
        import torch

        n = int(_flags[key] or 0)
        if n > 0:
            torch.set_num_threads(n)
    if key in ("FLAGS_fraction_of_gpu_memory_to_use", "FLAGS_gpu_memory_limit_mb"):
        apply_memory_limit()
    if key == "FLAGS_use_autotune" and _flags[key]:
        try:
            from ..incubate import autotune

            autotune.enable_gemm_autotune(tuning=True)
        except Exception:  # pragma: no cover - GPU only
            pass


def apply_memory_limit(device=None):
    """FLAGS_gpu_memory_limit_mb / FLAGS_fraction_of_gpu_memory_to_use -> the caching allocator's
    per-process cap (called when a device is selected and when the flags change)."""
    import torch

    if not torch.cuda.is_available():
        return
    dev = torch.cuda.current_device() if device is None else device
    limit_mb = int(_flags.get("FLAGS_gpu_memory_limit_mb") or 0)
    if limit_mb > 0:
        total = torch.cuda.get_device_properties(dev).total_memory
        frac = min(1.0, limit_mb * (1 << 20) / total)
    else:
        frac = float(_flags.get("FLAGS_fraction_of_gpu_memory_to_use") or 1.0)
    if 0 < frac < 1.0 and ("FLAGS_fraction_of_gpu_memory_to_use" in os.environ or limit_mb > 0
                           or _flags.get("_memory_limit_explicit")):
        torch.cuda.set_per_process_memory_fraction(frac, dev)
