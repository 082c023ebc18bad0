"""Native device allocator front-end (reference: paddle/phi/core/memory/allocation/allocator_facade.cc +
auto_growth_best_fit_allocator.cc / stream_safe_cuda_allocator.cc; strategy flags in paddle/common/flags.cc).

The allocator itself is C++ (csrc/alloc/auto_growth.cpp -> paddle2_amd/_pd_alloc.so).  Two ways in:

* process-wide: ``enable()`` (or ``FLAGS_use_native_allocator=1`` in the environment, applied at import)
  swaps torch's caching allocator for it through ``CUDAPluggableAllocator`` — must happen before the first
  device allocation; every framework tensor is then carved from its chunks;
* scoped: ``mem_pool()`` returns a ``torch.cuda.MemPool`` whose segments come from it (usable any time, e.g.
  to give one subsystem its own arena).

``stats()`` / ``empty_cache()`` / ``reset_peak()`` read and manage it through ctypes; ``device.cuda``'s memory
queries consult it when it is the active allocator.
"""
from __future__ import annotations

import ctypes
import os

import torch

_LIB = None
_PLUG = None
_ACTIVE = [False]
_HOOKED = [False]
_FIELDS = ("allocated", "reserved", "peak_allocated", "peak_reserved", "num_allocs", "num_frees", "num_chunks",
           "num_grow", "num_oom_retries", "cross_stream_reuse", "record_stream", "deferred_frees", "deferred_pending")


def library_path():
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_pd_alloc.so")


def lib():
    global _LIB
    if _LIB is None:
        path = library_path()
        if not os.path.exists(path):
            raise RuntimeError(f"native allocator not built ({path}); run paddle2_amd._build.build_allocator()")
        L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)  # the torch hook resolves pd_alloc_* from it
        L.pd_alloc_configure.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.pd_alloc_set_headroom.argtypes = [ctypes.c_uint64]
        L.pd_alloc_stats.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        L.pd_alloc_reset_peak.argtypes = [ctypes.c_int]
        L.pd_alloc_empty_cache.argtypes = [ctypes.c_int]
        L.pd_alloc_empty_cache.restype = ctypes.c_uint64
        L.pd_alloc_fragmentation.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        L.pd_alloc_debug.argtypes = [ctypes.c_uint64, ctypes.c_int]
        L.pd_alloc_violations.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
        L.pd_alloc_violations.restype = ctypes.c_uint64
        _LIB = L
    return _LIB


def configure(chunk_mb=None, limit_bytes=None):
    """Chunk size (FLAGS_auto_growth_chunk_size_in_mb) and byte cap (0 = none)."""
    from ..framework import flags

    if chunk_mb is None:
        chunk_mb = int(flags.flag("FLAGS_auto_growth_chunk_size_in_mb", 0) or 0) or 256
    if limit_bytes is None:
        limit_mb = int(flags.flag("FLAGS_gpu_memory_limit_mb", 0) or 0)
        limit_bytes = limit_mb << 20
    lib().pd_alloc_configure(int(chunk_mb) << 20, int(limit_bytes))
    # device bytes every growth leaves free for the HIP runtime (kernel scratch), RCCL and the driver
    headroom_mb = int(flags.flag("FLAGS_native_allocator_headroom_mb", 0) or 0)
    lib().pd_alloc_set_headroom(int(headroom_mb) << 20)


def _pluggable():
    global _PLUG
    if _PLUG is None:
        _PLUG = torch.cuda.memory.CUDAPluggableAllocator(library_path(), "pd_alloc_malloc", "pd_alloc_free")
    return _PLUG


def enable(chunk_mb=None, limit_bytes=None):
    """Make the native allocator torch's device allocator for this process (before any device allocation)."""
    if _ACTIVE[0]:
        return
    if torch.cuda.is_initialized():
        raise RuntimeError("the native allocator must be enabled before the first device allocation "
                           "(set FLAGS_use_native_allocator=1 in the environment or call enable() first)")
    configure(chunk_mb, limit_bytes)
    hook = os.path.join(os.path.dirname(library_path()), "_pd_alloc_torch.so")
    if os.path.exists(hook):
        # C++ install with Tensor.record_stream -> pd_alloc_record_stream (cross-stream lifetime fencing)
        lib()
        H = ctypes.CDLL(hook)
        if H.pd_alloc_install_torch() != 0:
            raise RuntimeError("native allocator: torch did not create a pluggable allocator")
        _HOOKED[0] = True
    else:  # no record-stream hook: side-stream users must keep their tensors alive themselves
        torch.cuda.memory.change_current_allocator(_pluggable())
    _ACTIVE[0] = True


def has_record_stream():
    """True when Tensor.record_stream reaches the native allocator (C++ install through _pd_alloc_torch.so)."""
    return _HOOKED[0]


def is_active():
    return _ACTIVE[0]


def mem_pool():
    """A torch MemPool whose segments are allocated by the native allocator."""
    lib()
    return torch.cuda.MemPool(_pluggable().allocator())


def stats(device=0):
    buf = (ctypes.c_uint64 * len(_FIELDS))()
    lib().pd_alloc_stats(int(device), buf)
    return dict(zip(_FIELDS, list(buf)))


def fragmentation(device=0):
    buf = (ctypes.c_uint64 * 2)()
    lib().pd_alloc_fragmentation(int(device), buf)
    return {"largest_free_block": buf[0], "free_blocks": buf[1]}


def reset_peak(device=0):
    lib().pd_alloc_reset_peak(int(device))


def empty_cache(device=0):
    """Return fully-free chunks to the driver; -> bytes released."""
    return int(lib().pd_alloc_empty_cache(int(device)))


def debug(guard_bytes=4096, canary=True):
    """Out-of-bounds-write detector: pad every block by ``guard_bytes`` and verify a canary pattern in the
    slack at free time (host sync per free: a debugging mode)."""
    lib().pd_alloc_debug(int(guard_bytes), 1 if canary else 0)


def violations(max_n=64):
    """[(ptr, requested_bytes, first_bad_offset)] recorded by the canary check."""
    buf = (ctypes.c_uint64 * (3 * max_n))()
    n = int(lib().pd_alloc_violations(buf, max_n))
    return [(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]) for i in range(min(n, max_n))]


def _maybe_enable_from_env():
    """The native allocator is the process default on a GPU machine (reference: allocator_facade.cc picks
    auto_growth); ``FLAGS_use_native_allocator=0`` keeps torch's caching allocator.  Enabled at import, before
    the first device allocation; if torch already allocated on the device (paddle2_amd imported late) the
    default quietly stays torch's, while an explicit ``=1`` raises."""
    v = os.environ.get("FLAGS_use_native_allocator", "").strip().lower()
    if v in ("0", "false", "no", "off"):
        return
    explicit = v in ("1", "true", "yes", "on")
    if not explicit:
        hook = os.path.join(os.path.dirname(library_path()), "_pd_alloc_torch.so")
        if not (os.path.exists(library_path()) and os.path.exists(hook)):
            return
        try:
            if torch.cuda.device_count() == 0 or torch.cuda.is_initialized():
                return
        except Exception:  # noqa: BLE001
            return
    guard = int(os.environ.get("PD_ALLOC_GUARD_BYTES", "0") or 0)
    if guard or os.environ.get("PD_ALLOC_CANARY"):
        debug(guard or 4096, bool(os.environ.get("PD_ALLOC_CANARY")))
    try:
        enable()
    except RuntimeError:
        if explicit:
            raise
