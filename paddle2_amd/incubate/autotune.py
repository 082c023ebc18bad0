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


# --------------------------------------------------------------------------------------------------
# Native-vs-library routing of the Linear GEMMs (ops/torch_ops.py _pass_native): with routing autotune on,
# the first time a (pass, M, N, K, dtype) is seen both the hand-written MFMA kernel (ops/gemm.py) and hipBLASLt
# run it a few times on scratch outputs, timed with device events, and the faster one is cached (in memory
# and in tuning/gemm_routing_gfx950.json, so later processes reuse the decision without re-timing).
DEFAULT_ROUTING_CACHE = os.path.join(_ROOT, "tuning", "gemm_routing_gfx950.json")
_routing = {"enable": False, "file": None, "table": {}, "iters": 3}


def enable_routing_autotune(filename=None, iters=3):
    filename = filename or DEFAULT_ROUTING_CACHE
    _routing.update(enable=True, file=filename, iters=int(iters))
    if os.path.exists(filename):
        with open(filename) as f:
            _routing["table"].update(json.load(f))
    return filename


def disable_routing_autotune():
    _routing["enable"] = False


def routing_table():
    return dict(_routing["table"])


def _bench(fn, iters):
    import torch

    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def route(pass_name, a, b):
    """True -> native kernel for this GEMM, False -> hipBLASLt; None when routing autotune is off."""
    if not _routing["enable"] or not a.is_cuda:
        return None
    import torch

    from ..ops import gemm as G

    if pass_name == "fwd":
        M, K = a.shape
        N = b.shape[1]
        nat, lib = (lambda: G.mm_fwd(a, b)), (lambda: torch.matmul(a, b))
    elif pass_name == "dgrad":
        M, N = a.shape
        K = b.shape[0]
        nat, lib = (lambda: G.mm_dgrad(a, b)), (lambda: torch.matmul(a, b.t()))
    elif pass_name in ("wgrad", "wgrad32"):
        K, M = a.shape[1], a.shape[0]
        N = b.shape[1]
        if pass_name == "wgrad":
            nat, lib = (lambda: G.mm_wgrad_bf16(a, b)), (lambda: torch.matmul(a.t(), b))
        else:
            scratch = torch.empty(K, N, dtype=torch.float32, device=a.device)
            nat = lambda: G.mm_wgrad(a, b, scratch, 0.0)  # noqa: E731
            lib = lambda: torch.addmm(scratch, a.t(), b, beta=0.0, out_dtype=torch.float32, out=scratch)  # noqa
    else:
        return None
    key = f"{pass_name}:{M}x{N}x{K}:{str(a.dtype).replace('torch.', '')}"
    hit = _routing["table"].get(key)
    if hit is not None:
        return hit == "native"
    tn, tl = _bench(nat, _routing["iters"]), _bench(lib, _routing["iters"])
    _routing["table"][key] = "native" if tn <= tl else "blas"
    if _routing["file"]:
        os.makedirs(os.path.dirname(_routing["file"]), exist_ok=True)
        with open(_routing["file"], "w") as f:
            json.dump(_routing["table"], f, indent=1, sort_keys=True)
    return tn <= tl
