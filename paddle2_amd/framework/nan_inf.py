"""NaN/Inf checker (reference: paddle/fluid/eager/nan_inf_utils.cc:84 ``CheckTensorHasNanOrInf``,
``FLAGS_check_nan_inf`` / ``FLAGS_check_nan_inf_level`` flags.cc:79).

The reference scans every op output inside the generated ``<op>_ad_func``.  Our eager ops are
PyTorch-ROCm kernels plus fused HIP nodes, so the scan sits at the Layer boundary: when the flag is
on, every ``Layer.__call__`` output is scanned (one fused ``isfinite().all()`` reduction per tensor),
and a gradient hook scans the gradient flowing back into that output, so a NaN is attributed to
the first layer (forward) or the last layer (backward) that produced it.

Levels (reference semantics): 0 = raise on the first NaN/Inf; 1 = log and continue;
2 = also log fp32 stats (min/max/mean) of offending tensors; 3 = log stats of every checked tensor.
Off (the default) costs one module-level bool test per layer call.
"""
from __future__ import annotations

import sys

import torch

enabled = False
level = 0
_log = []   # (where, name, n_nan, n_inf) records for levels >= 1


def _sync_from_flags():
    global enabled, level
    from . import flags

    enabled = bool(flags.flag("FLAGS_check_nan_inf", False))
    level = int(flags.flag("FLAGS_check_nan_inf_level", 0))


def _tensors(out):
    from .tensor import Tensor

    if isinstance(out, Tensor):
        yield out._t
    elif isinstance(out, torch.Tensor):
        yield out
    elif isinstance(out, (list, tuple)):
        for o in out:
            yield from _tensors(o)
    elif isinstance(out, dict):
        for o in out.values():
            yield from _tensors(o)


def check_tensor(t: torch.Tensor, where: str, name: str = ""):
    if not (t.is_floating_point() or t.is_complex()) or t.numel() == 0:
        return
    ok = bool(torch.isfinite(t).all())
    if ok and level < 3:
        return
    n_nan = int(torch.isnan(t).sum()) if not ok else 0
    n_inf = int(torch.isinf(t).sum()) if not ok else 0
    msg = f"[check_nan_inf] {where} {name}: shape={list(t.shape)} dtype={t.dtype} nan={n_nan} inf={n_inf}"
    if level >= 2 or (level >= 3 and ok):
        f = t.float()
        fin = f[torch.isfinite(f)]
        if fin.numel():
            msg += f" min={float(fin.min()):.4g} max={float(fin.max()):.4g} mean={float(fin.mean()):.4g}"
    if not ok and level == 0:
        raise RuntimeError(msg + " (set FLAGS_check_nan_inf_level>=1 to log instead of raising)")
    _log.append((where, name, n_nan, n_inf))
    print(msg, file=sys.stderr)


def check_layer(layer, out):
    lname = getattr(layer, "_full_name", None) or type(layer).__name__
    for i, t in enumerate(_tensors(out)):
        check_tensor(t, f"forward {lname}", f"output[{i}]")
        if t.requires_grad:
            t.register_hook(lambda g, _n=lname, _i=i: (check_tensor(g, f"backward {_n}", f"grad(output[{_i}])"),
                                                        None)[1])


def records():
    return list(_log)
